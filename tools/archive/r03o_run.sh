#!/bin/bash
# Round 3: D2H as GPU stores into pinned host memory (copy_kernels.hip):
# GPU suite incl. tests/test_copy_gpu.py, the host-origin rows of the default
# bench line (stores vs copy engine, same run), and the drop-in's single-call
# latency A/B against the previous build (all copies on the copy engine).
set -o pipefail
O=gpurun_out/r03o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=10 > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
  RNSTOK_LIB=build_exp/prev/librnstok.so timeout -k 10 120 python -u tools/single_call_latency.py --calls 2000 > $O/lat_prev_$r.json 2>&1 || { echo lat prev failed; tail $O/lat_prev_$r.json; exit 1; }
  timeout -k 10 120 python -u tools/single_call_latency.py --calls 2000 > $O/lat_new_$r.json 2>&1 || { echo lat new failed; tail $O/lat_new_$r.json; exit 1; }
done
tail -1 $O/lat_prev_2.json; tail -1 $O/lat_new_2.json
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value']);print(json.dumps(d['e2e_pcie']))"
echo all ok
