#!/bin/bash
# GPU tests, then per-call latency of the drop-in Token for the current build
# and the A/B builds under tools/_ab (if present).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_tests.txt
: > gpurun_out/single.jsonl
for lib in reticulum_amd/librnstok.so tools/_ab/*.so; do
  [ -f "$lib" ] || continue
  echo "== $lib"
  RNSTOK_LIB=$PWD/$lib timeout -k 10 180 python -u tools/single_call_latency.py --calls 3000 > gpurun_out/single_one.json || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/single_one.json')); d['lib']=sys.argv[1]; print(json.dumps(d))" "$lib" | tee -a gpurun_out/single.jsonl
done
# kernel A/B against the first tools/_ab build, device-resident
ab=$(ls tools/_ab/*.so 2>/dev/null | head -1)
if [ -n "$ab" ]; then
  for args in "--packets 1048576" "--packets 65536" "--packets 1048576 --keys 64" "--packets 2048 --length 16384"; do
    echo "== exp_bench $args"
    timeout -k 10 240 python -u tools/exp_bench.py reticulum_amd/librnstok.so "$ab" $args --rounds 11 || exit 1
  done
fi
