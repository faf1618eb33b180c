#!/bin/bash
# Round 3, session 2, end-of-session evidence on the final tree: the whole GPU
# suite, the smoke, the default bench line, and the kernel trace + PMC passes
# of the headline (interleaved) layout (tools/profile.sh).
set -o pipefail
O=gpurun_out/r03af; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=10 > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['roofline']['frac'], d['kernels']['encrypt']['ms'], d['kernels']['decrypt']['ms'])"
bash tools/profile.sh r03af_ilv --layout interleaved || { echo profile failed; exit 1; }
tail -30 gpurun_out/prof_r03af_ilv/pmc_summary.txt
echo all ok
