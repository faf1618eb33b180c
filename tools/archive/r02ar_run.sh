#!/bin/bash
# Round-2 (session 4, after the container restore) end-of-round evidence: GPU tests, smoke, the headline
# bench line, then kernel trace + PMC passes of bench.py (tools/profile.sh).
set -o pipefail
O=gpurun_out/r02ar; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
cut -c1-300 $O/bench.json
bash tools/profile.sh r02ar || { echo profile failed; exit 1; }
echo all ok
