#!/bin/bash
# Round 3 evidence.  PART=tests: full GPU tests, smoke, the headline bench line
# (rows) and the interleaved-layout line.  PART=prof: kernel trace + PMC of
# both layouts (tools/profile.sh).
set -o pipefail
O=gpurun_out/r03i; mkdir -p $O
export TMPDIR=/tmp
if [ "${PART:-tests}" = tests ]; then
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 300 python -u bench.py --layout interleaved --cpu-seconds 0 > $O/bench_ilv.json 2> $O/bench_ilv.err || { echo bench ilv failed; tail $O/bench_ilv.err; exit 1; }
cut -c1-300 $O/bench_ilv.json
else
bash tools/profile.sh r03i --layout rows || { echo profile failed; exit 1; }
bash tools/profile.sh r03i_ilv --layout interleaved || { echo profile ilv failed; exit 1; }
fi
echo all ok
