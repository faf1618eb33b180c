#!/bin/bash
# Round-2 full check: GPU tests, smoke, headline bench, sharded configs at N=1.
set -o pipefail
O=gpurun_out/r02l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 --no-e2e --cpu-seconds 0 > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
echo all ok
