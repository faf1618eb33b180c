#!/bin/bash
# full GPU suite + smoke + default bench line: tools/r06_suite.sh <tag>
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
