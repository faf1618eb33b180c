#!/bin/bash
# The default bench line with node_pipeline and c4_rank_share_8gpu (the composed interface
# path and the c4 8-GPU rank share at N = 1): the bench GPU tests, then the default line.
set -o pipefail
O=gpurun_out/r03aj; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bench_gpu.py tests/test_pipeline_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['roofline']['frac'], json.dumps(d['node_pipeline'])[:300], json.dumps(d['c4_rank_share_8gpu']))"
