#!/bin/bash
# pipeline tests (incl. the side-stream case) after the plumbing cleanup
set -o pipefail
O=gpurun_out/r03ai; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_bench_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
