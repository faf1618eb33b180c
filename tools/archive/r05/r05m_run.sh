#!/bin/bash
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
l=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(l['value'], l['roofline']['frac'], l['roofline']['clock_ghz'])
print(json.dumps(l['per_call_threads']))"
