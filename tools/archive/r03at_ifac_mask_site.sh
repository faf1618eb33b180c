#!/bin/bash
# The product with the one-site PRK prologue in the mask template only:
# wire + pipeline + C-host + compact tests, then the wire config and its kernel trace.
set -o pipefail
O=gpurun_out/r03at; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wire.py tests/test_pipeline_gpu.py tests/test_c_host_gpu.py tests/test_compact_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/bench_configs.py --config wire --steps 20 >> $O/wire.jsonl 2>> $O/wire.err || { echo wire failed; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_configs.py --config wire --steps 20 > $O/trace.log 2>&1 || { echo trace failed; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$O/trace/run_kernel_stats.csv')):
    if 'ifac' in r['Name']: print(r['Name'].split('k_ifac')[1][:8], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
