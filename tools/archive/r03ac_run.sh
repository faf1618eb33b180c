#!/bin/bash
# Header pack from registers, then: the interface path composed on the device (reticulum_amd.pipeline): the full GPU
# tests against the oracle's composition, then the node config (2^20 DATA
# packets out through IFAC + framing, and the stream back in), with a kernel
# trace of one run.
set -o pipefail
O=gpurun_out/r03ac; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pipeline_tests.log 2>&1 || { echo tests failed; tail -30 $O/pipeline_tests.log; exit 1; }
tail -1 $O/pipeline_tests.log
timeout -k 10 300 python -u tools/bench_configs.py --config node --steps 10 > $O/node.json 2> $O/node.err || { echo node failed; tail $O/node.err; exit 1; }
cat $O/node.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_configs.py --config node --steps 10 > $O/trace.log 2>&1 || { echo trace failed; exit 1; }
python3 -c "
import csv
rows=sorted(csv.DictReader(open('$O/trace/run_kernel_stats.csv')), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:24]: print(r['Name'].split('(')[0][-44:], r['Calls'], round(float(r['AverageNs'])/1000,1), 'us')
"
