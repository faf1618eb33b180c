#!/bin/bash
# Inbound pipeline glue on the device (rt_frames_compact, rt_token_spans)
# instead of torch ops: their tests, the pipeline tests, the node config and
# its kernel trace.
set -o pipefail
O=gpurun_out/r03ao; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_compact_gpu.py tests/test_pipeline_gpu.py tests/test_wire.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/bench_configs.py --config node >> $O/node.jsonl 2>> $O/node.err || { echo node failed; tail -5 $O/node.err; exit 1; }
done
cat $O/node.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/bench_configs.py --config node > $O/trace.log 2>&1 || { echo trace failed; exit 1; }
echo ok
timeout -k 10 300 python -u tools/archive/r03ao_inbound_ab.py > $O/inbound_ab.json 2> $O/inbound_ab.err || { echo ab failed; tail -5 $O/inbound_ab.err; exit 1; }
cat $O/inbound_ab.json
