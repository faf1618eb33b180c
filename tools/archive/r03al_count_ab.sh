#!/bin/bash
# HDLC framing count pass: build_exp/pairs (two packet groups per step, the
# first two windows of both loaded before counting, RNSTOK_COUNT_PAIRS) vs
# build_exp/base (one group per step; the product), then the wire tests on pairs.
set -o pipefail
O=gpurun_out/r03al; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in pairs base; do
    RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 python -u tools/bench_configs.py --config wire --steps 20 >> $O/wire_$v.jsonl 2>> $O/wire_$v.err || { echo "$v failed"; tail -5 $O/wire_$v.err; exit 1; }
  done
done
for v in pairs base; do
  RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 tools/bench_configs.py --config wire --steps 20 > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  f=$(find $O/trace_$v -name "*kernel_stats.csv"); grep -h "hdlc\|flag\|unescape" $f | cut -d, -f1-4
done
RNSTOK_LIB=build_exp/pairs/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_wire.py tests/test_pipeline_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pairs_tests.log 2>&1 || { echo pairs tests failed; tail -20 $O/pairs_tests.log; exit 1; }
tail -1 $O/pairs_tests.log
