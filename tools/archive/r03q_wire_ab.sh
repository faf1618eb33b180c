#!/bin/bash
# A/B of the wire kernels' partial-window loads: build_exp/prev (a branch and
# a wait per byte for the last lane of every packet or frame) vs build_exp/cur
# (clamped byte loads all in flight; unescape: one 16-B load masked inside
# the stream), alternating processes, then a kernel trace of one run of each
# and the wire GPU tests on the new build.
set -o pipefail
O=gpurun_out/r03q; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in prev cur; do
    RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 python -u tools/bench_configs.py --config wire --steps 20 >> $O/wire_$v.jsonl 2>> $O/wire_$v.err || { echo "$v failed"; tail -5 $O/wire_$v.err; exit 1; }
  done
done
for v in prev cur; do
  RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 tools/bench_configs.py --config wire --steps 20 > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  find $O/trace_$v -name "*kernel_stats.csv" | head -1 | xargs grep -h "unescape\|hdlc\|flag" | cut -d, -f1-4
done
for v in prev cur; do echo == $v; python3 -c "
import json,sys
for l in open('$O/wire_$v.jsonl'):
    d=json.loads(l); print(d['ok'], {k: round(s.get('ms', s.get('median_ms', 0)),4) if isinstance(s, dict) else s for k, s in d['stages'].items()})
"; done
timeout -k 10 300 python -u -m pytest tests/test_wire.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/wire_tests.log 2>&1 || { echo wire tests failed; tail -20 $O/wire_tests.log; exit 1; }
tail -1 $O/wire_tests.log
