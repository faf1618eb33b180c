#!/bin/bash
# Partial windows of the framing and flag kernels: build_exp/wirebytetail (up
# to 15 byte loads in turn, RNSTOK_WIRE_BYTE_TAIL) vs build_exp/cur (the one
# or two aligned 16-B blocks holding the bytes, shifted into place; the
# product), then the whole GPU suite.
set -o pipefail
O=gpurun_out/r03w; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in wirebytetail cur; do
    RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 python -u tools/bench_configs.py --config wire --steps 20 >> $O/wire_$v.jsonl 2>> $O/wire_$v.err || { echo "$v failed"; tail -5 $O/wire_$v.err; exit 1; }
  done
done
for v in wirebytetail cur; do
  RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 tools/bench_configs.py --config wire --steps 20 > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  find $O/trace_$v -name "*kernel_stats.csv" | head -1 | xargs grep -h "unescape\|hdlc\|flag" | cut -d, -f1-4
done
for v in wirebytetail cur; do echo == $v; python3 -c "
import json,sys
for l in open('$O/wire_$v.jsonl'):
    d=json.loads(l); print(d['ok'], {k: round(s.get('ms', s.get('median_ms', 0)),4) if isinstance(s, dict) else s for k, s in d['stages'].items()})
"; done
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/wire_tests.log 2>&1 || { echo wire tests failed; tail -20 $O/wire_tests.log; exit 1; }
tail -1 $O/wire_tests.log
