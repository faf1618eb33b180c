#!/bin/bash
# A/B of the HDLC unescape kernel: neighbour-byte tests on shifted data words (unesc_old,
# RNSTOK_UNESC_SHIFTED_WORDS) vs on shifted flag words (unesc_new, the product);
# alternating builds in separate processes (RNSTOK_LIB), kernel trace of one
# run of each.
set -o pipefail
O=gpurun_out/r03j; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in unesc_old unesc_new; do
    RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 python -u tools/bench_configs.py --config wire --steps 20 >> $O/wire_$v.jsonl 2>> $O/wire_$v.err || { echo "$v failed"; tail -5 $O/wire_$v.err; exit 1; }
  done
done
for v in unesc_old unesc_new; do
  RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 tools/bench_configs.py --config wire --steps 20 > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  grep -h "unescape\|hdlc\|flag" $O/trace_$v/run_kernel_stats.csv | cut -d, -f1-4
done
for v in unesc_old unesc_new; do echo == $v; python3 -c "
import json,sys
for l in open('$O/wire_$v.jsonl'):
    d=json.loads(l); print(d['ok'], {k: round(s.get('ms', s.get('median_ms', 0)),4) if isinstance(s, dict) else s for k, s in d['stages'].items()})
"; done
RNSTOK_LIB=build_exp/unesc_new/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_wire.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/wire_tests_new.log 2>&1 || { echo wire tests failed; tail -20 $O/wire_tests_new.log; exit 1; }
tail -1 $O/wire_tests_new.log
