#!/bin/bash
# Deframe flag positions: build_exp/prev (count pass + scatter pass, two reads
# of the stream) vs build_exp/cur (one pass writing chunk-local positions,
# then a small gather after the scan; the product), alternating processes, a
# kernel trace of one run of each, then the whole GPU suite on the product.
set -o pipefail
O=gpurun_out/r03aa; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in prev cur; do
    RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 python -u tools/bench_configs.py --config wire --steps 20 >> $O/wire_$v.jsonl 2>> $O/wire_$v.err || { echo "$v failed"; tail -5 $O/wire_$v.err; exit 1; }
  done
done
for v in prev cur; do
  RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- python3 tools/bench_configs.py --config wire --steps 20 > $O/trace_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
done
for v in prev cur; do echo == $v; python3 -c "
import json,sys
for l in open('$O/wire_$v.jsonl'):
    d=json.loads(l); print(d['ok'], {k: round(s.get('ms', 0),4) for k, s in d['stages'].items()})
"; done
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
