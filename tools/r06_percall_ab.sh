#!/bin/bash
# bench.per_call_rate (one Token call per packet from 16 threads and from one) per library variant
set -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $R); do
  for v in "$@"; do
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -k 10 200 python -c "
import json, bench
d = bench.per_call_rate(calls=400)
print(json.dumps(d))" > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    python3 - $O/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%-6s 16 threads %.0f calls/s  one thread %.0f calls/s  ok %s %s" % (sys.argv[2], d["threads"]["calls_s"],
      d["one_thread"]["calls_s"], d["threads"]["ok"], d["one_thread"]["ok"]))
PY
  done
done | tee $O/summary.txt
