#!/bin/bash
# Per-call latency (tools/single_call_latency.py, 383-B packets) and
# bench.per_call_rate per library variant, R rounds, variants in turn.
#   tools/r06_h2d_ab.sh <tag> <R> <variant>...   (libraries in exp_ship/<variant>/)
set -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $R); do
  for v in "$@"; do
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -k 10 200 python tools/single_call_latency.py --calls 3000 --length 383 \
      > $O/${v}_lat_$r.json 2> $O/${v}_lat_$r.err || { tail -5 $O/${v}_lat_$r.err; exit 1; }
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -k 10 200 python -c "
import json, bench
print(json.dumps(bench.per_call_rate(calls=400)))" > $O/${v}_rate_$r.json 2> $O/${v}_rate_$r.err || { tail -5 $O/${v}_rate_$r.err; exit 1; }
    python3 - $O/${v}_lat_$r.json $O/${v}_rate_$r.json $v <<'PY'
import json, sys
lat = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("%-6s token enc %5.1f dec %5.1f us | abi enc %5.1f dec %5.1f | device enc %5.1f dec %5.1f | sync %4.1f | "
      "16 threads %.0f calls/s one thread %.0f ok %s %s" % (
      sys.argv[3], lat["token_encrypt_us"], lat["token_decrypt_us"], lat["host_abi_encrypt_us"],
      lat["host_abi_decrypt_us"], lat["device_encrypt_us"], lat["device_decrypt_us"], lat["sync_only_us"],
      d["threads"]["calls_s"], d["one_thread"]["calls_s"], d["threads"]["ok"], d["one_thread"]["ok"]))
PY
  done
done | tee $O/summary.txt
