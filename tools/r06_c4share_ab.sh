#!/bin/bash
# bench.shard_rate (c4's 8-GPU rank share: 32 768 x 16 KiB, the long-token kernels full) per library variant
set -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $R); do
  for v in "$@"; do
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -k 10 200 python -c "
import json, torch, bench
from reticulum_amd import _native
print(json.dumps(bench.shard_rate(torch.device('cuda', 0), _native.load().rt_num_cus(_native.context(0)))))" > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    python3 - $O/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%-7s enc %.3f ms %.3f GHz %.3f Mcyc | dec %.3f ms %.3f GHz %.3f Mcyc ok %s" % (sys.argv[2], d["encrypt"]["ms"], d["encrypt"].get("clock_ghz") or 0,
      (d["encrypt"].get("cycles_per_launch") or 0) / 1e6, d["decrypt"]["ms"], d["decrypt"].get("clock_ghz") or 0, (d["decrypt"].get("cycles_per_launch") or 0) / 1e6, d.get("ok")))
PY
  done
done | tee $O/summary.txt
