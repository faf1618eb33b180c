#!/bin/bash
# Decrypt plaintext stores grouped by 64-B sector (RNSTOK_DEC_ST_SECTOR*): c5's
# rank share (packed outputs) per variant, each a sustained run
set -o pipefail
O=gpurun_out/r06u
mkdir -p $O
for r in 1 2; do
  for v in "$@"; do
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -k 10 200 python tools/c5_share.py > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err || { tail -5 $O/c5_${v}_$r.err; exit 1; }
    python3 - $O/c5_${v}_$r.json $v <<'PY'
import json, sys
c = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%-8s enc %.4f ms %.3f GHz | dec %.4f ms %.3f GHz %.3f Mcyc ok %s" % (sys.argv[2],
    c["encrypt"]["ms"], c["encrypt"]["kernel_clock_ghz"],
    c["decrypt"]["ms"], c["decrypt"]["kernel_clock_ghz"], c["decrypt"]["kernel_cycles_per_launch"] / 1e6, c["ok"]))
PY
  done
done | tee $O/summary.txt
