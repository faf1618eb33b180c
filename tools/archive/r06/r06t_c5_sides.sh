#!/bin/bash
# c5 rank share: which buffer's 128-B slot placement moves the clock (each a sustained run)
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
for r in 1 2; do
  for sides in none dec_in dec_out enc_in enc_out all; do
    if [ $sides = all ]; then A="--align"; elif [ $sides = none ]; then A=""; else A="--align-sides $sides"; fi
    timeout -k 10 200 python tools/c5_share.py $A > $O/${sides}_$r.json 2> $O/${sides}_$r.err || { tail -5 $O/${sides}_$r.err; exit 1; }
    python3 - $O/${sides}_$r.json $sides <<'PY'
import json, sys
c = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%-8s enc %.4f ms %.3f GHz %.3f Mcyc | dec %.4f ms %.3f GHz %.3f Mcyc ok %s" % (sys.argv[2],
    c["encrypt"]["ms"], c["encrypt"]["kernel_clock_ghz"], c["encrypt"]["kernel_cycles_per_launch"] / 1e6,
    c["decrypt"]["ms"], c["decrypt"]["kernel_clock_ghz"], c["decrypt"]["kernel_cycles_per_launch"] / 1e6, c["ok"]))
PY
  done
done | tee $O/summary.txt
