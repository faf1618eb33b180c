#!/bin/bash
# tools/sync_floor_probe.py under the runtime's wait policies (device flags, and
# ROCr's interrupt-free signal waits), two rounds
set -o pipefail
O=gpurun_out/r06av; mkdir -p $O
for r in 1 2; do
  for f in 0 1 2 4; do
    timeout -k 10 120 python tools/sync_floor_probe.py --flags $f --calls 2000 --length 383 > $O/f${f}_$r.json 2> $O/f${f}_$r.err || { tail -5 $O/f${f}_$r.err; exit 1; }
    echo "flags $f $(cat $O/f${f}_$r.json)"
  done
  HSA_ENABLE_INTERRUPT=0 timeout -k 10 120 python tools/sync_floor_probe.py --flags 0 --calls 2000 --length 383 > $O/noint_$r.json 2> $O/noint_$r.err || { tail -5 $O/noint_$r.err; exit 1; }
  echo "HSA_ENABLE_INTERRUPT=0 $(cat $O/noint_$r.json)"
done | tee $O/summary.txt
