#!/bin/bash
# Chunk counters everywhere (decrypt batches of whole passes, split encrypt)
# vs the product, more shapes and a long c2 A/B.
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
L="build_exp/base7/librnstok.so build_exp/dynall/librnstok.so"
for args in "--rounds 40" "--rounds 40" "--length 1000" "--length 100" "--length 4096 --packets 262144" "--length 1500 --packets 524288" "--packets 1500000" "--packets 600000" "--keys 65536 --packets 983040"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L --rounds 20 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt | grep -v round-trip
grep "round-trip" $O/ab.txt | grep -c "ok=True tokens==variant0: True"
