#!/bin/bash
# Chunk counters, third box: the product (base7), decrypt and k_encrypt through
# the counter for batches of whole passes too (qall), and qall plus the split
# encrypt's batches from a counter (dynall).
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
L="build_exp/base7/librnstok.so build_exp/qall/librnstok.so build_exp/dynall/librnstok.so"
for args in "--packets 786432" "--packets 983040" "--packets 1179648" "--length 1000" "--length 1500" "--length 100" "--packets 1500000" ""; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L --rounds 30 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt | grep -v round-trip
grep "round-trip" $O/ab.txt | grep -c "ok=True tokens==variant0: True"
