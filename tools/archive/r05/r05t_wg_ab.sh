#!/bin/bash
# Single-key multi-pass decrypt at 512 / 640 threads (2 / 2.5 waves per SIMD)
# vs the product's 768.
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
L="build_exp/base9/librnstok.so build_exp/d512/librnstok.so build_exp/d640/librnstok.so"
for args in "--rounds 30" "--ilv" "--length 1500" "--length 400"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L --rounds 20 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt | grep -v round-trip
grep "round-trip" $O/ab.txt | grep -c "ok=True tokens==variant0: True"
