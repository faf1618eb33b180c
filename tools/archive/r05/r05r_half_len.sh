#!/bin/bash
# The half-quad 1024-thread decrypt (h1024) against the product by length.
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
L="build_exp/base8/librnstok.so build_exp/h1024/librnstok.so build_exp/h768/librnstok.so build_exp/p1024/librnstok.so"
for len in 16 64 100 160 250 350 430; do
  echo "== --length $len" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L --rounds 20 --length $len >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
echo "== --length 100 --packets 1500000" >> $O/ab.txt
timeout -k 10 240 python tools/exp_bench.py $L --rounds 20 --length 100 --packets 1500000 >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
echo "== --packed 16 --length 200" >> $O/ab.txt
timeout -k 10 240 python tools/exp_bench.py $L --rounds 20 --packed 16 --length 200 >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt | grep -v round-trip
grep "round-trip" $O/ab.txt | grep -c "ok=True tokens==variant0: True"
