#!/bin/bash
# Compiler scheduling strategies (max-ilp, max-memory-clause) and AES-wave
# priority in the split encrypt (s_setprio 1 / 3) vs the product build (base6).
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
L="build_exp/base6/librnstok.so build_exp/silp/librnstok.so build_exp/smem/librnstok.so build_exp/aprio1/librnstok.so build_exp/aprio3/librnstok.so"
for args in "" "--ilv" "--length 1500" "--keys 65536" "--packed 64 --length 1500"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L --rounds 16 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt | grep -v round-trip
grep "round-trip" $O/ab.txt | grep -c "ok=True tokens==variant0: True"
