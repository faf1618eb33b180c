#!/bin/bash
# One-pass single-key decrypt (the 1024-thread k_decrypt instance): paired quad
# loads (HEAD build, 38 VGPRs spilled) against single quads (11 spilled).
set -o pipefail
O=gpurun_out/r04aa
mkdir -p $O
for args in "--packets 262144" "--packets 262144 --length 4096" "--packets 262144 --length 16384" "--packets 131072 --length 1500"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py build_exp/pair1024/librnstok.so build_exp/base/librnstok.so --rounds 16 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt
