#!/bin/bash
# A/B of k_encrypt_long for small variable-length (packed) batches vs the general kernel.
set -o pipefail
mkdir -p gpurun_out build_exp/lp
make -s -C reticulum_amd/csrc OUT=$PWD/build_exp/lp/librnstok.so \
  FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -Wno-unused-value -DRNSTOK_LONG_PACKED" || exit 1
for K in 1 64; do
  for LO in 0 400; do
    for N in 1 256 8192 32768; do
      echo "== lengths $LO..600 N=$N keys=$K"
      timeout -k 10 120 python3 tools/exp_bench.py reticulum_amd/librnstok.so build_exp/lp/librnstok.so --packets $N --length 600 --packed $LO --keys $K --rounds 21 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
