#!/bin/bash
# A/B of the long-token kernels for short packets: default threshold (1 KiB) vs 0.
# The variant library is built here on the box (keeps the pushed tree small).
set -o pipefail
mkdir -p gpurun_out build_exp/lat
make -s -C reticulum_amd/csrc OUT=$PWD/build_exp/lat/librnstok.so \
  FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -Wno-unused-value -DRNSTOK_LONG_MIN_LEN=0u" || exit 1
for L in 500 100 0 1000; do
  for N in 1 64 1024 8192 32768; do
    echo "== L=$L N=$N"
    timeout -k 10 120 python3 tools/exp_bench.py reticulum_amd/librnstok.so build_exp/lat/librnstok.so --packets $N --length $L --rounds 21 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
