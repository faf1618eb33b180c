#!/bin/bash
# A/B of the per-key long-token encrypt for short packets: 1 KiB floor vs none.
set -o pipefail
mkdir -p gpurun_out build_exp/lpk
make -s -C reticulum_amd/csrc OUT=$PWD/build_exp/lpk/librnstok.so \
  FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -Wno-unused-value -DRNSTOK_LONG_PERKEY_MIN_LEN=0u" || exit 1
for L in 500 100 1000; do
  for N in 1 1024 32768; do
    echo "== L=$L N=$N keys=64"
    timeout -k 10 120 python3 tools/exp_bench.py reticulum_amd/librnstok.so build_exp/lpk/librnstok.so --packets $N --length $L --keys 64 --rounds 21 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
