#!/bin/bash
# Build an experimental librnstok variant: tools/build_variant.sh <name> <extra hipcc flags...>
# Output: $EXP_DIR/<name>/librnstok.so, EXP_DIR default build_exp (gpurun-ignored: use
# EXP_DIR=exp_ship for a variant that must travel to the GPU box)  (load with tools/exp_bench.py)
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${EXP_DIR:-build_exp}
mkdir -p $ROOT/$OUT/$NAME
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -w "$@" -shared -o $ROOT/$OUT/$NAME/librnstok.so \
  $ROOT/reticulum_amd/csrc/token_kernels.hip $ROOT/reticulum_amd/csrc/hkdf_kernels.hip $ROOT/reticulum_amd/csrc/resource_kernels.hip \
  $ROOT/reticulum_amd/csrc/wire_kernels.hip $(ls $ROOT/reticulum_amd/csrc/copy_kernels.hip 2>/dev/null) \
  $ROOT/reticulum_amd/csrc/token_capi.hip
echo built $OUT/$NAME
