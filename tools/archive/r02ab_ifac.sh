#!/bin/bash
# IFAC kernel variants: fenced compressions (fewer VGPRs, 5 waves/SIMD), and
# forced occupancy.  One process per variant through RNSTOK_LIB, twice each.
# (RNSTOK_IFAC_FENCED / RNSTOK_IFAC_WAVES lived in the experimental k_ifac only;
# the tree kept the original kernel after this A/B.)
set -o pipefail
mkdir -p gpurun_out
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -Wno-unused-value"
declare -A V=( [base]="" [fenced]="-DRNSTOK_IFAC_FENCED" [f6]="-DRNSTOK_IFAC_FENCED -DRNSTOK_IFAC_WAVES=6" )
for k in base fenced f6; do
  mkdir -p build_exp/ifac_$k
  make -s -C reticulum_amd/csrc OUT=$PWD/build_exp/ifac_$k/librnstok.so FLAGS="$F ${V[$k]}" 2>/dev/null || exit 1
done
for r in 1 2; do
  for k in base fenced f6; do
    echo -n "$k run $r: "
    RNSTOK_LIB=$PWD/build_exp/ifac_$k/librnstok.so timeout -k 10 120 python3 tools/bench_configs.py --config wire --steps 10 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ok'], {k: round(v['ms'], 4) for k, v in d['stages'].items() if 'ifac' in k})" || exit 1
  done
done
