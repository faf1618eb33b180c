#!/bin/bash
# The lane-cooperative long-token kernels (k_encrypt_long4: a quad of lanes
# per CBC chain, hashing on waves of their own; k_decrypt_long2: the HMAC
# split into a schedule-producer and a rounds-consumer wave) forced onto the
# c2 batch (build_exp/coop, RNSTOK_LONG_MAX_PER_CU) against the product's one
# packet per lane (build_exp/base); A/B in one process, tokens cross-checked.
set -o pipefail
O=gpurun_out/r03ah; mkdir -p $O
export TMPDIR=/tmp
V="build_exp/base/librnstok.so build_exp/coop/librnstok.so"
for cfg in "--packets 1048576 --length 500" "--packets 262144 --length 500"; do
  echo "== $cfg" >> $O/ab.txt
  timeout -k 10 300 python3 tools/exp_bench.py $V --rounds 10 $cfg >> $O/ab.txt 2>&1 || { echo ab failed; tail $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt
