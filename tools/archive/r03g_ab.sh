#!/bin/bash
# Round 3: k_encrypt_long4 at the c4 8-GPU shard (32768 x 16 KiB): ring swizzle,
# round key folded into a DPP xor, 2 vs 4 hashing waves; A/B in one process.
set -o pipefail
O=gpurun_out/r03g; mkdir -p $O
export TMPDIR=/tmp
V="build_exp/l4_base/librnstok.so build_exp/l4_swz/librnstok.so build_exp/l4_fold/librnstok.so build_exp/l4_fold_hw4/librnstok.so"
for cfg in "--packets 32768 --length 16384" "--packets 1024 --length 500" "--packets 32768 --length 500"; do
  echo "== $cfg" >> $O/ab.txt
  timeout -k 10 240 python3 tools/exp_bench.py $V --rounds 20 $cfg >> $O/ab.txt 2>&1 || { echo ab failed; tail $O/ab.txt; exit 1; }
done
cat $O/ab.txt
