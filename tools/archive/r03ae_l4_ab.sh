#!/bin/bash
# k_encrypt_long4: each lookup issued right after its address, in the order
# the terms are used (a variant built from a local edit of enc_block4 described in DESIGN.md §4.2 (d) and not kept; build_exp/l4il) vs the compiler's
# grouping (build_exp/base); A/B in one process at the c4 8-GPU shard, one
# Token-sized call and a 128-per-CU batch of 500-B packets.
set -o pipefail
O=gpurun_out/r03ae; mkdir -p $O
export TMPDIR=/tmp
V="build_exp/base/librnstok.so build_exp/l4il/librnstok.so"
for cfg in "--packets 32768 --length 16384" "--packets 1 --length 500" "--packets 32768 --length 500"; do
  echo "== $cfg" >> $O/ab.txt
  timeout -k 10 240 python3 tools/exp_bench.py $V --rounds 20 $cfg >> $O/ab.txt 2>&1 || { echo ab failed; tail $O/ab.txt; exit 1; }
done
cat $O/ab.txt
