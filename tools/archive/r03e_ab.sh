#!/bin/bash
# Round 3: v_perm vs shift+and_or T-table addresses (RNSTOK_PERM_ADDR), A/B in one process per config.
set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
export TMPDIR=/tmp
A=build_exp/permaddr/librnstok.so; B=build_exp/shiftaddr/librnstok.so
timeout -k 10 120 build_exp/issue_model_probe X_ 2000 > $O/probe.txt 2>&1 || { echo probe failed; exit 1; }
cat $O/probe.txt
for cfg in "" "--keys 65536" "--packets 32768 --length 16384" "--packets 1024" "--length 100"; do
  echo "== $cfg" | tee -a $O/ab.txt
  timeout -k 10 180 python3 tools/exp_bench.py $A $B --rounds 20 $cfg >> $O/ab.txt 2>&1 || { echo ab failed; tail $O/ab.txt; exit 1; }
done
cat $O/ab.txt
