#!/bin/bash
# Round 3: trace + PMC of both layouts (tools/r03i_run.sh PART=prof), the
# unescape A/B (tools/r03j_unesc_ab.sh), and decrypt at 1024 vs 768 threads
# in both layouts (A/B in one process).
set -o pipefail
O=gpurun_out/r03k; mkdir -p $O
export TMPDIR=/tmp
for lay in "--ilv" ""; do
  echo "== dec WG A/B $lay" >> $O/dec_wg_ab.txt
  timeout -k 10 200 python3 tools/exp_bench.py build_exp/prod/librnstok.so build_exp/dec1024/librnstok.so --rounds 20 $lay >> $O/dec_wg_ab.txt 2>&1 || { echo ab failed; tail $O/dec_wg_ab.txt; exit 1; }
done
cat $O/dec_wg_ab.txt
PART=prof bash tools/r03i_run.sh && bash tools/r03j_unesc_ab.sh
