#!/bin/bash
# Split encrypt on packed rows: LDS ring (product) vs read-back of every
# quad from the token rows (RNSTOK_SPLIT_ROWS_RB=1), by packet length.
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
for args in "" "--length 1000" "--length 1500" "--length 4096 --packets 262144" "--length 16384 --packets 262144" "--keys 65536 --length 1500"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py build_exp/base/librnstok.so build_exp/rowsrb/librnstok.so --rounds 16 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt
