#!/bin/bash
# Split-role encrypt, three builds in one process per shape: the product
# (k_encrypt), split (rows: LDS ring, interleaved: read-back), splitrb (rows:
# read-back, interleaved: LDS ring); tokens compared across builds.
set -o pipefail
O=gpurun_out/${1:-r04f}
mkdir -p $O
for args in "" "--ilv" "--length 1500" "--length 1500 --ilv"; do
  echo "== $args" >> $O/split_ab.txt
  timeout -k 10 200 python tools/exp_bench.py build_exp/base/librnstok.so build_exp/split/librnstok.so build_exp/splitrb/librnstok.so --rounds 24 $args >> $O/split_ab.txt 2>&1 || { tail -20 $O/split_ab.txt; exit 1; }
done
cat $O/split_ab.txt
