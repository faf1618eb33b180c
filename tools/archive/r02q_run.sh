#!/bin/bash
O=gpurun_out/r02q; mkdir -p $O
for k in random zero seq sorted; do
  echo "== kidx=$k" >> $O/c3_kidx.txt
  timeout -k 10 200 python -u tools/exp_bench.py reticulum_amd/librnstok.so --keys 65536 --kidx $k --rounds 12 >> $O/c3_kidx.txt 2>&1 || exit 1
done
echo done
