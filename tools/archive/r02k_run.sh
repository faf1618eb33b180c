#!/bin/bash
O=gpurun_out/r02k; mkdir -p $O
for n in 1 2 17 64 65 129 300; do
  echo "== n=$n" >> $O/edge.log
  timeout -k 5 40 python -u tools/dl2_edge.py $n >> $O/edge.log 2>&1 || { echo "FAILED rc=$? n=$n" >> $O/edge.log; exit 1; }
done
timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py -x -q -m gpu -k "long" --timeout 120 --timeout-method thread > $O/tests_long.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/exp_bench.py build_exp/dlv1/librnstok.so build_exp/static/librnstok.so build_exp/dyn/librnstok.so build_exp/dynp3/librnstok.so build_exp/dl2aes/librnstok.so build_exp/dl2sha/librnstok.so --packets 32768 --length 16384 --rounds 12 --probe > $O/ab_dyn.txt 2>&1
echo done >> $O/edge.log
