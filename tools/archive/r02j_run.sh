#!/bin/bash
O=gpurun_out/r02j; mkdir -p $O
for lib in build_exp/static/librnstok.so build_exp/dyn/librnstok.so; do
  for n in 300 1 2 17 64 65; do
    echo "== $lib n=$n" >> $O/edge.log
    RNSTOK_LIB=$lib timeout -k 5 40 python -u tools/dl2_edge.py $n >> $O/edge.log 2>&1 || { echo "FAILED rc=$? $lib n=$n" >> $O/edge.log; exit 0; }
  done
done
echo done >> $O/edge.log
