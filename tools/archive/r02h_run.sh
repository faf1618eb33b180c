#!/bin/bash
set -e
O=gpurun_out/r02h; mkdir -p $O
timeout -k 10 300 python -u tools/exp_bench.py build_exp/dlv1/librnstok.so build_exp/dl2a12/librnstok.so build_exp/p3/librnstok.so build_exp/p3c/librnstok.so build_exp/p1/librnstok.so build_exp/p3a8/librnstok.so --packets 32768 --length 16384 --rounds 12 > $O/ab_prio.txt 2>&1
echo done
