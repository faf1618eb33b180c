#!/bin/bash
set -e
O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 300 python -u tools/exp_bench.py build_exp/dlv1/librnstok.so build_exp/dlv1aes/librnstok.so build_exp/dlv1sha/librnstok.so build_exp/dl2a12/librnstok.so build_exp/dl2aes/librnstok.so build_exp/dl2sha/librnstok.so --packets 32768 --length 16384 --rounds 12 --probe > $O/ab_probes.txt 2>&1
echo done
