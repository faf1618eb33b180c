#!/bin/bash
set -e
O=gpurun_out/r02i; mkdir -p $O
timeout -k 10 300 python -u tools/exp_bench.py build_exp/dlv1/librnstok.so build_exp/static/librnstok.so build_exp/dyn/librnstok.so build_exp/dynp3/librnstok.so build_exp/dyna8/librnstok.so build_exp/dynp3a8/librnstok.so --packets 32768 --length 16384 --rounds 12 > $O/ab_dyn.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py -x -q -m gpu -k "long" --timeout 120 --timeout-method thread > $O/tests_long.log 2>&1
echo done
