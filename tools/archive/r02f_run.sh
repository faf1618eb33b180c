#!/bin/bash
# c4 per-GPU shard decrypt: k_decrypt_long (v1) vs k_decrypt_long2 (schedule producers) with 4/8/12 AES waves; long-token GPU tests.
set -e
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py -x -q -m gpu -k "long" --timeout 120 --timeout-method thread > $O/tests_long.log 2>&1
timeout -k 10 300 python -u tools/exp_bench.py build_exp/dlv1/librnstok.so build_exp/dl2a4/librnstok.so build_exp/dl2a8/librnstok.so build_exp/dl2a12/librnstok.so --packets 32768 --length 16384 --rounds 12 > $O/ab_c4s8.txt 2>&1
echo done
