#!/bin/bash
# Decrypt with plaintext blocks stored inside the quad (RNSTOK_DEC_STORE_IN: 151 VGPRs at
# 768 threads, 3 spilled at 1024 instead of 11), at 768 and at 1024 threads, against
# the product build; token/split/interleaved tests on the variant.
set -o pipefail
O=gpurun_out/r04af
mkdir -p $O
RNSTOK_LIB=build_exp/storein1024/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py tests/test_split_gpu.py tests/test_interleaved_gpu.py tests/test_large_shapes_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for args in "" "--ilv" "--length 1500" "--packets 262144" "--packets 262144 --length 16384"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py build_exp/base/librnstok.so build_exp/storein/librnstok.so build_exp/storein1024/librnstok.so --rounds 20 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt
