#!/bin/bash
# One-key decrypt quads as two half-quads (half the AES state and plaintext
# live: 165 -> 149 VGPRs at 768 threads; 128 with 3 spilled at 1024 threads,
# 4 waves/SIMD) vs the product (base8).
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
for v in h768 h1024; do
RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py tests/test_large_shapes_gpu.py tests/test_interleaved_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
tail -1 $O/tests_$v.log
done
L="build_exp/base8/librnstok.so build_exp/h768/librnstok.so build_exp/h1024/librnstok.so"
for args in "--rounds 30" "--ilv" "--length 1500" "--length 100" "--packed 64 --length 1500" "--packets 983040" "--rounds 30"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L --rounds 20 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt | grep -v round-trip
grep "round-trip" $O/ab.txt | grep -c "ok=True tokens==variant0: True"
