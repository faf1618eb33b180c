#!/bin/bash
# Phase-staggered decrypt quads (RNSTOK_DEC_STAGGER 1-4) vs the product (base), one process.
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
RNSTOK_LIB=build_exp/stag1/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py tests/test_large_shapes_gpu.py tests/test_interleaved_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
L="build_exp/base/librnstok.so build_exp/stag1/librnstok.so build_exp/stag2/librnstok.so build_exp/stag3/librnstok.so build_exp/stag4/librnstok.so build_exp/stag1f/librnstok.so"
for args in "" "--ilv" "--length 1500" "--length 100" "--packed 64 --length 1500"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L --rounds 20 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt
