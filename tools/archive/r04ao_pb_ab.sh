#!/bin/bash
# Decrypt: the block before the tail quad read only when the tail needs it (tb < 3) vs HEAD.
set -o pipefail
O=gpurun_out/r04ao
mkdir -p $O
RNSTOK_LIB=build_exp/base/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py tests/test_large_shapes_gpu.py tests/test_fuzz_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for args in "" "--ilv" "" "--length 100" "--length 1500"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py build_exp/head/librnstok.so build_exp/base/librnstok.so --rounds 30 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt | grep -E "==|ms"
