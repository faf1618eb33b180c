#!/bin/bash
# Split encrypt, one key: next batch's IVs loaded during this batch (RNSTOK_SPLIT_IV_EARLY) vs product.
set -o pipefail
O=gpurun_out/r04am
mkdir -p $O
RNSTOK_LIB=build_exp/ive/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py tests/test_large_shapes_gpu.py tests/test_interleaved_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for args in "" "--ilv" "" "--ilv" "--length 1500" "--length 100"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py build_exp/base/librnstok.so build_exp/ive/librnstok.so --rounds 30 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt | grep -E "==|ms"
