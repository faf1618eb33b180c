#!/bin/bash
# Uniform short tokens (<= 320 B) routed to the 1024-thread decrypt (short1024)
# vs the product (base8), and the same build against p1024 (every decrypt at
# 1024 threads) at the lengths around the threshold.
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
RNSTOK_LIB=build_exp/short1024/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py tests/test_large_shapes_gpu.py tests/test_interleaved_gpu.py tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
L="build_exp/base8/librnstok.so build_exp/short1024/librnstok.so"
for args in "--length 16" "--length 64" "--length 100" "--length 200" "--length 271" "--length 272" "--length 500" "--length 100 --packets 1500000" "--length 100 --packets 600000" "--length 64 --ilv"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L --rounds 20 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt | grep -v round-trip
grep "round-trip" $O/ab.txt | grep -c "ok=True tokens==variant0: True"
