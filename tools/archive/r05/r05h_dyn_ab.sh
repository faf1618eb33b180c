#!/bin/bash
# Chunk counter vs static stride: decrypt batches of whole passes through the
# counter (qall), and the split encrypt taking its 64-packet batches from a
# counter (sdyn), against the product (base7); one process per shape.
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
RNSTOK_LIB=build_exp/sdyn/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py tests/test_token_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests_sdyn.log 2>&1 || { tail -30 $O/tests_sdyn.log; exit 1; }
tail -1 $O/tests_sdyn.log
RNSTOK_LIB=build_exp/qall/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py tests/test_large_shapes_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests_qall.log 2>&1 || { tail -30 $O/tests_qall.log; exit 1; }
tail -1 $O/tests_qall.log
L="build_exp/base7/librnstok.so build_exp/qall/librnstok.so build_exp/sdyn/librnstok.so"
for args in "" "--packets 983040" "--packets 1179648" "--length 1500" "--keys 65536" "--packets 786432"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L --rounds 20 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt | grep -v round-trip
grep "round-trip" $O/ab.txt | grep -vc "ok=True tokens==variant0: True"
