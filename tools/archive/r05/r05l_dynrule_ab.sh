#!/bin/bash
# Split encrypt: counter batches only where the static stride leaves AES waves
# unevenly loaded (dynrule) vs the round's product (base7).
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
RNSTOK_LIB=build_exp/dynrule/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py tests/test_token_gpu.py tests/test_large_shapes_gpu.py tests/test_launch_clock_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
L="build_exp/base7/librnstok.so build_exp/dynrule/librnstok.so"
for args in "" "--packets 983040" "--packets 1500000" "--packets 1500000 --length 1000" "--packets 1500000 --length 100" "--packets 983040 --keys 65536" "--packets 700000 --length 1500" ""; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L --rounds 24 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt | grep -v round-trip
grep "round-trip" $O/ab.txt | grep -c "ok=True tokens==variant0: True"
