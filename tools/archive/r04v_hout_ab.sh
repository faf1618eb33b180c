#!/bin/bash
# Outer HMAC compression on the split encrypt's AES waves (RNSTOK_SPLIT_HOUT)
# against the product build: split/token tests on the variant, one-process
# A/Bs, the wait probe of the variant.
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
RNSTOK_LIB=build_exp/hout/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py tests/test_token_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for args in "" "--length 1500" "--length 100" "--packed 64 --length 1500"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 200 python tools/exp_bench.py build_exp/base/librnstok.so build_exp/hout/librnstok.so --rounds 24 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt
for args in "" "--length 1500"; do
  RNSTOK_LIB=build_exp/houtprobe/librnstok.so timeout -k 10 120 python tools/split_wait_probe.py $args >> $O/split_wait.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
done
cut -c1-420 $O/split_wait.jsonl
