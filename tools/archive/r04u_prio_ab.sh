#!/bin/bash
# Hashing waves of the split encrypt at s_setprio 2 (RNSTOK_SPLIT_PRIO), with
# and without the no-wait hand-over, against the product build; wait probe.
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
RNSTOK_LIB=build_exp/prio/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for args in "" "--length 1500" "--keys 65536" "--ilv" "--packed 64 --length 1500"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 200 python tools/exp_bench.py build_exp/base/librnstok.so build_exp/prio/librnstok.so build_exp/nowaitprio/librnstok.so --rounds 24 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt
for args in "" "--length 1500"; do
  RNSTOK_LIB=build_exp/prioprobe/librnstok.so timeout -k 10 120 python tools/split_wait_probe.py $args >> $O/split_wait.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
done
cut -c1-420 $O/split_wait.jsonl
