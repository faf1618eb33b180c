#!/bin/bash
# Per-key decrypt at 512 threads (2 waves/SIMD, paired quad loads, no spills)
# against the product's 768 (3 waves/SIMD, 18 VGPRs spilled): c3 and the c5
# rank share; per-key decrypt tests on the variant.
set -o pipefail
O=gpurun_out/r04x
mkdir -p $O
RNSTOK_LIB=build_exp/pk512/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py tests/test_runtime_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for args in "--keys 65536" "--keys 65536 --length 1500" "--keys 65536 --packed 64 --length 4096"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py build_exp/base/librnstok.so build_exp/pk512/librnstok.so --rounds 16 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt
for r in 1 2; do
  for v in base pk512; do
    RNSTOK_LIB=build_exp/$v/librnstok.so timeout -k 10 120 python tools/c5_share.py > $O/c5_${v}_$r.json 2>/dev/null || exit 1
  done
done
for f in $O/c5_*.json; do python -c "
import json; d=json.load(open('$f')); print('$f', round(d['encrypt']['ms'],4), round(d['decrypt']['ms'],4), round(d['decrypt']['frac_of_valu_peak'],4), d['ok'])"; done
