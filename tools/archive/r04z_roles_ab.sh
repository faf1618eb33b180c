#!/bin/bash
# Decrypt with roles by queue (k_decrypt_roles + k_decrypt_fixup, RNSTOK_DEC_ROLES)
# against the product's k_decrypt: decrypt GPU tests on the variant, then
# one-process A/Bs with 12 / 8 / 10 AES waves at the start.
set -o pipefail
O=gpurun_out/r04z3
mkdir -p $O
RNSTOK_LIB=build_exp/roles8pf/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py tests/test_token_gpu.py tests/test_interleaved_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for args in "" "--ilv" "--length 1500" "--length 100"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py build_exp/base/librnstok.so build_exp/roles8/librnstok.so build_exp/roles8pf/librnstok.so --rounds 16 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt
