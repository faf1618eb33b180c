#!/bin/bash
# Split-role encrypt A/B: the product build against the
# k_encrypt_split build, one process each shape, interleaved rounds, tokens
# compared; then the token GPU tests on the split build.
set -o pipefail
O=gpurun_out/${1:-r04c}
mkdir -p $O
for args in "" "--ilv" "--length 1500" "--length 1500 --ilv" "--packets 262144"; do
  echo "== $args" >> $O/split_ab.txt
  timeout -k 10 150 python tools/exp_bench.py build_exp/base/librnstok.so build_exp/split/librnstok.so --rounds 20 $args >> $O/split_ab.txt 2>&1 || { tail -20 $O/split_ab.txt; exit 1; }
done
cat $O/split_ab.txt
RNSTOK_LIB=build_exp/split/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py tests/test_interleaved_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/split_tests.log 2>&1 || { tail -30 $O/split_tests.log; exit 1; }
tail -2 $O/split_tests.log
