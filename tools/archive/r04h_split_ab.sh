#!/bin/bash
# Split-role encrypt + decrypt A/B against the product build (one process per
# shape, interleaved rounds, tokens compared), then the token GPU tests and
# tests/test_split_gpu.py on the split build.
set -o pipefail
O=gpurun_out/${1:-r04h}
mkdir -p $O
RNSTOK_LIB=build_exp/split/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py tests/test_token_gpu.py tests/test_interleaved_gpu.py tests/test_rank_shapes_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/split_tests.log 2>&1 || { tail -30 $O/split_tests.log; exit 1; }
tail -2 $O/split_tests.log
for args in "" "--ilv" "--length 1500" "--length 1500 --ilv"; do
  echo "== $args" >> $O/split_ab.txt
  timeout -k 10 200 python tools/exp_bench.py build_exp/base/librnstok.so build_exp/split/librnstok.so --rounds 24 $args >> $O/split_ab.txt 2>&1 || { tail -20 $O/split_ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/split_ab.txt
