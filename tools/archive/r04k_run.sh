#!/bin/bash
# c5 share on the generalized split encrypt (packed, length-ordered, per-key)
# against the build without it; then the split / token / rank-shape / runtime
# GPU tests on the product build.
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py tests/test_token_gpu.py tests/test_rank_shapes_gpu.py tests/test_runtime_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  RNSTOK_LIB=build_exp/nogen/librnstok.so timeout -k 10 120 python tools/c5_share.py > $O/c5_nogen_$r.json 2>/dev/null || exit 1
  timeout -k 10 120 python tools/c5_share.py > $O/c5_gen_$r.json 2>/dev/null || exit 1
done
for f in $O/c5_*.json; do python -c "
import json,sys; d=json.load(open('$f')); print('$f', round(d['encrypt']['ms'],4), round(d['decrypt']['ms'],4), round(d['encrypt']['frac_of_valu_peak'],4), d['ok'])"; done
