#!/bin/bash
# Paired quad loads in the packed-rows decrypt (RNSTOK_DEC_PAIR) against the
# product build: token/decrypt GPU tests on the variant, one-process A/Bs,
# then FETCH/WRITE counters of both variants' decrypt.
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
[ -n "$PMC_ONLY" ] || RNSTOK_LIB=build_exp/pair/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pair_tests.log 2>&1 || { tail -30 $O/pair_tests.log; exit 1; }
tail -2 $O/pair_tests.log
[ -n "$PMC_ONLY" ] || for args in "" "--length 1500" "--length 100" "--packed 64 --length 1500"; do
  echo "== $args" >> $O/pair_ab.txt
  timeout -k 10 200 python tools/exp_bench.py build_exp/base/librnstok.so build_exp/pair/librnstok.so --rounds 24 $args >> $O/pair_ab.txt 2>&1 || { tail -20 $O/pair_ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/pair_ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base pair; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/p_$v/pmc_1 -o run --output-format csv -- python3 tools/exp_bench.py build_exp/$v/librnstok.so --rounds 3 > $O/pmc_$v.log 2>&1 || { tail -20 $O/pmc_$v.log; exit 1; }
done
python tools/pmc_summary.py $O/p_base > $O/pmc_base.txt 2>&1; python tools/pmc_summary.py $O/p_pair > $O/pmc_pair.txt 2>&1
grep -A6 "^decrypt" $O/pmc_base.txt $O/pmc_pair.txt
