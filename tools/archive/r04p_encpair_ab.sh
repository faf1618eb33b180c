#!/bin/bash
# Paired plaintext quad loads in the split encrypt's AES waves (RNSTOK_ENC_PAIR)
# against the product build (decrypt pairs on in both): tests on the variant,
# one-process A/Bs, FETCH counters of both.
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
RNSTOK_LIB=build_exp/encpair/librnstok.so timeout -k 10 300 python -u -m pytest tests/test_token_gpu.py tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for args in "" "--length 1500" "--keys 65536" "--packed 64 --length 1500"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 200 python tools/exp_bench.py build_exp/base/librnstok.so build_exp/encpair/librnstok.so --rounds 24 $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base encpair; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/p_$v/pmc_1 -o run --output-format csv -- python3 tools/exp_bench.py build_exp/$v/librnstok.so --rounds 3 > $O/pmc_$v.log 2>&1 || { tail -20 $O/pmc_$v.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/p_$v/pmc_2 -o run --output-format csv -- python3 tools/exp_bench.py build_exp/$v/librnstok.so --rounds 3 > $O/pmc2_$v.log 2>&1 || { tail -20 $O/pmc2_$v.log; exit 1; }
done
python tools/pmc_summary.py $O/p_base > $O/pmc_base.txt 2>&1; python tools/pmc_summary.py $O/p_encpair > $O/pmc_encpair.txt 2>&1
grep -A8 "^encrypt\|^decrypt" $O/pmc_base.txt $O/pmc_encpair.txt | grep -E "crypt|FETCH|WRITE|hbm"
