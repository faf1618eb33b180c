#!/bin/bash
# One-process A/B of library variants (tools/exp_bench.py, outputs cross-checked),
# then per-variant PMC of bench.py's c2 kernels (FETCH_SIZE, WRITE_SIZE, GRBM).
#   tools/r06_ab_pmc.sh <out-tag> "<exp_bench args>;<exp_bench args>..." <variant>...
# variants are exp_ship/<name>/librnstok.so
set -o pipefail
TAG=$1; CASES=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
L=""; for v in "$@"; do L="$L exp_ship/$v/librnstok.so"; done
IFS=';' read -ra CS <<< "$CASES"
for args in "${CS[@]}"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 300 python tools/exp_bench.py $L $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt
[ -n "$NO_PMC" ] && exit 0
BASE="--steps 30 --warmup 2 --cpu-seconds 0 --no-e2e --no-node --one-layout --no-aligned $BENCH_ARGS"
for v in "$@"; do
  IFS=';' read -ra PS <<< "${PMC_PASSES:-FETCH_SIZE;WRITE_SIZE;GRBM_GUI_ACTIVE GRBM_COUNT}"
  for PASS in "${PS[@]}"; do
    N=$(echo $PASS | tr ' ' '_' | cut -c1-40)
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $O/${v}_$N -o run \
      -- python3 bench.py $BASE > $O/${v}_$N.log 2>&1 || { echo "pmc $v $N failed rc=$?"; tail -5 $O/${v}_$N.log; exit 1; }
  done
done
python3 tools/r06_pmc_cmp.py $O "$@" | tee $O/pmc_cmp.txt
