#!/bin/bash
# Round 6: packed-row decrypt line reuse.  Variants (exp_ship/<name>/librnstok.so):
#   base      the product
#   touch     odd quads touch the next pair's first unit (L2-served load)
#   tag       tag units loaded at the start of the last quad instead of before the loop
#   touchtag  both
# One-process A/B (tools/exp_bench.py, tokens and plaintexts cross-checked), then
# per-variant PMC of bench.py's decrypt: FETCH_SIZE, WRITE_SIZE, GRBM_GUI_ACTIVE.
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
V="base touch tag touchtag"
L=""; for v in $V; do L="$L exp_ship/$v/librnstok.so"; done
for args in "--rounds 20" "--rounds 20 --length 1500" "--rounds 20 --length 383"; do
  echo "== $args" >> $O/ab.txt
  timeout -k 10 240 python tools/exp_bench.py $L $args >> $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
done
grep -v amdgpu.ids $O/ab.txt
BASE="--steps 30 --warmup 2 --cpu-seconds 0 --no-e2e --no-node --one-layout --no-aligned"
for v in base touch touchtag; do
  for PASS in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    N=$(echo $PASS | tr ' ' '_' | cut -c1-40)
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $O/${v}_$N -o run \
      -- python3 bench.py $BASE > $O/${v}_$N.log 2>&1 || { echo "pmc $v $N failed rc=$?"; tail -5 $O/${v}_$N.log; exit 1; }
  done
done
python3 tools/r06_pmc_cmp.py $O base touch touchtag | tee $O/pmc_cmp.txt
echo done
