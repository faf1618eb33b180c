#!/bin/bash
# PMC of bench.py's c2 kernels for the base / touch variants (tools/r06a_touch_ab.sh)
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
BASE="--steps 30 --warmup 2 --cpu-seconds 0 --no-e2e --no-node --one-layout --no-aligned"
for v in base touch; do
  for PASS in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    N=$(echo $PASS | tr ' ' '_' | cut -c1-40)
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $O/${v}_$N -o run \
      -- python3 bench.py $BASE > $O/${v}_$N.log 2>&1 || { echo "pmc $v $N failed rc=$?"; tail -5 $O/${v}_$N.log; exit 1; }
  done
done
python3 tools/r06_pmc_cmp.py $O base touch | tee $O/pmc_cmp.txt
