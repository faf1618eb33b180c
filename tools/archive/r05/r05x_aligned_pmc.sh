#!/bin/bash
# HBM traffic and clock of c2 packed rows vs the same rows in 128-B-aligned
# slots: FETCH_SIZE, WRITE_SIZE, GRBM_GUI_ACTIVE and the
# fabric read requests, one rocprofv3 --pmc pass each, per layout.
set -o pipefail
OUT=gpurun_out/r05x
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
BASE="--steps 30 --warmup 2 --cpu-seconds 0 --no-e2e --no-node --one-layout"
for LAY in packed aligned; do
  if [ $LAY = aligned ]; then ARGS="$BASE --pt-stride 512 --tok-stride 640 --tok-offset 112"; else ARGS="$BASE"; fi
  for PASS in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    N=$(echo $PASS | tr ' ' '_' | cut -c1-40)
    timeout -s KILL 120 rocprofv3 --pmc $PASS --output-format csv -d $OUT/${LAY}_$N -o run -- python3 bench.py $ARGS \
      > $OUT/${LAY}_$N.log 2>&1 || { echo "pmc $LAY $N failed rc=$?"; tail -5 $OUT/${LAY}_$N.log; exit 1; }
  done
done
echo pmc done
