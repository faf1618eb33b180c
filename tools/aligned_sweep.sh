#!/bin/bash
# Packed rows vs the same rows in 128-B-aligned slots (bench.py's aligned_rows)
# over plaintext lengths, one bench process per length.  Usage: tools/aligned_sweep.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/aligned_sweep}
mkdir -p $O
for LN in "64 1048576" "128 1048576" "256 1048576" "383 1048576" "500 1048576" "1000 524288" "1500 349525"; do
  set -- $LN
  timeout -k 10 200 python -u bench.py --length $1 --packets $2 --steps 10 --warmup 2 --no-node --no-e2e --cpu-seconds 0 \
    > $O/L$1.json 2> $O/L$1.err || { echo "L=$1 failed"; tail -5 $O/L$1.err; exit 1; }
done
echo sweep done
