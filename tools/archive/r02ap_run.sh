#!/bin/bash
# Profile of bench.py with the steady-state warmup (kernel trace + PMC passes),
# then the headline line on the same box.
set -o pipefail
O=gpurun_out/r02ap; mkdir -p $O
export TMPDIR=/tmp
bash tools/profile.sh r02ap || { echo profile failed; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
cut -c1-200 $O/bench.json
echo all ok
