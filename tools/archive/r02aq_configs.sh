#!/bin/bash
# Every non-headline config with the steady-state warmup (tools/bench_configs.py).
set -o pipefail
O=gpurun_out/r02aq; mkdir -p $O
for c in ${CONFIGS:-c3 ident c4 c4s8 c5 wire resource ratchet}; do
  timeout -k 10 240 python tools/bench_configs.py --config $c 2>>$O/configs.err | tee -a $O/configs.jsonl | cut -c1-260 || { echo "config $c failed"; exit 1; }
done
echo all ok
