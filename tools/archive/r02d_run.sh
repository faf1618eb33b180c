#!/bin/bash
# Round-2 measurement batch: headline bench, sharded configs at N=1, derive_keyset A/B (fused vs two launches).
set -e
O=gpurun_out/r02d
mkdir -p $O
T="timeout -k 10"
$T 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err
$T 300 python -u bench.py --config c4 --sharded-reps 3 --no-e2e --cpu-seconds 0 > $O/bench_c4.json 2> $O/bench_c4.err
$T 300 python -u bench.py --config c5 --sharded-reps 3 --no-e2e --cpu-seconds 0 > $O/bench_c5.json 2> $O/bench_c5.err
for r in 1 2; do
  $T 200 python -u tools/bench_configs.py --config ident --steps 10 >> $O/ident_fused.jsonl
  RNSTOK_LIB=build_exp/nofused/librnstok.so $T 200 python -u tools/bench_configs.py --config ident --steps 10 >> $O/ident_twolaunch.jsonl
done
$T 300 python -u tools/bench_configs.py --config c5 --steps 10 > $O/c5_tool.json
echo done
