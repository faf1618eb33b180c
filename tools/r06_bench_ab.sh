#!/bin/bash
# Whole-bench A/B of library variants: each variant times its own sustained
# run (bench.py, headline kernels only), so clock effects show (an A/B that
# interleaves variants launch by launch shares one clock between them).
#   tools/r06_bench_ab.sh <out-tag> <rounds> <variant>...   (exp_ship/<variant>/librnstok.so)
set -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
B="--steps 40 --warmup 2 --cpu-seconds 0 --no-e2e --no-node --one-layout --no-aligned $BENCH_ARGS"
for r in $(seq 1 $R); do
  for v in "$@"; do
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -k 10 200 python bench.py $B > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    python3 - $O/${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ic = d["roofline"]["in_run_clock"]
print("%-10s value %.4f G/s  enc %.4f ms %.3f GHz %.3f Mcyc | dec %.4f ms %.3f GHz %.3f Mcyc" % (
    sys.argv[2], d["value"] / 1e9, d["kernels"]["encrypt"]["ms"], ic["encrypt"]["clock_ghz"],
    ic["encrypt"]["cycles_per_launch"] / 1e6, d["kernels"]["decrypt"]["ms"], ic["decrypt"]["clock_ghz"],
    ic["decrypt"]["cycles_per_launch"] / 1e6))
PY
  done
done | tee $O/summary.txt
