#!/bin/bash
# Library variants (exp_ship/<v>), each in its own sustained run: the c3 bench
# line (2^20 x 500 B, 65 536 keys) and c5's rank share (tools/c5_share.py).
set -o pipefail
O=gpurun_out/${PERKEY_TAG:-r06q}
mkdir -p $O
B="--steps 40 --warmup 2 --cpu-seconds 0 --no-e2e --no-node --one-layout --no-aligned --keys 65536"
for r in 1 2; do
  for v in "$@"; do
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -k 10 200 python bench.py $B > $O/c3_${v}_$r.json 2> $O/c3_${v}_$r.err || { tail -5 $O/c3_${v}_$r.err; exit 1; }
    RNSTOK_LIB=exp_ship/$v/librnstok.so timeout -k 10 200 python tools/c5_share.py > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err || { tail -5 $O/c5_${v}_$r.err; exit 1; }
    python3 - $O/c3_${v}_$r.json $O/c5_${v}_$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ic = d["roofline"]["in_run_clock"]
print("%-9s c3 %.4f G/s enc %.4f ms %.3f GHz dec %.4f ms %.3f GHz | c5 enc %.4f ms %.3f GHz dec %.4f ms %.3f GHz ok %s" % (
    sys.argv[3], d["value"] / 1e9, d["kernels"]["encrypt"]["ms"], ic["encrypt"]["clock_ghz"],
    d["kernels"]["decrypt"]["ms"], ic["decrypt"]["clock_ghz"],
    c["encrypt"]["ms"], c["encrypt"]["kernel_clock_ghz"], c["decrypt"]["ms"], c["decrypt"]["kernel_clock_ghz"], c["ok"]))
PY
  done
done | tee $O/summary.txt
