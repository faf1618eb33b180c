#!/bin/bash
# The product's c2 line with plaintext rows packed (500 B) vs on 512-B rows, tokens packed: what
# aligned plaintext reads would buy the encrypt (sustained runs, three each)
set -o pipefail
O=gpurun_out/r06ad
mkdir -p $O
B="--steps 40 --warmup 2 --cpu-seconds 0 --no-e2e --no-node --one-layout --no-aligned"
for r in 1 2 3; do
  for c in "pp:" "pa:--pt-stride 512"; do
    n=${c%%:*}; a=${c#*:}
    timeout -k 10 200 python bench.py $B $a > $O/${n}_$r.json 2> $O/${n}_$r.err || { tail -5 $O/${n}_$r.err; exit 1; }
    python3 - $O/${n}_$r.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ic = d["roofline"]["in_run_clock"]
print("%s value %.4f enc %.4f ms %.3f GHz %.3f Mcyc | dec %.4f ms %.3f GHz %.3f Mcyc" % (sys.argv[2], d["value"] / 1e9,
    d["kernels"]["encrypt"]["ms"], ic["encrypt"]["clock_ghz"], ic["encrypt"]["cycles_per_launch"] / 1e6,
    d["kernels"]["decrypt"]["ms"], ic["decrypt"]["clock_ghz"], ic["decrypt"]["cycles_per_launch"] / 1e6))
PY
  done
done | tee $O/summary.txt
