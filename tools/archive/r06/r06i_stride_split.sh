#!/bin/bash
# Which side of the aligned-slot gain is whose: plaintext rows packed (500) or
# line-aligned (512), token rows packed (560) or ciphertext on a line (640, +112),
# each combination a bench.py run (headline kernels, stamped clock).
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
B="--steps 30 --warmup 2 --cpu-seconds 0 --no-e2e --no-node --one-layout --no-aligned"
for r in 1 2; do
for c in "pp:" "pa:--pt-stride 512" "tp:--tok-stride 640 --tok-offset 112" "aa:--pt-stride 512 --tok-stride 640 --tok-offset 112"; do
  n=${c%%:*}; a=${c#*:}
  timeout -k 10 200 python bench.py $B $a > $O/${n}_$r.json 2> $O/${n}_$r.err || { tail -5 $O/${n}_$r.err; exit 1; }
  python3 - $O/${n}_$r.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ic = d["roofline"]["in_run_clock"]
print(sys.argv[2], "enc %.4f ms %.3f GHz %.3f Mcyc | dec %.4f ms %.3f GHz %.3f Mcyc" % (
    d["kernels"]["encrypt"]["ms"], ic["encrypt"]["clock_ghz"], ic["encrypt"]["cycles_per_launch"] / 1e6,
    d["kernels"]["decrypt"]["ms"], ic["decrypt"]["clock_ghz"], ic["decrypt"]["cycles_per_launch"] / 1e6))
PY
done
done
