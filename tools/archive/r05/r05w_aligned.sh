#!/bin/bash
# Packed rows vs rows in 128-B-aligned slots (plaintext rows at 512 B, token
# rows at 640 B with the ciphertext starting on a line): the same kernels,
# alternated, each run with its in-run clock.
set -o pipefail
O=gpurun_out/r05w
mkdir -p $O
A="--one-layout --no-node --no-e2e --cpu-seconds 0"
for r in 1 2 3; do
  timeout -k 10 200 python bench.py $A > $O/packed_$r.json 2> $O/err || { tail $O/err; exit 1; }
  timeout -k 10 200 python bench.py $A --pt-stride 512 --tok-stride 640 --tok-offset 112 > $O/aligned_$r.json 2> $O/err || { tail $O/err; exit 1; }
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05w/*.json")):
    l = json.loads(open(f).read().strip().splitlines()[-1])
    r = l["roofline"]; k = l["kernels"]; c = r["in_run_clock"]
    print(f.split("/")[-1], "%.4f G/s" % (l["value"] / 1e9), "enc %.4f dec %.4f ms" % (k["encrypt"]["ms"], k["decrypt"]["ms"]),
          "clk enc %.3f dec %.3f" % (c["encrypt"]["clock_ghz"], c["decrypt"]["clock_ghz"]),
          "cyc enc %.3fM dec %.3fM" % (c["encrypt"]["cycles_per_launch"] / 1e6, c["decrypt"]["cycles_per_launch"] / 1e6))
PY
