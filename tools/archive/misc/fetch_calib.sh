#!/bin/bash
# FETCH_SIZE calibration on the token kernels' access pattern (tools/fetch_calib.hip); run via gpurun.
set -o pipefail
OUT=gpurun_out/fetch_calib
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for K in packets stream; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$K -o run -- ./build_tools/fetch_calib $K > $OUT/$K.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for k in ("packets", "stream"):
    vals = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/fetch_calib/{k}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "FETCH_SIZE" and "k_" in r["Kernel_Name"]:
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = sorted(vals.values())
    alg = (1 << 20) * 500
    print(k, "FETCH_SIZE KiB per launch:", v, " algorithmic KiB:", alg / 1024,
          " ratio FETCH/alg:", [round(x * 1024 / alg, 3) for x in v])
PY
