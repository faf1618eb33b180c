#!/bin/bash
# FETCH_SIZE and fabric read requests on the token kernels' access patterns
# against known byte counts (tools/fetch_calib.hip); run via gpurun.
set -o pipefail
OUT=gpurun_out/fetch_calib
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for K in packets stream rows560 rows640; do
  for PASS in "FETCH_SIZE" "TCC_EA0_RDREQ_sum"; do
    N=$(echo $PASS | cut -c1-12)
    timeout -s KILL 60 rocprofv3 --pmc $PASS --output-format csv -d $OUT/${K}_$N -o run -- ./tools/_bin/fetch_calib $K > $OUT/${K}_$N.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import csv, glob, collections
alg = {"packets": (1 << 20) * 500, "stream": (1 << 20) * 500, "rows560": (1 << 20) * 560, "rows640": (1 << 20) * 560}
for k in alg:
    out = {}
    for c, d in (("FETCH_SIZE", "FETCH_SIZE"), ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDRE")):
        vals = collections.defaultdict(float)
        for f in glob.glob(f"gpurun_out/fetch_calib/{k}_{d}/**/run_counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_" in r["Kernel_Name"]:
                    vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
        out[c] = sorted(vals.values())[len(vals) // 2] if vals else None
    f_kib, rq = out["FETCH_SIZE"], out["TCC_EA0_RDREQ_sum"]
    print("%-8s known %.1f MB  FETCH_SIZE %.1f MB (%.3fx)  requests %.3g (%.1f B per request for the known bytes)" % (
        k, alg[k] / 1e6, f_kib * 1024 / 1e6, f_kib * 1024 / alg[k], rq, alg[k] / rq))
PY
