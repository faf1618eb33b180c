#!/bin/bash
# c5 rank share PMC on the round-6 build: packed, decrypt outputs in slots, everything in slots.
# FETCH_SIZE, WRITE_SIZE, GRBM, and the fabric read/write requests, one pass each.
set -o pipefail
O=gpurun_out/r06c5pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for V in packed dec_out all; do
  A=""; [ $V = all ] && A="--align"; [ $V = dec_out ] && A="--align-sides dec_out"
  for P in FETCH_SIZE WRITE_SIZE "GRBM_GUI_ACTIVE GRBM_COUNT" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    N=$(echo $P | tr ' ' '_')
    timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $O/${V}_$N -o run -- python3 tools/c5_share.py --steps 5 $A > $O/${V}_$N.log 2>&1 || { echo "fail $V $N"; tail -5 $O/${V}_$N.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections, json
out = {}
for v in ("packed", "dec_out", "all"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/r06c5pmc/{v}_*/run_counter_collection.csv") + glob.glob(f"gpurun_out/r06c5pmc/{v}_*/*/run_counter_collection.csv"):
        per = collections.defaultdict(float)
        rows = list(csv.DictReader(open(f)))
        for r in rows:
            k = r["Kernel_Name"]
            kind = "decrypt" if "k_decrypt" in k else ("encrypt" if "k_encrypt" in k else None)
            if kind:
                per[(kind, r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (kind, c, _), val in per.items():
            agg[kind][c].append(val)
    out[v] = {k: {c: sorted(x)[len(x) // 2] for c, x in d.items()} for k, d in agg.items()}
for v, d in out.items():
    for k, m in sorted(d.items()):
        print("%-8s %-8s FETCH %.3f GB  WRITE %.3f GB  RDREQ %.3g  WRREQ %.3g  GRBM/XCD %.4g" % (v, k,
              m.get("FETCH_SIZE", 0) * 1024 / 1e9, m.get("WRITE_SIZE", 0) * 1024 / 1e9, m.get("TCC_EA0_RDREQ_sum", 0),
              m.get("TCC_EA0_WRREQ_sum", 0), m.get("GRBM_GUI_ACTIVE", 0) / 8))
json.dump(out, open("gpurun_out/r06c5pmc/summary.json", "w"), indent=1)
PY
