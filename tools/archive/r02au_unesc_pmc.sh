#!/bin/bash
# PMC of the wire config (HDLC unescape and friends): instruction counts per
# kernel, to see what bounds k_hdlc_unescape (store instructions vs VALU).
set -o pipefail
O=gpurun_out/r02au; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc1 -o run -- python3 tools/bench_configs.py --config wire --steps 5 > $O/pmc1.log 2>&1 || { echo pmc1 failed; tail -5 $O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc2 -o run -- python3 tools/bench_configs.py --config wire --steps 5 > $O/pmc2.log 2>&1 || { echo pmc2 failed; tail -5 $O/pmc2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for p in ("pmc1", "pmc2"):
    f = glob.glob(f"gpurun_out/r02au/{p}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    disp = set()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        if not any(s in k for s in ("unescape", "flag", "hdlc")): continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add((k, r["Dispatch_Id"]))
    nd = collections.Counter(k for k, _ in disp)
    for k in agg:
        print(p, k, {c: round(v / nd[k]) for c, v in agg[k].items()})
PY
