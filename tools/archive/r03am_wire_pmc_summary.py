"""Per-kernel PMC means of the wire config (r03am_wire_pmc.sh) with the
issue-slot model of DESIGN.md §4.5: slots per SIMD = (SQ_INSTS_VALU -
SQ_ACTIVE_INST_VALU2 + SQ_INSTS_LDS) / 1024, cycles per XCD =
GRBM_GUI_ACTIVE / 8, clock = cycles / kernel-trace duration.  HBM bytes per
MI355X_MICROARCH.md: (2 * FETCH_SIZE + WRITE_SIZE) KiB."""
import collections
import csv
import glob
import sys

root = sys.argv[1]


def name(k):
    k = k.replace("rnstok::", "").replace("(anonymous namespace)::", "").replace("void ", "")
    return k.split("(")[0].strip()


agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/pmc_*/run_counter_collection.csv"):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "rnstok" not in r["Kernel_Name"]:
            continue
        per[(name(r["Kernel_Name"]), r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (k, c, _), v in per.items():
        agg[k][c].append(v)
dur = {}
for r in csv.DictReader(open(root + "/trace/run_kernel_stats.csv")):
    if "rnstok" in r["Name"]:
        dur[name(r["Name"])] = float(r["AverageNs"])
for k in sorted(agg):
    m = {c: sum(v) / len(v) for c, v in agg[k].items()}
    valu, valu2, lds = m.get("SQ_INSTS_VALU", 0), m.get("SQ_ACTIVE_INST_VALU2", 0), m.get("SQ_INSTS_LDS", 0)
    slots = (valu - valu2 + lds) / 1024
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    ns = dur.get(k)
    line = [f"{k}: {ns / 1e3:.1f} us" if ns else f"{k}:"]
    line.append(f"VALU {valu:.3e} dual {valu2 / valu:.1%}" if valu else "")
    line.append(f"LDS {lds:.3e} SALU {m.get('SQ_INSTS_SALU', 0):.3e} VMEM rd {m.get('SQ_INSTS_VMEM_RD', 0):.3e} wr {m.get('SQ_INSTS_VMEM_WR', 0):.3e}")
    if cyc:
        line.append(f"slots/SIMD {slots:.4g} cycles/XCD {cyc:.4g} slots*4/cycles {4 * slots / cyc:.1%}")
        if ns:
            line.append(f"clock {cyc / ns:.2f} GHz")
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        line.append(f"HBM {(2 * m['FETCH_SIZE'] + m['WRITE_SIZE']) * 1024 / 1e9:.3f} GB")
    print(" | ".join(x for x in line if x))
