"""Per-case PMC table of tools/issue_model_probe.hip runs under rocprofv3 --pmc.

  python tools/probe_pmc_summary.py gpurun_out/r03b/pmc1/run_counter_collection.csv [more.csv ...]

Counters are summed over the XCDs of each dispatch; the last dispatch of each
case (a steady one) is printed, with the dual-issued share of the VALU
instructions (2 x SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU)."""
import collections
import csv
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sys.argv[1:]:
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(r["Kernel_Name"], int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, d, c), v in sorted(per.items(), key=lambda x: x[0][1]):
            agg[k.split("(")[0].replace("void ", "")][c].append(v)
    cols = ["SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU2", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY",
            "SQ_IFETCH", "GRBM_GUI_ACTIVE"]
    print("%-30s" % "case" + "".join("%15s" % c.replace("SQ_", "") for c in cols) + "  dual-issued share")
    for k, d in agg.items():
        if not k.startswith("k_"):
            continue
        last = {c: d[c][-1] for c in cols if d.get(c)}
        share = 2 * last.get("SQ_ACTIVE_INST_VALU2", 0) / last["SQ_INSTS_VALU"] if last.get("SQ_INSTS_VALU") else 0
        print("%-30s" % k[2:32] + "".join("%15.4g" % last.get(c, float("nan")) for c in cols) + "  %.3f" % share)


if __name__ == "__main__":
    main()
