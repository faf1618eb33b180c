"""Compare per-launch PMC of the c2 token kernels between library variants.

  python tools/r06_pmc_cmp.py <dir> <variant>...

<dir>/<variant>_<PASS>/run_counter_collection.csv are rocprofv3 --pmc passes of
bench.py (one pass per counter group).  Per kernel class (encrypt / decrypt):
mean FETCH_SIZE / WRITE_SIZE / GRBM_GUI_ACTIVE per dispatch, the traffic in GB
per launch ((2 x FETCH + WRITE) x 1 KiB, MI355X_MICROARCH.md §HBM) and its
ratio to the algorithmic bytes of a c2 launch.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import kernel_class  # noqa: E402

ALGO = {"encrypt": 1.128e9, "decrypt": 1.120e9}   # c2: 2^20 x 500 B, DESIGN.md §4


def variant(root, v):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{root}/{v}_*/run_counter_collection.csv") + glob.glob(f"{root}/{v}_*/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "rnstok" not in k:
                continue
            agg[kernel_class(k)][(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = {}
    for k, d in agg.items():
        per = collections.defaultdict(list)
        for (c, _), val in d.items():
            per[c].append(val)
        out[k] = {c: sum(x) / len(x) for c, x in per.items()}
        m = out[k]
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["traffic_gb"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024 / 1e9
            if k in ALGO:
                m["traffic_x"] = m["traffic_gb"] * 1e9 / ALGO[k]
    return out


def main():
    root, vs = sys.argv[1], sys.argv[2:]
    res = {v: variant(root, v) for v in vs}
    for k in ("encrypt", "decrypt"):
        print(k)
        for v in vs:
            v_name = v
            m = res[v].get(k, {})
            print("  %-10s fetch %8.3f GB  write %8.3f GB  traffic %6.3f GB (%.2fx)  GRBM_GUI_ACTIVE %10.0f" % (
                v, 2 * m.get("FETCH_SIZE", 0) * 1024 / 1e9, m.get("WRITE_SIZE", 0) * 1024 / 1e9,
                m.get("traffic_gb", 0), m.get("traffic_x", 0), m.get("GRBM_GUI_ACTIVE", 0)))
            if "SQ_INSTS_VALU" in m:
                v, v2 = m["SQ_INSTS_VALU"], m.get("SQ_ACTIVE_INST_VALU2", 0)
                print("  %-10s VALU %.4g  VALU2 %.4g (dual-issued %.1f %%)  LDS %.4g  issue slots (VALU-VALU2+LDS) %.4g" % (
                    v_name, v, v2, 200 * v2 / v, m.get("SQ_INSTS_LDS", 0), v - v2 + m.get("SQ_INSTS_LDS", 0)))
    with open(os.path.join(root, "pmc_cmp.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
