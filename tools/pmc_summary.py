"""Summarise rocprofv3 PMC csv passes per rnstok kernel (mean over dispatches).

  python tools/pmc_summary.py gpurun_out/prof_<tag> [--json out.json]

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide
16-B-per-lane reads, so traffic = (2*FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import collections
import csv
import glob
import json
import sys


def kernel_class(name):
    """encrypt / decrypt (the c2 kernels, as bench.py expects), or the kernel's
    own name for the others (long-token, verify, key setup, hkdf, ...)."""
    base = name.replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].replace("rnstok::", "").replace("void ", "").strip()
    if base in ("k_encrypt", "k_decrypt", "k_encrypt_split"):
        return base[2:].replace("_split", "")
    return base


def summarise(root):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(root + "/pmc_*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "rnstok" not in k:
                continue
            k = kernel_class(k)
            agg[k][(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = {}
    for k, d in agg.items():
        per = collections.defaultdict(list)
        for (c, disp), v in d.items():
            per[c].append(v)
        out[k] = {c: sum(v) / len(v) for c, v in sorted(per.items())}
        if "FETCH_SIZE" in out[k] and "WRITE_SIZE" in out[k]:
            out[k]["hbm_bytes_per_launch"] = (2 * out[k]["FETCH_SIZE"] + out[k]["WRITE_SIZE"]) * 1024
            out[k]["hbm_bytes_per_launch_uncorrected"] = (out[k]["FETCH_SIZE"] + out[k]["WRITE_SIZE"]) * 1024
    return out


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_r01"
    out = summarise(root)
    for k, d in out.items():
        print(k)
        for c, v in d.items():
            print("  %-34s %16.6g" % (c, v))
    if "--workload" in sys.argv:   # e.g. --workload 1048576,500,1  (packets,length,keys)
        p, l, k = (int(x) for x in sys.argv[sys.argv.index("--workload") + 1].split(","))
        out["_workload"] = {"packets": p, "length": l, "keys": k}
    if "--json" in sys.argv:
        path = sys.argv[sys.argv.index("--json") + 1]
        with open(path, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
        print("wrote", path)


if __name__ == "__main__":
    main()
