"""Summarise rocprofv3 PMC csv passes per rnstok kernel (mean over dispatches)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_r01"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
ndisp = collections.defaultdict(set)
for f in glob.glob(root + "/pmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "rnstok" not in k:
            continue
        k = "encrypt" if "encrypt" in k else ("decrypt" if "decrypt" in k else "key_setup")
        agg[k][(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
        ndisp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k, d in agg.items():
    per = collections.defaultdict(list)
    for (c, disp), v in d.items():
        per[c].append(v)
    print(k)
    for c in sorted(per):
        v = per[c]
        print("  %-28s %14.6g" % (c, sum(v) / len(v)))
