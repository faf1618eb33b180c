"""Cross-check of the in-run launch clock (rt_clock_stamps) against the PMC.

  python tools/clock_check.py <pmc dir with run_counter_collection.csv> <bench json line> [steps]

The bench run under `rocprofv3 --pmc GRBM_GUI_ACTIVE` prints its own
roofline.in_run_clock (stamped by the kernels over the timed steps); the PMC
gives GRBM_GUI_ACTIVE (summed over the 8 XCDs) and the start/end of every
dispatch.  For the last `steps` dispatches of each kernel (the timed ones):
PMC clock = GRBM_GUI_ACTIVE / 8 / duration.  Prints both and their ratio.
"""
import collections
import csv
import glob
import json
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from pmc_summary import kernel_class  # noqa: E402


def main():
    root, line_path = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    disp = collections.defaultdict(dict)
    for f in glob.glob(root + "/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rnstok" not in r["Kernel_Name"] or r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                continue
            k = kernel_class(r["Kernel_Name"])
            d = int(r["Dispatch_Id"])
            disp[k][d] = (float(r["Counter_Value"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    line = None
    for ln in open(line_path):
        ln = ln.strip()
        if ln.startswith("{"):
            line = json.loads(ln)
    stamped = line["roofline"]["in_run_clock"]
    out = {}
    for k in ("encrypt", "decrypt"):
        ds = [disp[k][d] for d in sorted(disp[k])][-steps:]
        if not ds or k not in stamped:
            continue
        pmc = sum(c / 8 / ns for c, ns in ds) / len(ds)          # cycles per ns = GHz
        cyc = sum(c / 8 for c, _ in ds) / len(ds)
        out[k] = {"pmc_clock_ghz": pmc, "stamped_clock_ghz": stamped[k]["clock_ghz"],
                  "ratio_stamped_over_pmc": stamped[k]["clock_ghz"] / pmc,
                  "pmc_cycles_per_launch": cyc, "stamped_cycles_per_launch": stamped[k]["cycles_per_launch"],
                  "pmc_dispatch_ms": sum(ns for _, ns in ds) / len(ds) / 1e6,
                  "stamped_wg_span_ms": stamped[k]["wg_span_ms"], "dispatches": len(ds)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
