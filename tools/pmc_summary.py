"""Mean per-dispatch PMC counter values of one kernel from rocprofv3 --pmc CSV directories (diagnostics).

    python tools/pmc_summary.py DIR [DIR ...] [--kernel step_kernel]
"""
import argparse
import collections
import csv
import os

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--kernel", default="step_kernel")
a = ap.parse_args()
for d in a.dirs:
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in rows:
        if a.kernel not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    waves = None
    for c in sorted(agg):
        v = agg[c] / len(disp[c])
        if c == "SQ_WAVES":
            waves = v
        print(f"{d:28s} {c:24s} {v:14.4g}")
