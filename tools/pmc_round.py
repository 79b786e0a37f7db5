"""Per-kernel medians of rocprofv3 --pmc counters for the shared-critic round kernels (diagnostics).
Usage: python tools/pmc_round.py DIR [DIR ...]  (each DIR one rocprofv3 -d output with a *counter_collection.csv)"""
import collections
import csv
import glob
import os
import statistics
import sys

KEYS = ("sc_k1", "sc_gemm", "sc_k3", "sc_bwd", "sc_grad_adam", "sc_prep_snapshot", "step_kernel")


def main():
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                name = row.get("Kernel_Name", "")
                k = next((k for k in KEYS if k in name), None)
                if k:
                    vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k in KEYS:
        if k in vals:
            print(k, {c: round(statistics.median(v), 1) for c, v in sorted(vals[k].items())})


if __name__ == "__main__":
    main()
