"""Summarise a rocprofv3 --pmc SQ pass (SQ_WAVES, SQ_INSTS_VALU, ...) of one kernel into
profiles/pmc_sq_<variant>[_ring]_N<N>_E<E>.json, which bench.py reads for its VALU roofline fields.

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES \\
        SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_sq -o run --output-format csv -- python3 bench.py ...
    python tools/pmc_sq_json.py gpurun_out/pmc_sq --kernel step_kernel --out profiles/pmc_sq_....json

SQ_INSTS_VALU counts wave instructions (each issues 64 lanes: 4 cycles on a 16-lane SIMD), so
lane-ops per launch = 64 x SQ_INSTS_VALU, and the VALU issue fraction of a launch of duration t is
64 x SQ_INSTS_VALU / t / 39.3e12 (256 CU x 4 SIMD x 16 lanes x 2.4 GHz, non-packed).
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+", help="one rocprofv3 -d directory per PMC pass")
    ap.add_argument("--kernel", default="step_kernel")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # counter -> dispatch -> value
    files = [f for d in a.dirs for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)]
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if a.kernel in row.get("Kernel_Name", ""):
                    per[row["Counter_Name"]][(f, row["Dispatch_Id"])] += float(row["Counter_Value"])
    if not per:
        raise SystemExit("no counter rows found")
    out = {"kernel": a.kernel, "dispatches": max(len(v) for v in per.values())}
    for c, d in sorted(per.items()):
        out[c] = statistics.median(d.values())
    if "SQ_INSTS_VALU" in out and "SQ_WAVES" in out:
        out["valu_insts_per_wave"] = out["SQ_INSTS_VALU"] / out["SQ_WAVES"]
    out["note"] = "median per dispatch; VALU lane-ops per launch = 64 x SQ_INSTS_VALU"
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
