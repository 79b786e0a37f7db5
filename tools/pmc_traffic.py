"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_<variant>_N<N>_E<E>.json.

Usage (on the GPU box, two separate passes as MI355X_MICROARCH.md §rocprofv3 prescribes — TCC cannot hold both):
    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py ...
    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --kernel step_kernel --out profiles/...

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming
read, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 is exact for streaming stores. Both raw values are
kept in the JSON.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def counter_values(d, counter, kernel):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == counter and kernel in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--kernel", default="step_kernel")
    ap.add_argument("--out", required=True)
    ap.add_argument("--algorithmic-bytes", type=float, default=None)
    ap.add_argument("--steps-per-launch", type=int, default=None, help="rollout launches: env steps per launch")
    a = ap.parse_args()
    fetch = counter_values(a.fetch_dir, "FETCH_SIZE", a.kernel)
    write = counter_values(a.write_dir, "WRITE_SIZE", a.kernel)
    if not fetch or not write:
        raise SystemExit(f"no counter rows found (fetch {len(fetch)}, write {len(write)})")
    f_kb, w_kb = statistics.median(fetch), statistics.median(write)
    read_b, write_b = 2.0 * f_kb * 1024, w_kb * 1024
    out = {"kernel": a.kernel, "dispatches": [len(fetch), len(write)],
           "FETCH_SIZE_kb_median": f_kb, "WRITE_SIZE_kb_median": w_kb,
           "read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
           "hbm_bytes_per_launch": read_b + write_b,
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count, MI355X_MICROARCH.md §HBM); "
                         "write = WRITE_SIZE x 1024"}
    if a.steps_per_launch:
        out["steps_per_launch"] = a.steps_per_launch
    if a.algorithmic_bytes:
        out["algorithmic_bytes_per_launch"] = a.algorithmic_bytes
        out["traffic_over_algorithmic"] = (read_b + write_b) / a.algorithmic_bytes
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
