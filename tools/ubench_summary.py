"""Merge tools/ubench_valu's timing JSON with its PMC pass (SQ_ACTIVE_INST_VALU, SQ_ACTIVE_INST_VALU2,
GRBM_GUI_ACTIVE per opcode kernel) into profiles/ubench_valu.json.

    python tools/ubench_summary.py gpurun_out/valu/ubench_valu.json gpurun_out/valu/ubench_pmc --out profiles/ubench_valu.json

Per opcode and occupancy (8 or 1 waves per SIMD):
  cyc          cycles per wave64 instruction per SIMD from the kernel's duration at the nominal 2.4 GHz;
  dual_frac    2 x SQ_ACTIVE_INST_VALU2 / instructions: the share of the instructions issued in a quad-cycle together
               with another wave's VALU instruction (gfx950 co-issues two of the simple ops from two waves);
  act_per_inst SQ_ACTIVE_INST_VALU quad-cycles per instruction (1 for most ops, 2 for the transcendental ones);
  issue_cyc    the VALU issue cost the counters charge per instruction: 4 x (ACT - ACT2) / instructions.
The class of an opcode is 2 (co-issued at 8 waves per SIMD), 4 or 8 cycles per wave64 instruction; a saturating stream
of any class reads a busy fraction 4 x (ACT - ACT2) / (SIMDs x cycles) of 0.86-0.97, which is what makes that
quantity the measured VALU occupancy bench.py reports (roofline.valu).
"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("timing")
    ap.add_argument("pmc_dir")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    with open(a.timing) as f:
        t = json.load(f)
    iters = t["iters"]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for fn in glob.glob(os.path.join(a.pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as fh:
            for r in csv.DictReader(fh):
                d = (fn, int(r["Dispatch_Id"]))
                per[d][r["Counter_Name"]] += float(r["Counter_Value"])
                per[d]["grid"] = float(r["Grid_Size"])
                name[d] = r["Kernel_Name"].split("(")[0][2:]
    pmc = collections.defaultdict(dict)  # op -> waves -> counters of its last (warm) launch
    for d in sorted(per):
        v = per[d]
        waves = v["grid"] / 64
        insts = waves * iters * 8
        occ = "8" if waves >= 8 * 1024 else "1"
        pmc[name[d]][occ] = {
            "insts": insts, "dual_frac": 2 * v["SQ_ACTIVE_INST_VALU2"] / insts,
            "act_per_inst": v["SQ_ACTIVE_INST_VALU"] / insts,
            "issue_cyc": 4 * (v["SQ_ACTIVE_INST_VALU"] - v["SQ_ACTIVE_INST_VALU2"]) / insts}
    ops = []
    for o in t["ops"]:
        e = dict(o)
        for occ in ("8", "1"):
            p = pmc.get(o["op"], {}).get(occ)
            if p:
                e[f"dual_frac_{occ}wave{'s' if occ == '8' else ''}"] = round(p["dual_frac"], 3)
                e[f"act_per_inst_{occ}wave{'s' if occ == '8' else ''}"] = round(p["act_per_inst"], 3)
                e[f"issue_cyc_{occ}wave{'s' if occ == '8' else ''}"] = round(p["issue_cyc"], 3)
        c = e.get("issue_cyc_8waves")
        if c is not None:
            e["issue_class_cyc"] = 2 if c < 3 else 4 if c < 6 else 8
        ops.append(e)
    out = {k: v for k, v in t.items() if k != "ops"}
    out["ops"] = ops
    out["source"] = "tools/ubench_valu.hip (timing) + rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 " \
                    "GRBM_GUI_ACTIVE (tools/gpu_r3_valu.sh); merged by tools/ubench_summary.py"
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for e in ops:
        print(f"{e['op']:16s} cyc8 {e['cyc_8waves']:6.2f} class {e.get('issue_class_cyc')} dual {e.get('dual_frac_8waves')}")


if __name__ == "__main__":
    main()
