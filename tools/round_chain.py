"""Which stream bounds the config-3 step (rocprofv3 --kernel-trace CSV of the gated loop): per learner round, the
critic k1's effective start = max(previous round's grad end, its snapshot's end), then the five kernel spans; counts
the rounds whose start was set by the snapshot (env stream) vs the previous round (learner chain).
Usage: python tools/round_chain.py TRACE.csv"""
import csv
import statistics as st
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r.get("Kernel_Name") or ""
    for k in ("sc_prep_snapshot", "sc_k1", "sc_gemm", "sc_k3", "sc_bwd", "sc_grad_adam", "step_kernel"):
        if k in n:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
            break
rows.sort()
snaps = [r for r in rows if r[2] == "sc_prep_snapshot"]
rounds = []
cur = None
for s, e, k in rows:
    if k == "sc_k1":
        cur = {"k1": (s, e)}
    elif cur is not None and k in ("sc_gemm", "sc_k3", "sc_bwd", "sc_grad_adam"):
        cur[k] = (s, e)
        if k == "sc_grad_adam":
            rounds.append(cur)
            cur = None
env_bound = chain_bound = 0
spans = {k: [] for k in ("wait", "k1", "gemm", "k3", "bwd", "grad", "total", "period")}
prev_end = None
prev_start = None
for i, r in enumerate(rounds[5:-5], 5):
    k1s, k1e = r["k1"]
    snap_end = max((e for s, e, _ in snaps if e <= k1e), default=k1s)
    start = max(snap_end, prev_end if prev_end else k1s)
    if prev_end is not None:
        if snap_end > prev_end:
            env_bound += 1
        else:
            chain_bound += 1
    spans["wait"].append((start - (prev_end or start)) / 1e3)
    spans["k1"].append((k1e - start) / 1e3)
    spans["gemm"].append((r["sc_gemm"][1] - k1e) / 1e3)
    spans["k3"].append((r["sc_k3"][1] - r["sc_gemm"][1]) / 1e3)
    spans["bwd"].append((r["sc_bwd"][1] - r["sc_k3"][1]) / 1e3)
    spans["grad"].append((r["sc_grad_adam"][1] - r["sc_bwd"][1]) / 1e3)
    spans["total"].append((r["sc_grad_adam"][1] - start) / 1e3)
    if prev_start is not None:
        spans["period"].append((start - prev_start) / 1e3)
    prev_end = r["sc_grad_adam"][1]
    prev_start = start
print(f"rounds {len(rounds)}: start set by the snapshot (env stream) {env_bound}, by the previous round {chain_bound}")
for k, v in spans.items():
    if v:
        q = sorted(v)
        print(f"  {k:7s} p10 {q[len(q) // 10]:6.1f}  p50 {st.median(v):6.1f}  p90 {q[9 * len(q) // 10]:6.1f} us")
