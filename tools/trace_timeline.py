"""Per-step timeline of the config-3 loop from a rocprofv3 --kernel-trace CSV (diagnostics).

For every env step (the step_kernel launches) and every learner round (its first kernel: sc_gate_kernel, sc_k1 or
sc_fwd, .. its last: sc_grad_adam or sc_bwdg) prints the start / end
relative to the first step, and summarises: the step period, the env launches' span, the round's span, the gap
between the snapshot and the round's first kernel, the gaps between the round's kernels, and which stream set the
period (did the env stream start its next step right after its previous one, or later).
Usage: python tools/trace_timeline.py TRACE.csv|RESULTS.db (rocprofv3's csv kernel trace or its sqlite database)"""
import csv
import sqlite3
import statistics as st
import sys


def load(path):
    rows = []
    if path.endswith(".db"):
        q = ("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
             "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
        rows = [(a, b, n) for n, a, b in sqlite3.connect(path).execute(q)]
        rows.sort()
        return rows
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    return rows


def short(name):
    # the fused rounds' kernels (sc_fwd, sc_bwdg) are checked before the prefixes they contain
    for key in ("step_kernel", "sc_prep_snapshot", "sc_gate_kernel", "sc_k1", "sc_fwd", "sc_bwdg", "sc_gemm", "sc_k3",
                "sc_bwd", "sc_grad_adam"):
        if key in name:
            return key
    return None


def main():
    rows = [(s, e, short(n)) for s, e, n in load(sys.argv[1])]
    rows = [r for r in rows if r[2]]
    # group: an env step = consecutive step_kernel launches followed by a snapshot; a round = k1..grad_adam
    env_steps, cur = [], []
    for s, e, k in rows:
        if k == "step_kernel":
            cur.append((s, e))
        elif k == "sc_prep_snapshot" and cur:
            env_steps.append((cur, (s, e)))
            cur = []
    rounds, rc, order = [], {}, None
    for s, e, k in rows:
        if k.startswith("sc_") and k != "sc_prep_snapshot":
            rc.setdefault("_order", []).append(k)
            rc[k] = (s, e)
            if k in ("sc_grad_adam", "sc_bwdg"):
                order = order or rc["_order"]
                rc["_first"] = rc[rc["_order"][0]]
                rounds.append(rc)
                rc = {}
    n = min(len(env_steps), len(rounds))
    skip = max(0, n - 60)  # the last 60 steps (the timed region sits at the end of a short bench)
    t0 = env_steps[skip][0][0][0]
    per, env_span, rnd_span, snap_gap, env_idle, between = [], [], [], [], [], []
    prev_end = None
    kgaps = {k: [] for k in order[1:]}
    kdur = {k: [] for k in order}
    for i in range(skip, n - 1):
        launches, snap = env_steps[i]
        nxt = env_steps[i + 1][0][0][0]
        per.append((nxt - launches[0][0]) / 1e3)
        env_span.append((launches[-1][1] - launches[0][0]) / 1e3)
        env_idle.append((nxt - snap[1]) / 1e3)
        # the round that consumes this step's snapshot starts after it
        r = next((rr for rr in rounds if rr["_first"][1] >= snap[1]), None)
        if r is None:
            continue
        if any(k not in r for k in order):
            continue
        snap_gap.append((r["_first"][1] - snap[1]) / 1e3)
        pr = rounds[rounds.index(r) - 1] if rounds.index(r) > 0 else None
        if pr is not None:
            between.append((r["_first"][0] - pr[order[-1]][1]) / 1e3)
        rnd_span.append((r[order[-1]][1] - r["_first"][0]) / 1e3)
        for a, b in zip(order, order[1:]):
            kgaps[b].append((r[b][0] - r[a][1]) / 1e3)
        for k in order:
            kdur[k].append((r[k][1] - r[k][0]) / 1e3)
        if i - skip < 12:
            ls = " ".join("%7.1f-%7.1f" % ((s - t0) / 1e3, (e - t0) / 1e3) for s, e in launches)
            print("step %3d env %s snap %7.1f-%7.1f | round %7.1f-%7.1f" % (
                i - skip, ls, (snap[0] - t0) / 1e3, (snap[1] - t0) / 1e3, (r["_first"][0] - t0) / 1e3,
                (r[order[-1]][1] - t0) / 1e3))

    def m(v):
        return "%.1f (p10 %.1f p90 %.1f)" % (st.mean(v), sorted(v)[len(v) // 10], sorted(v)[9 * len(v) // 10])

    print("steps analysed", len(per))
    print("step period us            ", m(per))
    print("env launches span us      ", m(env_span))
    print("env stream idle after snap", m(env_idle))
    print("round order               ", " ".join(order))
    print("snapshot end -> 1st k end ", m(snap_gap))
    print("round span us             ", m(rnd_span))
    if between:
        print("previous round end -> 1st k start", m(between))
    for k, v in kdur.items():
        print("  %-13s dur %s" % (k, m(v)))
    for k, v in kgaps.items():
        print("  gap before %-13s %s" % (k, m(v)))


if __name__ == "__main__":
    main()
