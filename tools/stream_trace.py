"""Per-kernel-name and per-stream summary of a rocprofv3 --kernel-trace CSV, plus one window of the timeline
(diagnostics). Usage: python tools/stream_trace.py TRACE.csv [window_start_index=200] [window_len=40]"""
import collections
import csv
import sys


def short(name):
    for key in ("step_kernel", "sc_prep_snapshot", "sc_k1", "sc_gemm", "sc_k3", "sc_bwd", "sc_grad_adam", "ncclDevKernel",
                "ncclKernel", "rccl", "adam", "sleep"):
        if key.lower() in name.lower():
            return key
    return name[:40]


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"],
                         r["Stream_Id"]))
    rows.sort()
    by = collections.defaultdict(list)
    for s, e, k, q, st in rows:
        by[(k, q, st)].append(e - s)
    print("kernel / queue / stream: calls, mean us")
    for (k, q, st), d in sorted(by.items(), key=lambda x: -sum(x[1])):
        print(f"  {k:20s} q{q:>3s} s{st:>3s} {len(d):5d} {sum(d) / len(d) / 1e3:9.2f}")
    w0 = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    wl = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    t0 = rows[w0][0]
    print(f"timeline from kernel {w0} (us, start-end, queue, stream)")
    for s, e, k, q, st in rows[w0:w0 + wl]:
        print(f"  {(s - t0) / 1e3:9.2f} {(e - t0) / 1e3:9.2f}  q{q:>3s} s{st:>3s} {k}")


if __name__ == "__main__":
    main()
