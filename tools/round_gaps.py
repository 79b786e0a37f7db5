"""The learner stream's gap before each round's first kernel (sc_k1 start - previous sc_grad_adam end), in order,
from a rocprofv3 kernel trace (csv or .db): which rounds pay it (diagnostics). Usage: python tools/round_gaps.py TRACE"""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_timeline import load  # noqa: E402


def main():
    rows = [(s, e, n) for s, e, n in load(sys.argv[1]) if "sc_k1" in n or "sc_grad_adam" in n]
    gaps, last = [], None
    for s, e, n in rows:
        if "sc_grad_adam" in n:
            last = e
        elif last is not None:
            gaps.append((s - last) / 1e3)
            last = None
    gaps = gaps[-60:]
    print("gap before each round's k1 (us), last %d rounds:" % len(gaps))
    print(" ".join("%.1f" % g for g in gaps))
    small = sum(g < 3.0 for g in gaps)
    print("rounds with a gap < 3 us: %d of %d" % (small, len(gaps)))


if __name__ == "__main__":
    main()
