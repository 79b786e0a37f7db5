"""Per-block timeline of one shared-critic learner round (diagnostics, not the product).

    python tools/sc_block_prof.py --build     # here (CPU): libflock_amd_scprof.so with -DFLOCK_SC_PROF
    python tools/sc_block_prof.py [--corun]   # GPU box: config-3 learner rounds alone (or beside env steps)

Each of the five round kernels records, per block, its start (thread 0) and end (max over its waves) with
s_memrealtime (100 MHz). Printed for the last round: every kernel's first block start / last block end relative to
the round's first block, the launch gaps between kernels, and the block-duration percentiles per block range.
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "marl_range_flocking_amd", "_build")
SO = os.path.join(BUILD, "libflock_amd_scprof.so")
KERNELS = ["k1", "gemm", "k3", "bwd", "grad_adam"]


def build():
    sys.path.insert(0, ROOT)
    from marl_range_flocking_amd.build import CSRC, HIPCC_FLAGS, INCLUDE, hipcc

    obj = os.path.join(BUILD, "flock_sc_prof.o")
    subprocess.check_call([hipcc()] + HIPCC_FLAGS + ["-DFLOCK_SC_PROF", "-c", "-I", INCLUDE, "-o", obj,
                                                     os.path.join(CSRC, "flock_sc.hip")])
    subprocess.check_call([hipcc()] + HIPCC_FLAGS + ["-shared", "-o", SO, os.path.join(BUILD, "flock_env.hip.o"),
                                                     os.path.join(BUILD, "flock_learn.hip.o"),
                                                     os.path.join(BUILD, "flock_act.hip.o"), obj])
    print(SO)


def run(corun, learns):
    # the learner launches through libflock_torch.so, which links _build/libflock_amd.so: run with the profiling
    # build copied over it (SWAPPED=1; tools/gpu_scprof.sh)
    if os.environ.get("SWAPPED") != "1":
        raise SystemExit("run through tools/gpu_scprof.sh (the -DFLOCK_SC_PROF build copied over _build/libflock_amd.so)")
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    from marl_range_flocking_amd import FlockConfig, VecFlockEnv, _native
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

    lib = _native.lib()
    assert hasattr(lib, "flock_sc_prof_read"), "not the -DFLOCK_SC_PROF build: " + lib._name
    dev = torch.device("cuda", 0)
    E, N = 4096, 256
    env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, range_start=(0, 253),
                                  sensor_range=14, collision_distance=2.5), device=dev)
    env.positions.uniform_(0, 253)
    a = torch.rand(E, N, 2, device=dev)
    hook = SharedCriticBench(env, dev)
    L = hook.learner
    for s in range(20):
        hook.step(s, a)
    hook.finish()
    torch.cuda.synchronize()
    for s in range(learns):
        if corun:
            hook.step(s, a)
        else:
            L.replay_slots(E * N)
            hook.after(s, a)
    torch.cuda.synchronize()  # no flush: the last round is a merged (critic + actor) one
    buf = (ctypes.c_ulonglong * (5 * 4096 * 2))()
    lib.flock_sc_prof_read.argtypes = [ctypes.c_void_p]
    assert lib.flock_sc_prof_read(buf) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(5, 4096, 2).astype(np.int64)
    # the last round: per kernel, the blocks whose start lies in the last round (after the last k1 start - 1 ms)
    k1_last = t[0, :, 0].max()
    lo = k1_last - 100_000  # 1 ms at 100 MHz
    print(f"mode: {'beside env steps' if corun else 'learner alone'}; times in us from the round's first block")
    starts = t[0, :, 0][t[0, :, 0] > lo]
    base = starts.min()
    prev_end = None
    for k, name in enumerate(KERNELS):
        sel = t[k, :, 0] > lo
        s, e = t[k, sel, 0], t[k, sel, 1]
        d = (e - s) / 100.0
        first, last = (s.min() - base) / 100.0, (e.max() - base) / 100.0
        gap = f"{first - prev_end:5.1f}" if prev_end is not None else "  -  "
        print(f"{name:10s} blocks {sel.sum():5d}  first start {first:6.1f}  last end {last:6.1f}  span {last - first:5.1f}"
              f"  gap {gap}  block dur p10/p50/p90/max {np.percentile(d, 10):5.1f} {np.percentile(d, 50):5.1f} "
              f"{np.percentile(d, 90):5.1f} {d.max():5.1f}")
        prev_end = last
        idx = np.nonzero(sel)[0]
        if name == "gemm":  # phase marks of the forward GEMM blocks (gemm_tile, FLOCK_SC_PROF)
            mk = (ctypes.c_ulonglong * (4096 * 8))()
            lib.flock_sc_mark_read.argtypes = [ctypes.c_void_p]
            assert lib.flock_sc_mark_read(mk) == 0
            m = np.frombuffer(mk, dtype=np.uint64).reshape(4096, 8).astype(np.int64)[idx]
            names = ["entry", "chunk0 in LDS", "barrier", "MFMA0 done", "chunk1 in LDS", "barrier", "MFMA1 done",
                     "partials in LDS"]
            rel = (m - t[k, idx, 0][:, None]) / 100.0
            print("    gemm phase marks (us from block start, p50 / p90): " + ", ".join(
                f"{n} {np.percentile(rel[:, i], 50):.2f}/{np.percentile(rel[:, i], 90):.2f}" for i, n in enumerate(names)))
        # block-index ranges (16 equal slices): median start offset and median duration
        for q in np.array_split(np.arange(len(idx)), min(16, len(idx))):
            if len(q) == 0:
                continue
            ii = idx[q]
            print(f"    blocks {ii[0]:5d}-{ii[-1]:5d}: start p50 {(np.median(t[k, ii, 0]) - base) / 100.0:6.1f}  "
                  f"dur p50 {np.median((t[k, ii, 1] - t[k, ii, 0]) / 100.0):5.1f}  max {((t[k, ii, 1] - t[k, ii, 0]) / 100.0).max():5.1f}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--corun", action="store_true")
    ap.add_argument("--learns", type=int, default=40)
    args = ap.parse_args()
    build() if args.build else run(args.corun, args.learns)
