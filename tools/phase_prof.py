"""Per-phase cycle breakdown of the env step kernel (diagnostics, not the product).

    python tools/phase_prof.py --build            # here (CPU): hipcc flock_env.hip -DFLOCK_PHASE_PROF
    python tools/phase_prof.py [--E 4096 --N 256]  # GPU box: run steps, print mean cycles per wave per phase

Every wave's lane 0 adds s_memtime deltas between phase marks of step_kernel into device counters (see the
PHASE() marks in flock_env.hip); counts: waves taking the 5x5 scan, the full scan, an ambiguous-bucket rescan.
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.environ.get("FLOCK_PROF_SO") or os.path.join(ROOT, "marl_range_flocking_amd", "_build", "libflock_env_prof.so")
NAMES = ["kinematics", "phase2 barrier", "cell binning", "3x3 scan", "5x5 scan", "finalize/fallback",
         "outputs", "any_done barrier"]


def build():
    from marl_range_flocking_amd.build import CSRC, FILE_FLAGS, HIPCC_FLAGS, INCLUDE, hipcc

    os.makedirs(os.path.dirname(SO), exist_ok=True)
    b = os.path.dirname(SO)
    obj = os.path.join(b, "flock_env_phase.o")
    cmd = [hipcc()] + HIPCC_FLAGS + FILE_FLAGS["flock_env.hip"] + ["-DFLOCK_PHASE_PROF", "-c", "-I", INCLUDE, "-o", obj,
                                                                 os.path.join(CSRC, "flock_env.hip")]
    print(" ".join(cmd))
    subprocess.check_call(cmd)
    # linked with the product's learner objects (flock_env.hip calls into flock_sc.hip for the diagnostics knob)
    subprocess.check_call([hipcc()] + HIPCC_FLAGS + ["-shared", "-o", SO, obj, os.path.join(b, "flock_learn.hip.o"),
                                                     os.path.join(b, "flock_sc.hip.o")])


def run(E, N, k, steps, variant="v2", seeds=False, windows=0):
    import numpy as np
    import torch

    lib = ctypes.CDLL(SO)
    lib.flock_phase_read.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    box = float(round(np.sqrt(250.0 * N)))
    g = torch.Generator(device=dev).manual_seed(0)
    pos = torch.rand(E, N, 2, device=dev, generator=g) * box
    head = torch.rand(E, N, device=dev, generator=g) * 4.71
    act = torch.stack([torch.rand(E, N, device=dev, generator=g),
                       torch.rand(E, N, device=dev, generator=g) * 3 - 1.5], -1).contiguous()
    vel = torch.empty(E, N, 2, device=dev)
    dnn = torch.empty(E, N, k, device=dev)
    idx = torch.empty(E, N, k, dtype=torch.int64, device=dev)
    rew = torch.empty(E, N, device=dev)
    done = torch.empty(E, N, dtype=torch.uint8, device=dev)
    anyd = torch.empty(E, dtype=torch.uint8, device=dev)
    f = lib.flock_step_v2
    f.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 3 + [ctypes.c_float] * 6 + [ctypes.c_int] * 2 + \
        [ctypes.c_void_p] * 9
    stream = torch.cuda.current_stream(dev).cuda_stream
    ext = None
    if seeds:  # the compact seed buffer, as VecFlockEnv passes it (v2, uwd)
        from marl_range_flocking_amd._native import FlockStepExt

        sb = torch.zeros(E, N, k, dtype=torch.int16, device=dev)
        ext = FlockStepExt(ring=None, seeds=sb.data_ptr(), launches=1, normalize_distance=0)
        fe = lib.flock_step_v2_ext
        fe.argtypes = f.argtypes + [ctypes.c_void_p]
    gd = lib.flock_step_uw_discrete
    gd.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 3 + [ctypes.c_float] * 5 + [ctypes.c_int] + \
        [ctypes.c_void_p] * 5 + [ctypes.c_float, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int] + \
        [ctypes.c_void_p] * 7
    gde = lib.flock_step_uw_discrete_ext
    gde.argtypes = gd.argtypes + [ctypes.c_void_p]
    gu = lib.flock_step_uw
    gu.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 3 + [ctypes.c_float] * 4 + [ctypes.c_int] + \
        [ctypes.c_void_p] * 12
    mem = torch.zeros(E, N, 4, k, device=dev)
    aid = torch.randint(0, 10, (E, N), device=dev, generator=g)
    table = torch.rand(10, 2, device=dev, generator=g)
    prev = torch.zeros(E, N, device=dev)

    def step():
        if variant == "v2" and ext is not None:
            rc = fe(stream, E, N, k, box, 14.0, 2.5, 0.1, 0.0, 2.5, 1, 0, pos.data_ptr(), head.data_ptr(),
                    act.data_ptr(), vel.data_ptr(), dnn.data_ptr(), idx.data_ptr(), rew.data_ptr(), done.data_ptr(),
                    anyd.data_ptr(), ctypes.addressof(ext))
        elif variant == "v2":
            rc = f(stream, E, N, k, box, 14.0, 2.5, 0.1, 0.0, 2.5, 1, 0, pos.data_ptr(), head.data_ptr(),
                   act.data_ptr(), vel.data_ptr(), dnn.data_ptr(), idx.data_ptr(), rew.data_ptr(), done.data_ptr(),
                   anyd.data_ptr())
        elif variant == "uw":
            rc = gu(stream, E, N, k, box, 14.0, 2.5, 0.1, 0, pos.data_ptr(), head.data_ptr(), prev.data_ptr(),
                    act.data_ptr(), mem.data_ptr(), mem.data_ptr(), vel.data_ptr(), dnn.data_ptr(), idx.data_ptr(),
                    rew.data_ptr(), done.data_ptr(), anyd.data_ptr())
        elif ext is not None:
            rc = gde(stream, E, N, k, box, 14.0, 2.5, 0.1, 2.5, 0, pos.data_ptr(), head.data_ptr(), prev.data_ptr(),
                     aid.data_ptr(), None, 0.1, 7, 0, table.data_ptr(), 10, vel.data_ptr(), dnn.data_ptr(),
                     idx.data_ptr(), rew.data_ptr(), done.data_ptr(), anyd.data_ptr(), None, ctypes.addressof(ext))
        else:
            rc = gd(stream, E, N, k, box, 14.0, 2.5, 0.1, 2.5, 0, pos.data_ptr(), head.data_ptr(), prev.data_ptr(),
                    aid.data_ptr(), None, 0.1, 7, 0, table.data_ptr(), 10, vel.data_ptr(), dnn.data_ptr(),
                    idx.data_ptr(), rew.data_ptr(), done.data_ptr(), anyd.data_ptr(), None)
        assert rc == 0, rc

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 32)()
    lib.flock_phase_read(buf)
    for w in range(windows):  # drift probe: kernel time and in-kernel clock per window of `steps` steps
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            step()
        e1.record()
        torch.cuda.synchronize()
        lib.flock_phase_read(buf)
        waves = buf[20]
        print(f"window {w:3d}: {e0.elapsed_time(e1) / steps * 1e3:6.1f} us/launch, clock "
              f"{buf[19] / max(buf[23], 1) * 0.1:.2f} GHz, wave lifetime {buf[23] / waves * 0.01:.2f} us, "
              f"kinematics {buf[0] / waves:.0f} scan {buf[3] / waves:.0f} binning {buf[2] / waves:.0f} cycles/wave, "
              f"rescan {buf[18] / waves:.5f}", flush=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        step()
    e1.record()
    torch.cuda.synchronize()
    lib.flock_phase_read(buf)
    waves = buf[20]
    tot = sum(buf[i] for i in range(8)) + buf[9] + buf[10] + buf[11]
    print(f"E={E} N={N} k={k}: kernel {e0.elapsed_time(e1) / steps * 1e3:.1f} us/launch, waves/launch "
          f"{waves / steps:.0f}")
    for i, n in enumerate(NAMES):
        print(f"  {n:20s} {buf[i] / waves:9.0f} cycles/wave  {100.0 * buf[i] / tot:5.1f} %")
    if buf[9]:  # v2: phase 0 split at the kinematics inputs' arrival, the stores, the late loads
        print(f"    (of the kinematics: inputs arrived after {buf[9] / waves:.0f} cycles/wave, arithmetic + stores "
              f"{buf[10] / waves:.0f}, late loads issued {buf[11] / waves:.0f}, pull issued {buf[0] / waves:.0f})")
    print(f"  waves taking 5x5: {buf[16] / waves:.4f}, full scan: {buf[17] / waves:.5f}, "
          f"ambiguous rescan: {buf[18] / waves:.5f}")
    print(f"  cell-scan pair iterations per wave: {buf[21] / waves:.1f} over {buf[22] / waves:.2f} row ranges")
    bb = (ctypes.c_ulonglong * (4096 * 2))()
    lib.flock_blk_read.argtypes = [ctypes.c_void_p]
    if lib.flock_blk_read(bb) == 0:
        t = np.frombuffer(bb, dtype=np.uint64).reshape(4096, 2).astype(np.int64)
        phb = (ctypes.c_ulonglong * (4096 * 8))()
        lib.flock_blkph_read.argtypes = [ctypes.c_void_p]
        lib.flock_blkph_read(phb)
        ph = np.frombuffer(phb, dtype=np.uint64).reshape(4096, 8).astype(np.int64)
        keep = t[:, 0] > t[:, 0].max() - 100_000  # the last launch's blocks (started within 1 ms of its last one)
        t, ph = t[keep], ph[keep]
        nb = len(t)
        t0 = t[:, 0].min()
        st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0
        span = en.max()
        grid = np.linspace(0, span, 60)
        conc = [int(((st <= g) & (en > g)).sum()) for g in grid]
        print(f"  last launch, {nb} blocks (of the first 4096): span {span:.1f} us, block lifetime p10/p50/p90 "
              f"{np.percentile(en - st, 10):.1f}/{np.percentile(en - st, 50):.1f}/{np.percentile(en - st, 90):.1f} us; "
              f"start p10/p50/p90 {np.percentile(st, 10):.1f}/{np.percentile(st, 50):.1f}/{np.percentile(st, 90):.1f}")
        print("  resident blocks over the launch (60 samples): " + " ".join(str(c) for c in conc))
        late = np.argsort(en)[-3:]
        ids = np.nonzero(keep)[0]
        print("  last blocks to end: " + ", ".join(f"block {ids[j]} start {st[j]:.1f} end {en[j]:.1f} us" for j in late))
        # thread 0's phase marks (us after its block's start): median block vs the three latest blocks
        rel = (ph - t[:, :1]) / 100.0
        print("  thread-0 phase marks, median block: " + " ".join(f"{np.median(rel[:, q]):.1f}" for q in range(8)))
        for j in late:
            print("  thread-0 phase marks, late block:   " + " ".join(f"{rel[j, q]:.1f}" for q in range(8)))
    print(f"  in-kernel clock (shader cycles / s_memrealtime x 100 MHz over the waves' lifetimes): "
          f"{buf[19] / max(buf[23], 1) * 0.1:.2f} GHz; mean wave lifetime {buf[23] / waves * 0.01:.2f} us")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--E", type=int, default=4096)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--variant", default="v2", choices=["v2", "uw", "uwd"])
    ap.add_argument("--seeds", action="store_true", help="v2 / uwd through the _ext entry with a seed buffer")
    ap.add_argument("--windows", type=int, default=0, help="first time this many windows of --steps steps (drift)")
    a = ap.parse_args()
    if a.build:
        build()
    else:
        run(a.E, a.N, a.k, a.steps, a.variant, a.seeds, a.windows)
