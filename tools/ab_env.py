"""A/B timing of env-step library builds (diagnostics): each .so is loaded with ctypes and its flock_step_v2 /
flock_step_uw_discrete timed with HIP events on the same resident state, interleaved rounds, median per launch.

    python tools/ab_env.py lib_a.so lib_b.so [--shapes 4096x256,2048x1024,1024x512]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--shapes", default="4096x256,2048x1024,1024x512")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variant", default="v2", choices=["v2", "uwd"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    libs = []
    for path in a.libs:
        lib = ctypes.CDLL(os.path.abspath(path))
        f = lib.flock_step_v2
        f.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 3 + [ctypes.c_float] * 6 + [ctypes.c_int] * 2 + \
            [ctypes.c_void_p] * 9
        g = lib.flock_step_uw_discrete
        g.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 3 + [ctypes.c_float] * 5 + [ctypes.c_int] + \
            [ctypes.c_void_p] * 5 + [ctypes.c_float, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                     ctypes.c_int] + [ctypes.c_void_p] * 7
        libs.append((path, f, g))
    for shape in a.shapes.split(","):
        E, N = map(int, shape.split("x"))
        k = 4
        box = float(round(np.sqrt(250.0 * N)))
        gen = torch.Generator(device=dev).manual_seed(0)
        pos0 = torch.rand(E, N, 2, device=dev, generator=gen) * box
        head0 = torch.rand(E, N, device=dev, generator=gen) * 4.71
        act = torch.stack([torch.rand(E, N, device=dev, generator=gen),
                           torch.rand(E, N, device=dev, generator=gen) * 3 - 1.5], -1).contiguous()
        aid = torch.randint(0, 10, (E, N), device=dev, generator=gen)
        table = torch.rand(10, 2, device=dev, generator=gen)
        outs = {}
        times = {p: [] for p, _, _ in libs}
        for r in range(a.rounds):
            for path, f, g in libs:
                pos, head = pos0.clone(), head0.clone()
                prev = torch.zeros(E, N, device=dev)
                vel = torch.empty(E, N, 2, device=dev)
                dnn = torch.empty(E, N, k, device=dev)
                idx = torch.empty(E, N, k, dtype=torch.int64, device=dev)
                rew = torch.empty(E, N, device=dev)
                done = torch.empty(E, N, dtype=torch.uint8, device=dev)
                anyd = torch.empty(E, dtype=torch.uint8, device=dev)

                def step():
                    if a.variant == "v2":
                        rc = f(stream, E, N, k, box, 14.0, 2.5, 0.1, 0.0, 2.5, 1, 0, pos.data_ptr(),
                               head.data_ptr(), act.data_ptr(), vel.data_ptr(), dnn.data_ptr(), idx.data_ptr(),
                               rew.data_ptr(), done.data_ptr(), anyd.data_ptr())
                    else:
                        rc = g(stream, E, N, k, box, 14.0, 2.5, 0.1, 2.5, 0, pos.data_ptr(), head.data_ptr(),
                               prev.data_ptr(), aid.data_ptr(), None, 0.1, 7, 0, table.data_ptr(), 10,
                               vel.data_ptr(), dnn.data_ptr(), idx.data_ptr(), rew.data_ptr(), done.data_ptr(),
                               anyd.data_ptr(), None)
                    assert rc == 0, rc

                for _ in range(3):
                    step()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    step()
                e1.record()
                torch.cuda.synchronize()
                times[path].append(e0.elapsed_time(e1) / a.iters * 1e3)
                if r == 0:
                    outs[path] = (pos.cpu(), idx.cpu(), dnn.cpu())
        ref = outs[libs[0][0]]
        for path, _, _ in libs:
            o = outs[path]
            same = all(torch.equal(x, y) for x, y in zip(o, ref))
            print(f"{a.variant} E={E} N={N}: {os.path.basename(path):32s} median {np.median(times[path]):7.1f} us "
                  f"(min {min(times[path]):.1f})  outputs {'==' if same else '!='} first lib", flush=True)


if __name__ == "__main__":
    main()
