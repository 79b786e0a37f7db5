"""Host cost per env step of the two launch paths of VecFlockEnv: launch="plan" (C ABI + recorded launch plan, one
ctypes call) vs launch="torch" (torch.ops.flock custom ops through the dispatcher), at BASELINE configs 2 and 3 (env
step only). Host = the Python loop's enqueue time per step; wall includes the GPU draining the queue."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv

dev = torch.device("cuda", 0)
for tag, variant, N, E in (("config 2", "uw", 64, 1024), ("config 3", "v2", 256, 4096)):
    box = float(round((250 * N) ** 0.5))
    for ops in ("plan", "torch"):
        env = VecFlockEnv(FlockConfig(variant=variant, num_envs=E, num_agents=N, k=4, range_start=(0, box),
                                      sensor_range=14.0, track_indices=variant == "v2"), device=dev, launch=ops)
        env.positions.uniform_(0, box)
        a = torch.rand(E, N, 2, device=dev)
        for _ in range(20):
            env.step(a)
        torch.cuda.synchronize()
        n = 300
        t0 = time.perf_counter()
        for _ in range(n):
            env.step(a)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{tag} {variant} N={N} E={E} launch={ops:5s}: host {1e6 * (t1 - t0) / n:6.1f} us/step, "
              f"wall {1e6 * (t2 - t0) / n:6.1f} us/step", flush=True)
