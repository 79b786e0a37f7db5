"""Probe (diagnostics, not the product): the config-3 env step alone (one launch, the fused ring insert off) from a
uniform random start, timed over consecutive windows of steps: does the kernel's time depend on how many steps the
swarm has moved since the start (the bench times 20 steps after 5 warmup steps)? Also counts the envs with a
collision (done) per window.

    python tools/env_drift_probe.py [steps] [window]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv

dev = torch.device("cuda", 0)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
win = int(sys.argv[2]) if len(sys.argv) > 2 else 20
E, N, box = 4096, 256, 253.0
env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, collision_distance=2.5,
                              range_start=(0, box), sensor_range=14.0, seed=1234, step_launches=1), device=dev)
g = torch.Generator(device=dev).manual_seed(1234)
env.positions.copy_(torch.rand(E, N, 2, device=dev, generator=g) * box)
env.headings.copy_((1.0 - torch.rand(E, N, device=dev, generator=g)) * 4.71)
pool = [torch.stack([torch.rand(E, N, device=dev, generator=g),
                     torch.rand(E, N, device=dev, generator=g) * 3 - 1.5], -1).contiguous() for _ in range(8)]
torch.cuda.synchronize()
for w0 in range(0, steps, win):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for s in range(w0, w0 + win):
        env.step(pool[s % len(pool)])
    e1.record()
    torch.cuda.synchronize()
    print(f"steps {w0:4d}-{w0 + win - 1:4d}: {e0.elapsed_time(e1) / win * 1e3:6.1f} us/step, envs done "
          f"{int(env.any_done.sum())}, mean speed-step displacement {float(env.velocities.norm(dim=-1).mean()):.4f}",
          flush=True)
