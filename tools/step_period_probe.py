"""Probe (diagnostics, not the product): per-step periods of the config-3 loop right after the warmup, from HIP events
recorded around every step's env launches (ScTrainLoop events, ev_every = 1). Shows where a short timed region (the
driver's --steps 20 --warmup 5) loses time against long runs: pipeline fill, a slow start, or the drain.

    python tools/step_period_probe.py [W ...]   (default W = 5 400)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

dev = torch.device("cuda", 0)


def run(W, K=40):
    E, N, box = 4096, 256, 253.0
    env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, collision_distance=2.5,
                                  range_start=(0, box), sensor_range=14.0, seed=1234, step_launches=3), device=dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    env.positions.copy_(torch.rand(E, N, 2, device=dev, generator=g) * box)
    env.headings.copy_((1.0 - torch.rand(E, N, device=dev, generator=g)) * 4.71)
    pool = [torch.stack([torch.rand(E, N, device=dev, generator=g),
                         torch.rand(E, N, device=dev, generator=g) * 3 - 1.5], -1).contiguous() for _ in range(8)]
    hook = SharedCriticBench(env, device=dev, seed=1234)
    hook.run_steps(0, W, pool)
    hook.prime()
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * K)]
    end = torch.cuda.Event(enable_timing=True)
    stream = torch.cuda.current_stream(dev)
    for e in evs:
        e.record(stream)
    end.record(stream)
    torch.cuda.synchronize()
    hook.run_steps(W, K, pool, evs, 1)
    hook.finish()
    end.record(stream)
    torch.cuda.synchronize()
    starts = np.array([evs[0].elapsed_time(evs[2 * s]) for s in range(K)]) * 1e3
    envk = np.array([evs[2 * s].elapsed_time(evs[2 * s + 1]) for s in range(K)]) * 1e3
    total = evs[0].elapsed_time(end) * 1e3
    per = np.diff(starts)
    print(f"W={W}: region {total:.0f} us for {K} steps ({total / K:.1f} us/step); drain after the last env step "
          f"{total - starts[-1] - envk[-1]:.0f} us", flush=True)
    print("  step periods (us): " + " ".join(f"{p:.0f}" for p in per), flush=True)
    print("  env launches (us): " + " ".join(f"{p:.0f}" for p in envk), flush=True)


if __name__ == "__main__":
    for w in [int(a) for a in sys.argv[1:]] or [5, 400]:
        run(w)
