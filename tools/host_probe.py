"""Probe (diagnostics): host-side cost of each part of the overlapped config-3 bench step (no syncs inside)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

dev = torch.device("cuda", 0)
E, N = 4096, 256
env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, range_start=(0, 253), sensor_range=14),
                  device=dev)
env.positions.uniform_(0, 253)
a = torch.rand(E, N, 2, device=dev)
hook = SharedCriticBench(env, dev, overlap=True)
for s in range(20):
    hook.step(s, a)
hook.finish()
torch.cuda.synchronize()
n = 200
tb = te = ta = 0.0
t_start = time.perf_counter()
for s in range(20, 20 + n):
    t0 = time.perf_counter()
    ring = hook.before(s)
    t1 = time.perf_counter()
    env.step(a, ring=ring)
    t2 = time.perf_counter()
    hook.after(s, a)
    t3 = time.perf_counter()
    tb += t1 - t0
    te += t2 - t1
    ta += t3 - t2
t_host = time.perf_counter() - t_start
hook.finish()
torch.cuda.synchronize()
t_all = time.perf_counter() - t_start
print(f"host per step: before {1e6 * tb / n:.1f} us, env.step {1e6 * te / n:.1f} us, after {1e6 * ta / n:.1f} us; "
      f"host loop {1e6 * t_host / n:.1f} us/step, with GPU drain {1e6 * t_all / n:.1f} us/step", flush=True)
