"""Host enqueue times vs GPU start times of the env step in the overlapped config-3 loop (diagnostics): is the
step period set by the host or by the GPU?"""
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
for s in range(30):
    hook.step(s, a)
hook.finish()
torch.cuda.synchronize()
n = 40
ev = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
base = torch.cuda.Event(enable_timing=True)
base.record()
t0 = time.perf_counter()
host = []
parts = []
for s in range(30, 30 + n):
    h0 = time.perf_counter()
    ring = hook.before(s)
    ev[s - 30].record()
    env.step(a, ring=ring)
    h1 = time.perf_counter()
    hook.after(s, a)
    h2 = time.perf_counter()
    host.append(h0 - t0)
    parts.append((h1 - h0, h2 - h1))
hook.finish()
torch.cuda.synchronize()
for i in range(n):
    print(f"step {i:2d}: host enqueue at {1e6 * host[i]:9.1f} us (env {1e6 * parts[i][0]:6.1f} after "
          f"{1e6 * parts[i][1]:6.1f}), GPU start {1e3 * base.elapsed_time(ev[i]):9.1f} us")
