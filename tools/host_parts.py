"""Host time of the pieces of one config-3 bench step (no GPU sync inside the loop; the GPU drains behind)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

dev = torch.device("cuda", 0)
E = 4096
env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=256, k=4, range_start=(0, 253), sensor_range=14),
                  device=dev)
env.positions.uniform_(0, 253)
a = torch.rand(E, 256, 2, device=dev)
hook = SharedCriticBench(env, dev, overlap=True)
for s in range(10):
    hook.step(s, a)
hook.finish()
torch.cuda.synchronize()
tb = te = ta = 0.0
n = 200
for s in range(10, 10 + n):
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
    if s % 50 == 0:
        torch.cuda.synchronize()
print(f"before {1e6 * tb / n:.1f} us, env.step(ring) {1e6 * te / n:.1f} us, after (snapshot + 2 phases) "
      f"{1e6 * ta / n:.1f} us")
L = hook.learner
slot = 0
import cProfile, pstats
pr = cProfile.Profile()
pr.enable()
for s in range(10 + n, 10 + 2 * n):
    hook.step(s, a)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
