"""Host-side cost of one config-3 bench step (env step with the fused replay insert, then learn()) against its GPU
time: if the host enqueue per step approaches the GPU time, the GPU idles between launches."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

dev = torch.device("cuda", 0)
E, N = int(os.environ.get("E", 4096)), int(os.environ.get("N", 256))
env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, range_start=(0, 253), sensor_range=14),
                  device=dev)
env.positions.uniform_(0, 253)
a = torch.rand(E, N, 2, device=dev)
hook = SharedCriticBench(env, dev)
L = hook.learner
for s in range(30):
    hook.step(s, a)
torch.cuda.synchronize()


def host(name, fn, n=200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name:14s} host {1e6 * (t1 - t0) / n:8.1f} us/call   wall {1e6 * (t2 - t0) / n:8.1f} us/call")


def after_only(i):
    L.replay_slots(E * N)
    hook.after(i, a)


host("replay_slots", lambda i: L.replay_slots(E * N))
host("env.step+ring", lambda i: env.step(a, ring=L.replay_slots(E * N)))
host("hook.after", after_only)
hook.finish()
host("bench step", lambda i: hook.step(i, a))
hook.finish()
