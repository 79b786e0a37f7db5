"""Config-3 step parts alone vs together (GPU wall time per call): the env step with the fused replay insert alone,
the learner (snapshot + one merged round per learn) alone, and the bench step (both, overlapped on two streams)."""
import os
import sys
import time

# FLOCK_TREE: run against another source tree (an _ab/<sha> export, tools/gpu_ab_trees.sh)
sys.path.insert(0, os.environ.get("FLOCK_TREE") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

dev = torch.device("cuda", 0)
E, N = int(os.environ.get("E", 4096)), int(os.environ.get("N", 256))
env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, range_start=(0, 253), sensor_range=14,
                              collision_distance=2.5), device=dev)
env.positions.uniform_(0, 253)
a = torch.rand(E, N, 2, device=dev)
hook = SharedCriticBench(env, dev)
L = hook.learner
for s in range(20):
    hook.step(s, a)
hook.finish()
torch.cuda.synchronize()


def wall(name, fn, n=200):
    for i in range(10):
        fn(i)
    hook.finish()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    hook.finish()
    torch.cuda.synchronize()
    print(f"{name:34s} {1e6 * (time.perf_counter() - t0) / n:8.1f} us/call", flush=True)


def learn_only(i):
    L.replay_slots(E * N)
    hook.after(i, a)


wall("env step + ring insert alone", lambda i: env.step(a, ring=L.replay_slots(E * N)))
wall("learner alone (snapshot + round)", learn_only)
wall("bench step (both)", lambda i: hook.step(i, a))
