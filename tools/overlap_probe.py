"""Timing probe for the config-3 bench loop (diagnostics): serial vs overlapped learner, with and without HIP
graphs. Prints ms per step for each mode."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

dev = torch.device("cuda", 0)
E, N = 4096, 256
for overlap, graph in ((False, True), (True, True), (True, False), (False, False)):
    env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, range_start=(0, 253),
                                  sensor_range=14), device=dev)
    env.positions.uniform_(0, 253)
    a = torch.rand(E, N, 2, device=dev)
    hook = SharedCriticBench(env, dev, overlap=overlap)
    hook.learner.use_graph = graph
    for s in range(20):
        hook.step(s, a)
    hook.finish()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 100
    for s in range(20, 20 + n):
        hook.step(s, a)
    t1 = time.perf_counter()
    hook.finish()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"overlap={overlap} graph={graph}: {1e3 * (t2 - t0) / n:.4f} ms/step (host {1e3 * (t1 - t0) / n:.4f})",
          flush=True)
