"""Break down the config-3 step: env kernel, replay insert, learn() — wall (host) vs GPU time."""
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
hook = SharedCriticBench(env, dev, fused=os.environ.get("FUSED", "1") != "0")
for s in range(5):
    env.step(a)
    hook.after_env_step(s, a)
torch.cuda.synchronize()


def timeit(name, fn, n=50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        fn(i)
    e1.record()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name:12s} host-enqueue {1e3 * (t1 - t0) / n:8.3f} ms  wall {1e3 * (t2 - t0) / n:8.3f} ms  "
          f"gpu {e0.elapsed_time(e1) / n:8.3f} ms")


L = hook.learner
n = E * N
timeit("env.step", lambda i: env.step(a))
timeit("store", lambda i: L.store_transitions(hook.prev_obs.reshape(n, -1), a.reshape(n, -1),
                                              env.reward.reshape(n, 1), env.dnn.reshape(n, -1), env.done.reshape(n)))
timeit("learn", lambda i: L.learn(i % N))
timeit("full", lambda i: (env.step(a), hook.after_env_step(i, a)))
