"""Probe (diagnostics): config-3 bench loop per-step time with the learner as one graph on one stream, as two phase
graphs on two streams (pipelined), and the pipelined phases eager."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

dev = torch.device("cuda", 0)
E = 4096


def run(pipelined, graph, with_env=True, n=100):
    env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=256, k=4, range_start=(0, 253),
                                  sensor_range=14), device=dev)
    env.positions.uniform_(0, 253)
    a = torch.rand(E, 256, 2, device=dev)
    os.environ["FLOCK_LEARN_PIPELINE"] = "1" if pipelined else "0"
    hook = SharedCriticBench(env, dev, overlap=True)
    hook.learner.use_graph = graph
    for s in range(10):
        hook.step(s, a)
    hook.finish()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(10, 10 + n):
        if with_env:
            hook.step(s, a)
        else:
            hook.after(s, a)
    hook.finish()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"pipelined={int(pipelined)} graph={int(graph)} env={int(with_env)}: host {1e6 * (t1 - t0) / n:6.1f} "
          f"wall {1e6 * (t2 - t0) / n:6.1f} us/step", flush=True)


order = os.environ.get("ORDER", "pg,sg,pg,sg")
for tok in order.split(","):
    run(tok[0] == "p", tok[1] == "g", True)
