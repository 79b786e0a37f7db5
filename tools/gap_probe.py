"""Probe (diagnostics): time per learn() update replayed back to back on one stream, (a) alone, (b) each preceded
by a wait on an already-complete event recorded on another stream, (c) plus an event record after each."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

dev = torch.device("cuda", 0)
env = VecFlockEnv(FlockConfig(variant="v2", num_envs=64, num_agents=256, k=4, range_start=(0, 253),
                              sensor_range=14), device=dev)
a = torch.rand(64, 256, 2, device=dev)
hook = SharedCriticBench(env, dev, overlap=True)
for s in range(8):
    hook.step(s, a)
hook.finish()
torch.cuda.synchronize()
L = hook.learner
other = torch.cuda.Stream(device=dev)
ev_other = torch.cuda.Event()
ev_other.record(other)
done = torch.cuda.Event()
n = 50
for mode in ("plain", "wait", "wait+record", "plain"):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(hook.stream):
        for i in range(n):
            if mode != "plain":
                hook.stream.wait_event(ev_other)
            L.update_slot(0, i % 256)
            if mode == "wait+record":
                done.record(hook.stream)
    torch.cuda.synchronize()
    print(f"{mode:12s} {1e6 * (time.perf_counter() - t0) / n:.1f} us per update", flush=True)
