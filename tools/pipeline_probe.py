"""Probe (diagnostics, results not used): learn() throughput when the actor phase of learn t runs on a second stream
beside the critic phase of learn t+1 (flock_sc_critic_update / flock_sc_actor_update as separate eager calls).
Modes: serial (one stream), pipe (actor(t) on stream 2 after critic(t); critic(t+1) does NOT wait: upper bound,
data races ignored), and the same two beside the config-3 env step loop."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv, _native
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench
from marl_range_flocking_amd.learners.core import _stream

dev = torch.device("cuda", 0)
E = int(os.environ.get("E", 4096))
env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=256, k=4, range_start=(0, 253),
                              sensor_range=14), device=dev)
env.positions.uniform_(0, 253)
a = torch.rand(E, 256, 2, device=dev)
hook = SharedCriticBench(env, dev, overlap=True)
for s in range(8):
    hook.step(s, a)
hook.finish()
torch.cuda.synchronize()
L = hook.learner
lib = _native.lib()
Sc, Sa = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
n = 100
evc = [torch.cuda.Event() for _ in range(n)]
eva = [torch.cuda.Event() for _ in range(n)]


def crit(i):
    u = ctypes.byref(L._slots[i & 1]["sc"])
    lib.flock_sc_critic_update(_stream(dev), u)


def act(i):
    u = ctypes.byref(L._slots[i & 1]["sc"])
    lib.flock_sc_actor_update(_stream(dev), u)


def run(mode, with_env):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        if with_env:
            env.step(a, ring=hook.before(i))
            ev = torch.cuda.Event()
            ev.record()
        with torch.cuda.stream(Sc):
            if with_env:
                Sc.wait_event(ev)
            if mode == "serial" and i:
                Sc.wait_event(eva[i - 1])
            crit(i)
            evc[i].record(Sc)
        with torch.cuda.stream(Sa if mode == "pipe" else Sc):
            torch.cuda.current_stream().wait_event(evc[i])
            act(i)
            eva[i].record()
    torch.cuda.synchronize()
    print(f"{mode:7s} env={int(with_env)}: {1e6 * (time.perf_counter() - t0) / n:7.1f} us per learn", flush=True)


for with_env in (False, True):
    for mode in ("serial", "pipe", "serial", "pipe"):
        run(mode, with_env)
