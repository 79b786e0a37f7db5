"""Overlap probe (diagnostics): the config-3 loop with the env step on a CU-masked stream (all CUs but R) and the
learner on a normal or high-priority stream. Prints ms per step per setting."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

hip = ctypes.CDLL("libamdhip64.so")
dev = torch.device("cuda", 0)
torch.cuda.init()
lo, hi = ctypes.c_int(), ctypes.c_int()
hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi))
print("hip priority range", lo.value, hi.value, "torch", torch.cuda.Stream.priority_range(), flush=True)
ncu = torch.cuda.get_device_properties(0).multi_processor_count
print("CUs", ncu, flush=True)


def masked_stream(reserve):
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in range(ncu):
        if c >= reserve:
            mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


def prio_stream(p):
    s = ctypes.c_void_p()
    rc = hip.hipStreamCreateWithPriority(ctypes.byref(s), 0, ctypes.c_int(p))
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


E, N = 4096, 256
for reserve, prio in ((0, None), (0, hi.value), (16, None), (32, None), (32, hi.value), (64, None)):
    env_stream = masked_stream(reserve) if reserve else torch.cuda.current_stream(dev)
    with torch.cuda.stream(env_stream):
        env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, range_start=(0, 253),
                                      sensor_range=14), device=dev)
        env.positions.uniform_(0, 253)
        a = torch.rand(E, N, 2, device=dev)
        hook = SharedCriticBench(env, dev, overlap=True)
        if prio is not None:
            hook.stream = prio_stream(prio)
        for s in range(20):
            hook.step(s, a)
        hook.finish()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        n = 100
        kt = []
        for s in range(20, 20 + n):
            e0.record(env_stream)
            env.step(a, ring=hook.before(s))
            e1.record(env_stream)
            hook.after(s, a)
            if s == 60:
                torch.cuda.synchronize()
                kt.append(e0.elapsed_time(e1))
        hook.finish()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    print(f"reserve={reserve:3d} prio={prio}: {1e3 * (t2 - t0) / n:.4f} ms/step, one env step {kt[0] * 1e3:.1f} us",
          flush=True)
