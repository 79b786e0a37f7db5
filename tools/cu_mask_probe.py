"""Probe: config-3 bench step with the env stream restricted to a subset of CUs (hipExtStreamCreateWithCUMask), so
that the learner stream's small launches always find free CUs. Also the learner stream at high priority.
Prints GPU wall time per step for each arrangement (fresh env + learner per arrangement)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

dev = torch.device("cuda", 0)
hip = ctypes.CDLL("libamdhip64.so")
NCU = torch.cuda.get_device_properties(dev).multi_processor_count


def masked_stream(off_bits):
    """A stream whose kernels may use every CU except the mask bits in off_bits."""
    words = (ctypes.c_uint32 * ((NCU + 31) // 32))()
    for i in range(NCU):
        if i not in off_bits:
            words[i // 32] |= 1 << (i % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


def run(name, stream, steps=200):
    env = VecFlockEnv(FlockConfig(variant="v2", num_envs=4096, num_agents=256, k=4, range_start=(0, 253),
                                  sensor_range=14, collision_distance=2.5), device=dev)
    env.positions.uniform_(0, 253)
    a = torch.rand(4096, 256, 2, device=dev)
    torch.cuda.synchronize()
    ctx = torch.cuda.stream(stream) if stream is not None else torch.cuda.stream(torch.cuda.current_stream(dev))
    with ctx:
        hook = SharedCriticBench(env, dev)
        for s in range(30):
            hook.step(s, a)
        hook.finish()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(30, 30 + steps):
            hook.step(s, a)
        hook.finish()
        torch.cuda.synchronize()
    print(f"{name:50s} {1e6 * (time.perf_counter() - t0) / steps:8.1f} us/step", flush=True)


print(f"{NCU} CUs", flush=True)
run("default", None)
for n in (8, 16, 32):
    run(f"env without the {n} lowest CU bits", masked_stream(set(range(n))))
    run(f"env without the {n} highest CU bits", masked_stream(set(range(NCU - n, NCU))))
    run(f"env without every {NCU // n}-th CU bit", masked_stream(set(range(0, NCU, NCU // n))))
run("default again", None)
