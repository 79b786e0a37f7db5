"""Probe (diagnostics, not the product): the config-3 loop with the LEARNER stream or the ENV stream restricted to a
subset of CUs (hipExtStreamCreateWithCUMask): a learner confined to fewer CUs (MODE=learner), or CUs kept free of env
blocks so that the learner's latency-bound round always finds room (MODE=env). Prints GPU wall time per step
(ScTrainLoop, 200 steps after 20 warmup steps) for each arrangement, interleaved."""
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


def masked_stream(on_bits):
    """A stream whose kernels may use only the CUs whose mask bits are in on_bits."""
    words = (ctypes.c_uint32 * ((NCU + 31) // 32))()
    for i in on_bits:
        words[i // 32] |= 1 << (i % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


def run(name, on_bits, steps=200, env_bits=None):
    E, N, box = 4096, 256, 253.0
    env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, collision_distance=2.5,
                                  range_start=(0, box), sensor_range=14.0, seed=1234, step_launches=3), device=dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    env.positions.copy_(torch.rand(E, N, 2, device=dev, generator=g) * box)
    env.headings.copy_((1.0 - torch.rand(E, N, device=dev, generator=g)) * 4.71)
    pool = [torch.stack([torch.rand(E, N, device=dev, generator=g),
                         torch.rand(E, N, device=dev, generator=g) * 3 - 1.5], -1).contiguous() for _ in range(8)]
    hook = SharedCriticBench(env, device=dev, seed=1234)
    if on_bits is not None:
        hook.stream = masked_stream(on_bits)
    torch.cuda.synchronize()
    es = masked_stream(env_bits) if env_bits is not None else torch.cuda.current_stream(dev)
    with torch.cuda.stream(es):
        hook.run_steps(0, 20, pool)
        hook.finish()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hook.run_steps(20, steps, pool)
        hook.finish()
        torch.cuda.synchronize()
    us = 1e6 * (time.perf_counter() - t0) / steps
    hook.learner.pipeline_check()
    print(f"{name:44s} {us:8.1f} us/step", flush=True)
    return us


if __name__ == "__main__":
    print(f"{NCU} CUs", flush=True)
    spread = lambda keep: [i for i in range(NCU) if (i * keep) // NCU != ((i + 1) * keep) // NCU]  # noqa: E731
    arr = [("default", None, None)]
    if os.environ.get("MODE", "learner") == "learner":
        for keep in (192, 128, 64):
            arr.append((f"learner on the lowest {keep} CU bits", list(range(keep)), None))
            arr.append((f"learner on {keep} CU bits spread", spread(keep), None))
    elif os.environ.get("MODE") == "split":
        arr.append(("both on all CU bits (masked streams)", list(range(NCU)), list(range(NCU))))
        for keep in [int(x) for x in os.environ.get("KEEP", "32,64,96,128").split(",")]:
            lb = list(range(keep))
            arr.append((f"learner lowest {keep} bits, env the rest", lb, [i for i in range(NCU) if i not in set(lb)]))
            lb = spread(keep)
            arr.append((f"learner {keep} spread bits, env the rest", lb, [i for i in range(NCU) if i not in set(lb)]))
    else:
        arr.append(("env on all CU bits (masked stream)", None, list(range(NCU))))
        for off in (8, 16, 32, 64):
            arr.append((f"env without the lowest {off} CU bits", None, list(range(off, NCU))))
            arr.append((f"env without {off} spread CU bits", None, [i for i in range(NCU) if i not in set(spread(off))]))
    for r in range(int(os.environ.get("REPS", 2))):
        for name, lb, eb in arr:
            run(name, lb, env_bits=eb)
