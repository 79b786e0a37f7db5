"""Probe (diagnostics, not the product): the config-3 step with the GPU partitioned between the two streams
(hipExtStreamCreateWithCUMask; KEEP spread CU bits for the learner stream, the rest for the env stream). For each
split: the env step alone (3 launches + insert), the learner alone (snapshot + one round per step) and the C++ loop
with both, GPU wall time per step. Masked streams are made ONCE per split (every masked stream is a hardware queue of
its own; making new ones per run oversubscribes the queues, round-5 / round-6 "random 3x outliers")."""
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
E, N, box = 4096, 256, 253.0


def masked_stream(on_bits):
    words = (ctypes.c_uint32 * ((NCU + 31) // 32))()
    for i in on_bits:
        words[i // 32] |= 1 << (i % 32)
    s = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), words) == 0
    return torch.cuda.ExternalStream(s.value, device=dev)


def spread(keep):
    return [i for i in range(NCU) if (i * keep) // NCU != ((i + 1) * keep) // NCU]


env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, collision_distance=2.5,
                              range_start=(0, box), sensor_range=14.0, seed=1234, step_launches=3), device=dev)
g = torch.Generator(device=dev).manual_seed(1234)
env.positions.copy_(torch.rand(E, N, 2, device=dev, generator=g) * box)
env.headings.copy_((1.0 - torch.rand(E, N, device=dev, generator=g)) * 4.71)
pool = [torch.stack([torch.rand(E, N, device=dev, generator=g),
                     torch.rand(E, N, device=dev, generator=g) * 3 - 1.5], -1).contiguous() for _ in range(8)]
hook = SharedCriticBench(env, device=dev, seed=1234)
L = hook.learner
own = hook.stream
torch.cuda.synchronize()
with torch.cuda.stream(torch.cuda.Stream(dev)):
    hook.run_steps(0, 30, pool)
    hook.finish()
torch.cuda.synchronize()
step = [30]


def timed(fn, n=200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(n)
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / n


def run_split(name, ls, es):
    hook.stream = ls

    def both(n):
        with torch.cuda.stream(es):
            hook.run_steps(step[0], n, pool)
            hook.finish()
        step[0] += n

    def env_alone(n):
        with torch.cuda.stream(es):
            for i in range(n):
                env.step(pool[i % 8], ring=L.replay_slots(E * N))

    def learner_alone(n):
        # snapshot + round per call on the learner stream, no env step between (the ring is not rewritten)
        with torch.cuda.stream(es):
            for i in range(n):
                L.replay_slots(E * N)
                L.pipeline_mark(es.cuda_stream)
                hook.after(step[0] + i, pool[0])
            hook.finish()
        step[0] += n

    hook._handles = None
    both(20)
    r = [timed(both), timed(env_alone), timed(learner_alone), timed(both)]
    L.pipeline_check()
    print(f"{name:40s} both {r[0]:7.1f} / {r[3]:7.1f}  env alone {r[1]:7.1f}  learner alone {r[2]:7.1f} us/step",
          flush=True)


if __name__ == "__main__":
    print(f"{NCU} CUs", flush=True)
    keeps = [int(x) for x in os.environ.get("KEEP", "32,48,64").split(",")]
    arr = [("own learner stream, torch env stream", own, torch.cuda.Stream(dev))]
    for keep in keeps:
        lb = spread(keep)
        arr.append((f"learner {keep} spread CUs, env the rest", masked_stream(lb),
                    masked_stream([i for i in range(NCU) if i not in set(lb)])))
    for rep in range(int(os.environ.get("REPS", 2))):
        for name, ls, es in arr:
            run_split(name, ls, es)
