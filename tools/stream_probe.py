"""Stream placement probe (verdict r5 item 2): five consecutive SharedCriticBench instances in ONE process, each
timing the config-3 loop (ScTrainLoop, 200 steps after 20 warmup steps) on the default (env) stream. MODE=own: the
learner's rounds on the pipeline's own stream (SharedCriticLearner.learner_stream, ScPipeline.stream: one per device
and priority, made once in C++); MODE=pool: a torch pool stream per instance, as before round 6; PRIORITY=high|normal
(MODE=own). Every instance should run within a few percent of the first."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

dev = torch.device("cuda", 0)
E, N, box = 4096, 256, 253.0
mode, prio = os.environ.get("MODE", "own"), os.environ.get("PRIORITY", "high")
g = torch.Generator(device=dev).manual_seed(1)
pool = [torch.stack([torch.rand(E, N, device=dev, generator=g),
                     torch.rand(E, N, device=dev, generator=g) * 3 - 1.5], -1).contiguous() for _ in range(8)]
first = None
for inst in range(int(os.environ.get("INSTANCES", 5))):
    env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, collision_distance=2.5,
                                  range_start=(0, box), sensor_range=14.0, step_launches=3), device=dev)
    env.positions.copy_(torch.rand(E, N, 2, device=dev, generator=g) * box)
    env.headings.copy_(torch.rand(E, N, device=dev, generator=g) * 4.7)
    hook = SharedCriticBench(env, device=dev, seed=3, learner_priority=prio)
    if mode == "pool":
        hook.stream = torch.cuda.Stream(dev)
    hook.run_steps(0, 20, pool)
    hook.finish()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hook.run_steps(20, 200, pool)
    hook.finish()
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / 200
    hook.learner.pipeline_check()
    first = first or ms
    print(f"MODE={mode} PRIORITY={prio} GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', 'default')} "
          f"instance {inst}: {ms:.4f} ms per step ({ms / first:.3f} of the first)", flush=True)
    del hook, env
