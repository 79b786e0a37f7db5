"""Host cost of the data-parallel config-3 loop's collectives over RCCL, on ONE GPU (diagnostics, not a scaling number).

    python tools/rccl_host_cost.py        # GPU box: one rank, backend "nccl", cuda:0

The config-3 bench loop (256 agents x 4096 envs, ScTrainLoop) with the learner forced onto its data-parallel path
(SharedCriticLearner(dp=True)): every round's all-reduces are ProcessGroupNCCL calls from C++ over a one-rank
communicator (ProcessGroupNCCL calls, or direct RCCL calls: ScPipeline.set_rccl). Printed per variant: the step time over 100 steps and the host's
enqueue time per step with the GPU held by a sleep kernel (as bench.py's host_enqueue_us_per_step), i.e. what the
host adds per step at N > 1 before the GPU is the bound.
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29531"), WORLD_SIZE="1",
                      RANK="0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.distributed.init_process_group("nccl", device_id=dev)
    from marl_range_flocking_amd import FlockConfig, VecFlockEnv
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

    E, N = 4096, 256
    g = torch.Generator(device=dev).manual_seed(1)
    pool = [torch.stack([torch.rand(E, N, device=dev, generator=g),
                         torch.rand(E, N, device=dev, generator=g) * 3 - 1.5], -1).contiguous() for _ in range(8)]
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None  # a variant name prefix
    if "--side-stream" in sys.argv:  # the env work on a non-blocking stream instead of the legacy default stream
        torch.cuda.set_stream(torch.cuda.Stream(dev))
    for name, kw in (("single GPU", dict(dp=False)),
                     ("DP unsplit, c10d", dict(dp=True, dp_split=False, dp_rccl=False)),
                     ("DP unsplit, RCCL", dict(dp=True, dp_split=False, dp_rccl=True)),
                     ("DP split, c10d", dict(dp=True, dp_split=True, dp_rccl=False)),
                     ("DP split, RCCL", dict(dp=True, dp_split=True, dp_rccl=True)),
                     ("single GPU", dict(dp=False))):
        if only and not name.startswith(only):
            continue
        env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, collision_distance=2.5,
                                      range_start=(0, 253.0), sensor_range=14.0, step_launches=3), device=dev)
        env.positions.copy_(torch.rand(E, N, 2, device=dev, generator=g) * 253.0)
        env.headings.copy_(torch.rand(E, N, device=dev, generator=g) * 4.7)
        hook = SharedCriticBench(env, device=dev, seed=3, **kw)
        assert hook.can_loop() and hook.learner.distributed == kw["dp"]
        hook.run_steps(0, 20, pool)
        hook.finish()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hook.run_steps(20, 100, pool)
        hook.finish()
        torch.cuda.synchronize()
        step_ms = (time.perf_counter() - t0) / 100 * 1e3
        torch.cuda._sleep(int(2.4e9 * 0.05))  # hold the GPU while the host enqueues (as bench.py: well under the gate's bound)
        t1 = time.perf_counter()
        hook.run_steps(120, 32, pool)
        host_us = (time.perf_counter() - t1) / 32 * 1e6
        hook.finish()
        torch.cuda.synchronize()
        if hook.learner.__dict__.get("_pipe") is not None:
            hook.learner.pipeline_check()
        print(f"{name:17s}: {step_ms:.4f} ms per step (100 steps), host enqueue {host_us:.1f} us per step", flush=True)
        del hook, env
        torch.cuda.empty_cache()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
