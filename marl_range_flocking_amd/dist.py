"""One process per GPU: env sharding and the learners' data-parallel gradient all-reduce.

* Env instances are independent, so ``env_shard`` splits them across ranks with no data-path collective
  (SURVEY.md §8(e)); each rank steps, stores and samples only its own envs.
* Learner replicas stay identical: parameters are broadcast from rank 0 once, and each update all-reduces the
  learner's flat gradient buffer (ONE collective per update over one contiguous bucket — the flat layout of
  learners/core.FlatParams makes the whole learner a single RCCL all-reduce over xGMI), then every rank applies
  the same Adam step. Backend "nccl" is RCCL on ROCm; "gloo" runs the same code on CPU (tests).
"""
import os

import torch
import torch.distributed as dist


def world_info():
    """(world_size, rank, local_rank) from the torchrun environment (1, 0, 0 when not launched distributed)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend="nccl"):
    """Initialise the default process group from the environment; returns (world, rank, device)."""
    world, rank, local = world_info()
    if backend == "nccl":
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return world, rank, dev


def active(group=None):
    return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1


def env_shard(total_envs, world, rank):
    """Contiguous, balanced split of ``total_envs`` envs: (first_env, count) of this rank."""
    base, rem = divmod(total_envs, world)
    count = base + (1 if rank < rem else 0)
    first = rank * base + min(rank, rem)
    return first, count


def allreduce_mean_(t, group=None):
    """In-place mean over ranks (no-op on one rank)."""
    if active(group):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(dist.get_world_size(group))
    return t


def allreduce_sum_(t, group=None):
    """In-place sum over ranks (no-op on one rank); the caller folds 1 / world into its consumer (the Adam
    kernels' device-side grad_scale), one elementwise launch fewer than allreduce_mean_."""
    if active(group):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def broadcast_(t, src=0, group=None):
    if active(group):
        dist.broadcast(t, src=src, group=group)
    return t


def max_over_ranks(x, device, group=None):
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    if active(group):
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def sync_params(flat_params, src=0, group=None):
    """Broadcast every state buffer of a FlatParams (params, target, moments) from ``src``."""
    for t in flat_params.state_tensors():
        broadcast_(t, src, group)
