"""Multi-process (world_size 2, 4 and 8, gloo, CPU) tests of the env-shard and data-parallel learner plumbing: the
global env split of configs 4 / 5 (8192 / 16384 envs over W ranks), the gradient all-reduce, the replica sync and the
max-over-ranks timing of bench.py."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from marl_range_flocking_amd import dist


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    try:
        w, r, dev = dist.init("gloo")
        assert (w, r) == (world, rank) and dev.type == "cpu"
        # env sharding: contiguous, balanced, covering
        first, count = dist.env_shard(4099, world, rank)
        spans = [None] * world
        torch.distributed.all_gather_object(spans, (first, count))
        # gradient all-reduce: mean of per-rank buffers (exact: small integers, a power-of-two world)
        g = torch.full((1000,), float(rank + 1))
        dist.allreduce_mean_(g)
        # parameter sync from rank 0 (FlatParams on CPU: only the HIP update kernels need a GPU)
        from marl_range_flocking_amd.learners.core import FlatParams

        fp = FlatParams({"w": (3, 4), "b": (3,)}, "cpu", agents=5, target=True)
        fp.data.fill_(float(rank) + 0.5)
        fp.target.fill_(float(rank) - 0.5)
        dist.sync_params(fp)
        m = dist.max_over_ranks(rank * 10.0, torch.device("cpu"))
        q.put((rank, spans, g[0].item(), g.sum().item(), fp.data.unique().tolist(), fp.target.unique().tolist(), m))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, "error", repr(e)))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_shard_allreduce_sync(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for o in out:
        assert o[1] != "error", o
    mean = (world + 1) / 2.0
    for rank, spans, g0, gsum, data_u, targ_u, m in out:
        assert sum(c for _, c in spans) == 4099
        assert spans[0][0] == 0 and all(spans[i + 1][0] == spans[i][0] + spans[i][1] for i in range(world - 1))
        assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
        assert g0 == mean and gsum == 1000 * mean
        assert data_u == [0.5] and targ_u == [-0.5]
        assert m == 10.0 * (world - 1)


def test_env_shard_single_process():
    assert dist.env_shard(10, 1, 0) == (0, 10)
    assert [dist.env_shard(10, 3, r) for r in range(3)] == [(0, 4), (4, 3), (7, 3)]
    assert not dist.active()
    t = torch.ones(3)
    assert dist.allreduce_mean_(t) is t and t.sum().item() == 3
