"""Data-parallel learner correctness on the GPU: W = 2, 4 or 8 ranks (gloo, all on cuda:0) each sample B rows,
all-reduce the flat gradient buckets and step; the result must equal ONE process updating on the union batch of W B
rows (the all-reduced mean of per-rank mean losses is the mean loss of the union; equal up to the summation order of
the row reductions, so within the tolerances below), and every replica must stay identical (bitwise).
Covers the three learners' distributed paths (MADDPG critic-only bucket, VDN whole-QNet bucket with the clip norm
taken after the all-reduce, shared critic's two buckets around the critic step)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, K, B, C, T = 3, 4, 8, 10, 60


def _make(kind, batch, group=None):
    if kind == "maddpg":
        from marl_range_flocking_amd.learners.maddpg import MADDPGLearner

        return MADDPGLearner(N, K, recurrent=True, hidden1=32, hidden2=24, batch_size=batch, chunk_size=C,
                             buffer_capacity=128, min_size_buffer=batch, device="cuda:0", seed=0, dist_group=group,
                             reference_action_layout=False)  # the reference's raw reshape mixes rows in a batch
    if kind == "vdn":
        from marl_range_flocking_amd.learners.vdn import VDNLearner

        return VDNLearner(N, K, 4, batch_size=batch, chunk_size=C, update_iter=1, device="cuda:0", seed=0,
                          dist_group=group)
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner

    return SharedCriticLearner(N, K, fc1=32, fc2=24, batch_size=batch, buffer_size=256, device="cuda:0", seed=0,
                               dist_group=group)


def _fill(kind, L):
    rng = np.random.default_rng(0)
    obs = rng.uniform(0, 14, (T + 1, N, K)).astype(np.float32)
    for t in range(T):
        a = rng.uniform(-1, 1, (N, 2)).astype(np.float32)
        r = rng.choice([-5.0, 0.01], (N,)).astype(np.float32)
        d = (rng.uniform(size=N) < 0.1).astype(np.float32)
        if kind == "maddpg":
            L.add_record(obs[t], obs[t + 1], a, obs[t], obs[t + 1], r, d)
        elif kind == "vdn":
            L.put(obs[t], rng.integers(0, 4, N), r, obs[t + 1], [int(d.max())])
        else:
            L.store_transitions(torch.tensor(obs[t]), torch.tensor(a), torch.tensor(r), torch.tensor(obs[t + 1]),
                                torch.tensor(d))


def _starts(kind):
    """The union batch's 2B draws; rank r of W takes rows [r 2B / W, (r + 1) 2B / W)."""
    hi = {"maddpg": T - C, "vdn": T - C, "sc": T * N}[kind]
    return np.random.default_rng(5).choice(hi, 2 * B, replace=False)


def _update(kind, L, st):
    if kind == "maddpg":
        L.train(starts=st)
    elif kind == "vdn":
        L.train(starts=[st])
    else:
        L.learn(0, idx=st)


def _state(kind, L):
    if kind == "maddpg":
        return L.critics.data.cpu().numpy(), L.critics.target.cpu().numpy()
    if kind == "vdn":
        return L.q.P.data.cpu().numpy(), L.q.P.data.cpu().numpy()
    return L.critic.data.cpu().numpy(), L.actors.data.cpu().numpy()


def _worker(kind, rank, port, q, world=2):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    try:
        torch.distributed.init_process_group("gloo")
        b = 2 * B // world
        L = _make(kind, b, torch.distributed.group.WORLD)
        _fill(kind, L)
        _update(kind, L, _starts(kind)[rank * b:(rank + 1) * b])
        q.put((rank,) + _state(kind, L))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, "error", traceback.format_exc() + repr(e)))


def _spawn(target, world, *args):
    """world ranks of target(rank, port, q, *args) (gloo on cuda:0); their results, sorted by rank."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=target, args=(r, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=300) for _ in range(world)], key=lambda o: o[0])
    for p in ps:
        p.join(timeout=60)
    for o in out:
        assert not isinstance(o[1], str), o
    return out


def _kind_worker(rank, port, q, kind, world):
    _worker(kind, rank, port, q, world)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("kind", ["maddpg", "vdn", "sc"])
def test_ranks_equal_union_batch(kind, world, cuda):
    out = _spawn(_kind_worker, world, kind, world)
    for o in out[1:]:  # replicas identical
        np.testing.assert_array_equal(out[0][1], o[1])
        np.testing.assert_array_equal(out[0][2], o[2])
    L = _make(kind, 2 * B)
    _fill(kind, L)
    _update(kind, L, _starts(kind))
    ref = _state(kind, L)
    for got, want in zip(out[0][1:], ref):
        err = np.abs(got - want)
        # Adam's first step is +-lr for every element with |g| >> eps; elements whose union-batch gradient is
        # ~0 may flip sign between the two summation orders and move by 2 lr: allow a small fraction of those
        bad = err > 1e-6 + 1e-4 * np.abs(want)
        assert bad.mean() < 0.01, (kind, int(bad.sum()), float(err.max()))


def _bench_worker(rank, port, q):
    """Both config-3 loops (serial, overlapped) on 2 data-parallel ranks (gloo, cuda:0): the overlapped one, whose
    update and its two all-reduces run on the learner stream, must end bitwise equal to the serial one."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2", RANK=str(rank))
    try:
        torch.distributed.init_process_group("gloo")
        from marl_range_flocking_amd import FlockConfig, VecFlockEnv
        from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

        dev = torch.device("cuda", 0)
        E, Na = 32, 16
        states = []
        for overlap in (False, True):
            env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=Na, k=4, collision_distance=2.5,
                                          range_start=(0, 63.0), sensor_range=14.0), device=dev)
            g = torch.Generator(device=dev).manual_seed(3 + rank)
            env.positions.copy_(torch.rand(E, Na, 2, device=dev, generator=g) * 63.0)
            env.headings.copy_(torch.rand(E, Na, device=dev, generator=g) * 4.7)
            hook = SharedCriticBench(env, device=dev, seed=11, overlap=overlap)
            assert hook.overlap == overlap and hook.learner.distributed
            ga = torch.Generator(device=dev).manual_seed(7 + rank)
            for s in range(6):
                a = torch.stack([torch.rand(E, Na, device=dev, generator=ga),
                                 torch.rand(E, Na, device=dev, generator=ga) * 3 - 1.5], -1).contiguous()
                ring = hook.before(s)
                env.step(a, ring=ring)
                hook.after(s, a)
            hook.finish()
            torch.cuda.synchronize()
            L = hook.learner
            states.append([L.critic.data.cpu().numpy(), L.actors.data.cpu().numpy(), L.losses.cpu().numpy()])
        q.put((rank, states))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, "error", traceback.format_exc() + repr(e)))


def test_two_ranks_overlapped_bench_loop_equals_serial(cuda):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_bench_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=300) for _ in range(2)], key=lambda o: o[0])
    for p in ps:
        p.join(timeout=60)
    for o in out:
        assert not isinstance(o[1], str), o
    for rank, (serial, overlapped) in out:
        for x, y in zip(serial, overlapped):
            np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(out[0][1][1][0], out[1][1][1][0])  # replicas identical


def _loop_worker(rank, port, q, world=2):
    """The data-parallel config-3 loop through the C++ ScTrainLoop (each round: gradients, the all-reduce over the
    c10d ProcessGroup enqueued from C++, the Adam launch) against the per-step Python data-parallel rounds
    (SharedCriticBench(pipelined=False): SharedCriticLearner.dp_learn) on `world` ranks (gloo, cuda:0), with the actor
    half of every round split off the learner chain (dp_split: the actor all-reduce over a second group and the actor
    Adam on the pipeline's actor stream) and without (one [critic | actor] all-reduce): all three bitwise equal."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    try:
        torch.distributed.init_process_group("gloo")
        from marl_range_flocking_amd import FlockConfig, VecFlockEnv
        from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

        dev = torch.device("cuda", 0)
        E, Na, S = 24, 16, 7
        ga = torch.Generator(device=dev).manual_seed(7 + rank)
        pool = [torch.stack([torch.rand(E, Na, device=dev, generator=ga),
                             torch.rand(E, Na, device=dev, generator=ga) * 3 - 1.5], -1).contiguous()
                for _ in range(3)]
        states = []
        # 8 ranks sharing the one GPU: the unsplit loop only (the split rounds' extra comm / actor streams put 8
        # processes' hardware queues well past what the GPU maps at once; one such run faulted)
        modes = ("python", "loop_split", "loop") if world <= 4 else ("python", "loop")
        for mode in modes:
            env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=Na, k=4, collision_distance=2.5,
                                          range_start=(0, 63.0), sensor_range=14.0, step_launches=3), device=dev)
            g = torch.Generator(device=dev).manual_seed(3 + rank)
            env.positions.copy_(torch.rand(E, Na, 2, device=dev, generator=g) * 63.0)
            env.headings.copy_(torch.rand(E, Na, device=dev, generator=g) * 4.7)
            hook = SharedCriticBench(env, device=dev, seed=11, dp_split=mode == "loop_split",
                                     pipelined=mode != "python")
            assert hook.learner.distributed and hook.learner.dp_split == (mode == "loop_split")
            if mode == "python":
                assert not hook.can_loop()
                for s in range(S):
                    hook.step(s, pool[s % len(pool)])
            else:
                assert hook.can_loop()
                hook.run_steps(0, 4, pool)
                hook.run_steps(4, S - 4, pool)
            hook.finish()
            torch.cuda.synchronize()
            L = hook.learner
            C, A = L.critic, L.actors
            states.append([t.cpu().numpy() for t in (C.data, C.exp_avg, C.exp_avg_sq, C.step_dev, A.data, A.target,
                                                     A.exp_avg, A.exp_avg_sq, L.actor_steps, L.losses,
                                                     env.positions, env.dnn)]
                          + [L.replay.counter, L._learn_calls])
        q.put((rank, states))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, "error", traceback.format_exc() + repr(e)))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ranks_dp_train_loop_equals_python_dp_rounds(world, cuda):
    """bench.py --gpus W's data-parallel config-3 loop (ScTrainLoop + the pipeline's all-reduces) at 2, 4 and 8 ranks:
    bitwise the per-step Python data-parallel rounds (the same all-reduce calls), and every learner replica identical
    (the split rounds at 2 and 4 ranks).
    The split rounds all-reduce the critic gradient in two calls of other sizes: a ring all-reduce's summation order
    per element follows its chunking, so beyond 2 ranks (where a + b == b + a) they agree to rounding."""
    out = _spawn(_loop_worker, world, world)
    for rank, states in out:
        py, loop = states[0], states[-1]
        pairs = ((states[1], "split loop"), (loop, "loop")) if len(states) == 3 else ((loop, "loop"),)
        for other, name in pairs:
            for i, (x, y) in enumerate(zip(py, other)):
                if name == "split loop" and world > 2 and np.asarray(x).dtype == np.float32:
                    np.testing.assert_allclose(y, x, rtol=1e-4, atol=1e-6, err_msg=f"rank {rank} {name} field {i}")
                else:
                    np.testing.assert_array_equal(x, y, err_msg=f"rank {rank} {name} field {i}")
    for o in out[1:]:
        for i in range(9):  # the learner replicas stay identical (env state differs per rank)
            np.testing.assert_array_equal(out[0][1][1][i], o[1][1][i])


def _rccl_worker(port, q):
    """The data-parallel C++ loops over RCCL itself: one rank, backend "nccl" on cuda:0, the learner forced onto its
    data-parallel path (SharedCriticLearner(dp=True)), so every round's critic all-reduces (the early fc2-onward
    part on the comm stream, the fc1 part on the learner stream) and the split actor all-reduce (second process group,
    the pipeline's actor stream) are ProcessGroupNCCL collectives enqueued from C++ on those streams. Against the
    per-step Python data-parallel rounds: bitwise equal (a one-rank sum is the identity; the grad scale is 1)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0")
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        torch.distributed.init_process_group("nccl", device_id=dev)
        from marl_range_flocking_amd import FlockConfig, VecFlockEnv
        from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

        E, Na, S = 24, 16, 7
        ga = torch.Generator(device=dev).manual_seed(7)
        pool = [torch.stack([torch.rand(E, Na, device=dev, generator=ga),
                             torch.rand(E, Na, device=dev, generator=ga) * 3 - 1.5], -1).contiguous()
                for _ in range(3)]
        states = []
        for mode in ("python", "loop_split", "loop"):
            env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=Na, k=4, collision_distance=2.5,
                                          range_start=(0, 63.0), sensor_range=14.0, step_launches=3), device=dev)
            g = torch.Generator(device=dev).manual_seed(3)
            env.positions.copy_(torch.rand(E, Na, 2, device=dev, generator=g) * 63.0)
            env.headings.copy_(torch.rand(E, Na, device=dev, generator=g) * 4.7)
            hook = SharedCriticBench(env, device=dev, seed=11, dp_split=mode == "loop_split", dp=True,
                                     pipelined=mode != "python")
            assert hook.learner.distributed and hook.learner.dp_split == (mode == "loop_split")
            if mode == "python":
                for s in range(S):
                    hook.step(s, pool[s % len(pool)])
            else:
                assert hook.can_loop()
                hook.run_steps(0, 4, pool)
                hook.run_steps(4, S - 4, pool)
            hook.finish()
            torch.cuda.synchronize()
            L = hook.learner
            C, A = L.critic, L.actors
            states.append([t.cpu().numpy() for t in (C.data, C.exp_avg, C.exp_avg_sq, C.step_dev, A.data, A.target,
                                                     A.exp_avg, A.exp_avg_sq, L.actor_steps, L.losses,
                                                     env.positions, env.dnn)]
                          + [L.replay.counter, L._learn_calls])
        q.put(states)
        torch.distributed.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put(traceback.format_exc() + repr(e))


def test_one_rank_rccl_dp_train_loop_equals_python_dp_rounds(cuda):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(port, q))
    p.start()
    out = q.get(timeout=300)
    p.join(timeout=60)
    assert not isinstance(out, str), out
    py, split, loop = out
    for other, name in ((split, "split loop"), (loop, "loop")):
        for i, (x, y) in enumerate(zip(py, other)):
            np.testing.assert_array_equal(x, y, err_msg=f"{name} field {i}")


NS = 8  # agents of the sharded test (divisible by the world size)


def _shard_make(batch, group=None, shard=False, layout=False):
    from marl_range_flocking_amd.learners.maddpg import MADDPGLearner

    return MADDPGLearner(NS, K, recurrent=True, hidden1=32, hidden2=24, batch_size=batch, chunk_size=C,
                         buffer_capacity=128, min_size_buffer=batch, device="cuda:0", seed=0, dist_group=group,
                         reference_action_layout=layout, agent_shard=shard)


def _shard_fill(L):
    rng = np.random.default_rng(1)
    obs = rng.uniform(0, 14, (T + 1, NS, K)).astype(np.float32)
    for t in range(T):
        a = rng.uniform(-1, 1, (NS, 2)).astype(np.float32)
        r = rng.choice([-5.0, 0.01], (NS,)).astype(np.float32)
        d = (rng.uniform(size=NS) < 0.1).astype(np.float32)
        L.add_record(obs[t], obs[t + 1], a, obs[t], obs[t + 1], r, d)


def _layers(fp, buf, lo, hi):
    return np.concatenate([fp.view(buf, n)[lo:hi].detach().cpu().numpy().ravel() for n in fp.shapes])


def _shard_worker(rank, port, q, layout, world=2):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    try:
        torch.distributed.init_process_group("gloo")
        b = 2 * B // world
        L = _shard_make(b, torch.distributed.group.WORLD, shard=True, layout=layout)
        assert L.shard and L.na == NS // world and L.a0 == rank * (NS // world)
        _shard_fill(L)
        st = np.random.default_rng(5).choice(T - C, 2 * B, replace=False)
        for s2 in (st, st[::-1].copy()):
            L.train(starts=s2[rank * b:(rank + 1) * b])
        A = L.actors
        other = (L.a0 + L.na) % NS  # an agent of the other rank: its critic and target actor live there
        for net, tgt in (("critic", False), ("critic", True), ("actor", True)):
            try:
                L.state_dict(net, other, target=tgt)
                raise AssertionError(f"{net} target={tgt} of agent {other} exported by rank {rank}")
            except KeyError:
                pass
        L.state_dict("actor", other)  # the frozen actors are whole on every rank
        # checkpoint writers (SuperAgent.save): exactly one rank writes each file
        writes = {(net, i, tg) for net in ("actor", "critic") for i in range(NS) for tg in (False, True)
                  if L.writes(net, i, tg)}
        assert all(L.owns(net, i, tg) for net, i, tg in writes)
        q.put((rank, _layers(L.critics, L.critics.data, 0, L.na), _layers(L.critics, L.critics.target, 0, L.na),
               _layers(A, A.target, L.a0, L.a0 + L.na), _layers(A, A.data, 0, NS), L.losses.cpu().numpy(),
               L.state_dict("critic", L.a0)["fc2.weight"].numpy(), writes))
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, "error", traceback.format_exc() + repr(e)))


def _shard_spawn_worker(rank, port, q, layout, world):
    _shard_worker(rank, port, q, layout, world)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("layout", [False, True], ids=["plain_actions", "reference_action_layout"])
def test_agent_sharded_critics_equal_union_batch(layout, world, cuda):
    """MADDPGLearner(agent_shard=True) on W = 2, 4, 8 ranks (config 5's critics at 8 GPUs): each rank owns the critics
    and target actors of NS / W agents, all-gathers every rank's minibatch and the actor heads' actions, and updates only
    its agents. After two train() calls each rank's critics, critic targets and target actors equal that slice of ONE
    process training every agent on the union batch (same tolerance as the data-parallel test); the frozen actors
    stay bitwise whole. With the reference's action layout (MADDPG.py:86's raw reshape, bench.py's config-5 default)
    the layout is applied to the union batch, as the single process applies it to its batch. Another rank's critics
    and target actors are not exported (KeyError)."""
    out = _spawn(_shard_spawn_worker, world, layout, world)
    ref = _shard_make(2 * B, layout=layout)
    _shard_fill(ref)
    st = np.random.default_rng(5).choice(T - C, 2 * B, replace=False)
    for s2 in (st, st[::-1].copy()):
        ref.train(starts=s2)
    h = NS // world
    writers = [o[7] for o in out]  # every (net, agent, target) file has exactly one writer
    assert sum(len(w) for w in writers) == 2 * 2 * NS and len(set().union(*writers)) == 2 * 2 * NS
    for rank, crit, ctgt, atgt, actors, losses, fc2, _ in out:
        lo, hi = rank * h, (rank + 1) * h
        for got, want in ((crit, _layers(ref.critics, ref.critics.data, lo, hi)),
                          (ctgt, _layers(ref.critics, ref.critics.target, lo, hi)),
                          (atgt, _layers(ref.actors, ref.actors.target, lo, hi))):
            err = np.abs(got - want)
            bad = err > 1e-6 + 1e-4 * np.abs(want)
            assert bad.mean() < 0.01, (rank, int(bad.sum()), float(err.max()))
        np.testing.assert_array_equal(actors, _layers(ref.actors, ref.actors.data, 0, NS))
        np.testing.assert_allclose(losses, ref.losses.cpu().numpy(), rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(fc2, ref.state_dict("critic", lo)["fc2.weight"].numpy(), rtol=1e-4, atol=1e-5)
