"""The step kernel's cell-list kNN (N >= 128) against its own full scan (flock_set_diag("no_cells", 1)) and the C
oracle.

The cell path must be indistinguishable from the all-pairs scan: every output of a step (positions, velocities,
headings, neighbour distances and indices, reward, done) is compared BITWISE between the two paths from the same
state, over uniform, clustered (many agents per cell, forcing long ranges and the full-scan fallback), box-edge
(x = box / tiny x, cell clamping and periodic ghosts) and integer-lattice (exact distance ties, the ambiguous-bucket
rescan), and sparse (a blob plus isolated outliers: the 5x5 and full-scan fallbacks) placements, N in 128..1024
and k up to 15; sampled envs are also checked against the oracle's exact kNN.
"""
import contextlib

import numpy as np
import pytest
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv, _native
from parity import _knn_exact

pytestmark = pytest.mark.gpu


def _positions(kind, E, N, box, rng):
    if kind == "uniform":
        return rng.uniform(0, box, (E, N, 2))
    if kind == "clustered":  # 4 tight blobs: ~N/4 agents in one or two cells
        centres = rng.uniform(0.1 * box, 0.9 * box, (E, 4, 2))
        pick = rng.integers(0, 4, (E, N))
        p = np.take_along_axis(centres, pick[..., None].repeat(2, -1), 1) + rng.normal(0, box / 60, (E, N, 2))
        return np.clip(p, 0.001, box)
    if kind == "edges":  # half the agents hugging the box edges and corners
        p = rng.uniform(0, box, (E, N, 2))
        m = rng.uniform(size=(E, N, 2)) < 0.25
        p[m] = np.where(rng.uniform(size=m.sum()) < 0.5, rng.uniform(0.001, 0.5, m.sum()),
                        rng.uniform(box - 0.5, box, m.sum()))
        return p
    if kind == "sparse":  # a dense blob plus isolated outliers: blob-edge agents need the 5x5 neighbourhood, the
        # outliers (fewer than L agents within 2 cells) the full scan
        c = rng.uniform(0.3 * box, 0.7 * box, (E, 1, 2))
        p = c + rng.normal(0, box / 25, (E, N, 2))
        m = rng.uniform(size=(E, N)) < 0.08
        p[m] = rng.uniform(0, box, (m.sum(), 2))
        return np.clip(p, 0.001, box)
    if kind == "lattice":  # integer grid, equal spacing -> exact d2 ties
        side = int(np.ceil(np.sqrt(N)))
        g = np.stack(np.meshgrid(np.arange(side), np.arange(side)), -1).reshape(-1, 2)[:N].astype(np.float64)
        g = g * (box / side) + 0.5
        return np.broadcast_to(g, (E, N, 2)).copy()
    raise ValueError(kind)


@contextlib.contextmanager
def diag(name, value, default=0):
    """Set one diagnostics knob of the step library (flock_set_diag) for the body, then restore its default."""
    lib = _native.lib()
    assert lib.flock_set_diag(name.encode(), int(value)) == 0
    try:
        yield
    finally:
        lib.flock_set_diag(name.encode(), int(default))


def _step(variant, periodic, pos, head, prev, vel, mem, act, noise, N, k, box, cuda, cells):
    E = pos.shape[0]
    env = VecFlockEnv(FlockConfig(variant=variant, num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                                  range_start=(0, box), sensor_range=14.0, periodic=periodic), device=cuda)
    env.set_state(positions=pos, headings=head, prev_headings=prev, velocities=vel,
                  obs_memory=mem if variant in ("uw", "flock") else None)
    with diag("no_cells", 0 if cells else 1):
        if variant == "uw_discrete":
            out = env.step(torch.from_numpy(act), noise=torch.from_numpy(noise))
        else:
            out = env.step(torch.from_numpy(act))
        torch.cuda.synchronize()
    obs, rew, (done, anyd), _ = out
    res = {"pos": env.positions, "vel": env.velocities, "head": env.headings, "dnn": env.dnn, "idx": env.nn_idx,
           "rew": rew, "done": done, "any": anyd}
    return {k2: v.detach().cpu().numpy().copy() for k2, v in res.items()}


CASES = [("v2", True, 256, 4, "uniform"), ("v2", True, 256, 4, "clustered"), ("v2", True, 256, 4, "edges"),
         ("v2", True, 256, 4, "lattice"), ("v2", False, 256, 4, "edges"), ("v2", True, 128, 1, "uniform"),
         ("v2", True, 500, 15, "uniform"), ("v2", True, 1024, 4, "uniform"), ("v2", True, 1024, 11, "clustered"),
         ("uw", False, 256, 4, "uniform"), ("uw", False, 512, 4, "edges"), ("uw_discrete", False, 512, 4, "uniform"),
         ("flock", False, 300, 6, "clustered"), ("v2", False, 1000, 9, "lattice"), ("v2", True, 256, 4, "sparse"),
         ("v2", True, 1024, 4, "sparse"), ("uw", False, 512, 7, "sparse"), ("v2", True, 600, 15, "sparse")]


@pytest.mark.parametrize("variant,periodic,N,k,kind", CASES,
                         ids=[f"{v}-{'per' if p else 'euc'}-N{n}-k{k}-{d}" for v, p, n, k, d in CASES])
def test_cell_list_step_is_bitwise_the_full_scan(variant, periodic, N, k, kind, cuda):
    E = 64 if N <= 512 else 16
    box = float(round(np.sqrt(250 * N)))
    rng = np.random.default_rng(N * 31 + k)
    pos = _positions(kind, E, N, box, rng).astype(np.float32)
    head = rng.uniform(0, 2 * np.pi, (E, N)).astype(np.float32)
    prev = rng.uniform(0, 2 * np.pi, (E, N)).astype(np.float32)
    vel = rng.standard_normal((E, N, 2)).astype(np.float32)
    vel /= np.linalg.norm(vel, axis=-1, keepdims=True)
    mem = rng.uniform(0, 14, (E, N, 4, k)).astype(np.float32)
    noise = None
    if variant == "uw_discrete":
        act = rng.integers(0, 10, (E, N)).astype(np.int64)
        noise = (0.1 * rng.standard_normal((E, N, 2))).astype(np.float32)
    else:
        act = rng.uniform(-1.5, 2.5, (E, N, 2)).astype(np.float32)
        if kind == "lattice":
            act[..., 0] = 0.0  # keep the lattice (and its ties) intact through the step
            act[..., 1] = 0.0
    args = (variant, periodic, pos, head, prev, vel, mem, act, noise, N, k, box, cuda)
    a = _step(*args, cells=True)
    b = _step(*args, cells=False)
    for key in a:
        np.testing.assert_array_equal(a[key], b[key], err_msg=key)
    sample = np.arange(0, E, max(1, E // 6))
    _knn_exact(a["pos"][sample], k, box, 14.0, periodic, variant != "flock", a["dnn"][sample], a["idx"][sample])


ROLLOUTS = [("v2", True, 256, 4, "uniform"), ("v2", True, 1024, 4, "uniform"), ("v2", True, 256, 4, "clustered"),
            ("v2", False, 300, 6, "sparse"), ("uw", False, 256, 4, "edges"), ("uw_discrete", False, 512, 4, "uniform"),
            ("flock", False, 256, 4, "uniform"), ("v2", True, 500, 15, "uniform")]


@pytest.mark.parametrize("variant,periodic,N,k,kind", ROLLOUTS,
                         ids=[f"{v}-{'per' if p else 'euc'}-N{n}-k{k}-{d}" for v, p, n, k, d in ROLLOUTS])
def test_seeded_rollout_is_bitwise_the_full_scan(variant, periodic, N, k, kind, cuda):
    """Multi-step rollouts, where the cell path takes its seeded scan (the previous step's neighbours from the compact
    seed buffer): every step's outputs equal the full scan's bit for bit, also after the seeds are overwritten with
    garbage (negative, out-of-range and repeated indices) mid-rollout."""
    E = 32 if N <= 512 else 8
    box = float(round(np.sqrt(250 * N)))
    rng = np.random.default_rng(N * 7 + k)
    pos = _positions(kind, E, N, box, rng).astype(np.float32)
    head = rng.uniform(0, 2 * np.pi, (E, N)).astype(np.float32)
    vel = rng.standard_normal((E, N, 2)).astype(np.float32)
    vel /= np.linalg.norm(vel, axis=-1, keepdims=True)
    mem = rng.uniform(0, 14, (E, N, 4, k)).astype(np.float32)
    envs = []
    for _ in range(2):
        env = VecFlockEnv(FlockConfig(variant=variant, num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                                      range_start=(0, box), sensor_range=14.0, periodic=periodic), device=cuda)
        env.set_state(positions=pos, headings=head, velocities=vel,
                      obs_memory=mem if variant in ("uw", "flock") else None)
        envs.append(env)
    assert envs[0].seeds is not None
    for t in range(7):
        if variant == "uw_discrete":
            act = torch.from_numpy(rng.integers(0, 10, (E, N)).astype(np.int64))
            kw = dict(noise=torch.from_numpy((0.1 * rng.standard_normal((E, N, 2))).astype(np.float32)))
        else:
            act = torch.from_numpy(rng.uniform(-1.0, 2.5, (E, N, 2)).astype(np.float32))
            kw = {}
        if t == 4:  # garbage seeds: both signs, beyond N, repeats
            g = rng.integers(-40000, 40000, (E, N, k)).astype(np.int16)
            g[:, : N // 3] = 3
            envs[0].seeds.copy_(torch.from_numpy(g))
        outs = []
        for i, env in enumerate(envs):
            with diag("no_cells", i):
                obs, rew, (done, anyd), _ = env.step(act, **kw)
                torch.cuda.synchronize()
            outs.append({"pos": env.positions, "vel": env.velocities, "head": env.headings, "dnn": env.dnn,
                         "idx": env.nn_idx, "rew": rew, "done": done, "any": anyd})
        for key in outs[0]:
            assert torch.equal(outs[0][key], outs[1][key]), f"step {t}: {key}"
        if t >= 1 and t != 4:  # the seed buffer holds this step's neighbours
            assert torch.equal(envs[0].seeds.to(torch.int64), envs[0].nn_idx)


SPEC = [("v2", True, 256, "uniform"), ("v2", True, 1024, "clustered"), ("uw_discrete", False, 512, "edges"),
        ("uw", False, 64, "uniform")]


@pytest.mark.parametrize("knob", ["no_spec", "no_split"])
@pytest.mark.parametrize("variant,periodic,N,kind", SPEC, ids=[f"{v}-N{n}-{d}" for v, _, n, d in SPEC])
def test_specialised_kernel_is_bitwise_the_generic_one(variant, periodic, N, kind, knob, cuda):
    """The BASELINE configurations' shapes launch step_kernel instantiations specialised on (variant, N, k = 4, cell
    grid); no_spec launches the generic instantiation. The config-2 shape (uw, N = 64) also splits its candidate scan
    over 4 lanes per agent; no_split takes the one-lane scan. Four-step rollouts agree bit for bit on every output,
    the observation memory and the seed buffer."""
    k, E = 4, (16 if N >= 512 else 64)
    box = float(round(np.sqrt(250 * N)))
    rng = np.random.default_rng(N + 5)
    pos = _positions(kind, E, N, box, rng).astype(np.float32)
    head = rng.uniform(0, 2 * np.pi, (E, N)).astype(np.float32)
    mem = rng.uniform(0, 14, (E, N, 4, k)).astype(np.float32)
    envs = []
    for _ in range(2):
        env = VecFlockEnv(FlockConfig(variant=variant, num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                                      range_start=(0, box), sensor_range=14.0, periodic=periodic), device=cuda)
        env.set_state(positions=pos, headings=head, obs_memory=mem if variant == "uw" else None)
        envs.append(env)
    for t in range(4):
        if variant == "uw_discrete":
            act = torch.from_numpy(rng.integers(0, 4, (E, N)).astype(np.int64))
            kw = dict(noise=torch.from_numpy((0.1 * rng.standard_normal((E, N, 2))).astype(np.float32)))
        else:
            act = torch.from_numpy(rng.uniform(-1.0, 2.5, (E, N, 2)).astype(np.float32))
            kw = {}
        outs = []
        for i, env in enumerate(envs):
            with diag(knob, i):
                obs, rew, (done, anyd), _ = env.step(act, **kw)
                torch.cuda.synchronize()
            o = obs["actors"] if isinstance(obs, dict) else obs
            outs.append({"pos": env.positions, "vel": env.velocities, "head": env.headings, "dnn": env.dnn,
                         "idx": env.nn_idx, "rew": rew, "done": done, "any": anyd, "obs": o.clone()})
            if env.seeds is not None:
                outs[-1]["seeds"] = env.seeds.clone()
        for key in outs[0]:
            assert torch.equal(outs[0][key], outs[1][key]), f"step {t}: {key}"


class _NoPlans(dict):
    """VecFlockEnv plan cache that never keeps a plan: every step takes the fully checked launch path."""

    def __setitem__(self, key, value):
        pass


@pytest.mark.parametrize("variant,periodic,N", [("v2", True, 256), ("uw", False, 64), ("uw_discrete", False, 512),
                                                ("flock", False, 128)])
def test_step_plan_replay_is_bitwise_the_checked_launch(variant, periodic, N, cuda):
    """ops.StepPlan (recorded launch per buffer parity, replayed with a new stream / action / dt / RNG offset)
    against the checked launch on every step of a 6-step rollout, including a dt change mid-rollout."""
    k, E = 4, 16
    box = float(round(np.sqrt(250 * N)))
    rng = np.random.default_rng(N + 11)
    pos = _positions("uniform", E, N, box, rng).astype(np.float32)
    head = rng.uniform(0, 2 * np.pi, (E, N)).astype(np.float32)
    envs = []
    for i in range(2):
        env = VecFlockEnv(FlockConfig(variant=variant, num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                                      range_start=(0, box), sensor_range=14.0, periodic=periodic), device=cuda,
                          launch="plan")
        env.set_state(positions=pos, headings=head)
        if i == 1:
            env.__dict__["_plans"] = _NoPlans()
        envs.append(env)
    for t in range(6):
        if variant == "uw_discrete":
            act = torch.from_numpy(rng.integers(0, 4, (E, N)).astype(np.int64)).to(cuda)
        else:
            act = torch.from_numpy(rng.uniform(-1.0, 2.5, (E, N, 2)).astype(np.float32)).to(cuda)
        dt = 0.1 if t < 4 else 0.05
        outs = []
        for env in envs:
            obs, rew, (done, anyd), _ = env.step(act, dt=dt)
            o = obs["actors"] if isinstance(obs, dict) else obs
            outs.append([env.positions.clone(), env.headings.clone(), env.dnn.clone(), env.nn_idx.clone(),
                         rew.clone(), done.clone(), anyd.clone(), o.clone()])
        torch.cuda.synchronize()
        for x, y in zip(*outs):
            assert torch.equal(x, y), f"step {t}"
    assert envs[0]._plans and all(p.fn is not None for p in envs[0]._plans.values())


@pytest.mark.parametrize("variant,periodic,N,kind", SPEC, ids=[f"{v}-N{n}-{d}" for v, _, n, d in SPEC])
def test_untracked_indices_change_nothing_else(variant, periodic, N, kind, cuda):
    """track_indices=False (bench.py's uw / uw_discrete configs: the reference returns no neighbour indices there)
    skips the int64 index stores; four-step rollouts agree bit for bit with the tracked run on every other output,
    the observation memory and the seed buffer."""
    k, E = 4, (16 if N >= 512 else 64)
    box = float(round(np.sqrt(250 * N)))
    rng = np.random.default_rng(N + 9)
    pos = _positions(kind, E, N, box, rng).astype(np.float32)
    head = rng.uniform(0, 2 * np.pi, (E, N)).astype(np.float32)
    mem = rng.uniform(0, 14, (E, N, 4, k)).astype(np.float32)
    envs = []
    for track in (True, False):
        env = VecFlockEnv(FlockConfig(variant=variant, num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                                      range_start=(0, box), sensor_range=14.0, periodic=periodic,
                                      track_indices=track), device=cuda)
        env.set_state(positions=pos, headings=head, obs_memory=mem if variant == "uw" else None)
        envs.append(env)
    assert envs[1].nn_idx is None
    for t in range(4):
        if variant == "uw_discrete":
            act = torch.from_numpy(rng.integers(0, 4, (E, N)).astype(np.int64))
            kw = dict(noise=torch.from_numpy((0.1 * rng.standard_normal((E, N, 2))).astype(np.float32)))
        else:
            act = torch.from_numpy(rng.uniform(-1.0, 2.5, (E, N, 2)).astype(np.float32))
            kw = {}
        outs = []
        for env in envs:
            obs, rew, (done, anyd), _ = env.step(act, **kw)
            torch.cuda.synchronize()
            o = obs["actors"] if isinstance(obs, dict) else obs
            outs.append({"pos": env.positions, "vel": env.velocities, "head": env.headings, "dnn": env.dnn,
                         "rew": rew, "done": done, "any": anyd, "obs": o.clone()})
            if env.seeds is not None:
                outs[-1]["seeds"] = env.seeds.clone()
        for key in outs[0]:
            assert torch.equal(outs[0][key], outs[1][key]), f"step {t}: {key}"


def test_env_range_launches_are_bitwise_one_launch(cuda):
    """flock_set_diag("env_launches", n) splits a step into n launches over consecutive env ranges (Params.env0): a four-step
    config-3-shape rollout (v2, N = 256, seeds, every output) is bit for bit the one-launch rollout."""
    k, E, N = 4, 37, 256  # E not a multiple of the split: the last range is short
    box = float(round(np.sqrt(250 * N)))
    rng = np.random.default_rng(11)
    pos = rng.uniform(0, box, (E, N, 2)).astype(np.float32)
    head = rng.uniform(0, 2 * np.pi, (E, N)).astype(np.float32)
    envs = []
    for _ in range(2):
        env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                                      range_start=(0, box), sensor_range=14.0), device=cuda)
        env.set_state(positions=pos, headings=head)
        envs.append(env)
    for t in range(4):
        act = torch.from_numpy(rng.uniform(-1.0, 2.5, (E, N, 2)).astype(np.float32))
        outs = []
        for i, env in enumerate(envs):
            with diag("env_launches", 4 if i else 1, default=1):
                obs, rew, (done, anyd), _ = env.step(act)
                torch.cuda.synchronize()
            outs.append({"pos": env.positions, "vel": env.velocities, "head": env.headings, "dnn": env.dnn,
                         "idx": env.nn_idx, "rew": rew, "done": done, "any": anyd,
                         "seeds": env.seeds.clone() if env.seeds is not None else rew})
        for key in outs[0]:
            assert torch.equal(outs[0][key], outs[1][key]), f"step {t}: {key}"


@pytest.mark.parametrize("variant,periodic,N,kind", SPEC[:3], ids=[f"{v}-N{n}-{d}" for v, _, n, d in SPEC[:3]])
def test_step_launches_are_bitwise_one_launch(variant, periodic, N, kind, cuda):
    """FlockConfig.step_launches > 1 (FlockStepExt.launches): the step as several launches over consecutive env
    ranges. Envs are independent, so three-step rollouts equal the one-launch step bit for bit."""
    k, E = 4, 37
    box = float(round(np.sqrt(250 * N)))
    rng = np.random.default_rng(N + 11)
    pos = _positions(kind, E, N, box, rng).astype(np.float32)
    head = rng.uniform(0, 2 * np.pi, (E, N)).astype(np.float32)
    envs = []
    for launches in (1, 3):
        env = VecFlockEnv(FlockConfig(variant=variant, num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                                      range_start=(0, box), sensor_range=14.0, periodic=periodic,
                                      step_launches=launches), device=cuda)
        env.set_state(positions=pos, headings=head)
        envs.append(env)
    for t in range(3):
        if variant == "uw_discrete":
            act = torch.from_numpy(rng.integers(0, 4, (E, N)).astype(np.int64))
            kw = dict(noise=torch.from_numpy((0.1 * rng.standard_normal((E, N, 2))).astype(np.float32)))
        else:
            act = torch.from_numpy(rng.uniform(-1.0, 2.5, (E, N, 2)).astype(np.float32))
            kw = {}
        outs = []
        for env in envs:
            obs, rew, (done, anyd), _ = env.step(act, **kw)
            torch.cuda.synchronize()
            outs.append({"pos": env.positions.clone(), "head": env.headings.clone(), "dnn": env.dnn.clone(),
                         "idx": env.nn_idx.clone(), "rew": rew.clone(), "done": done.clone(), "any": anyd.clone()})
        for key in outs[0]:
            assert torch.equal(outs[0][key], outs[1][key]), f"step {t}: {key}"


@pytest.mark.parametrize("N,E", [(1024, 1100), (256, 2600)], ids=["config5-shape", "config3-shape"])
@pytest.mark.parametrize("kind", ["uniform", "clustered"])
def test_l2_pull_ahead_is_bitwise_the_plain_launch(kind, N, E, cuda):
    """Config 5's and config 3's shapes (v2, N = 1024 / 256, periodic) as one launch of more env blocks than fit on
    the device at once: each block then pulls the kinematics inputs of the block pf_ahead places later into the
    caches (pf = -1, the default there); pf = 0 launches the plain blocks. E above the resident blocks (512 / 2048;
    the last blocks pull nothing) with the RNN-MADDPG record insert (one ring row per env, the actor copies as 16-B
    stores): three steps agree bit for bit on every output, the seed buffer and every replay field."""
    from marl_range_flocking_amd.learners.maddpg import MADDPGLearner

    k = 4
    box = float(round(np.sqrt(250 * N)))
    rng = np.random.default_rng(11)
    pos = _positions(kind, E, N, box, rng).astype(np.float32)
    head = rng.uniform(0, 2 * np.pi, (E, N)).astype(np.float32)
    envs, learners = [], []
    for _ in range(2):
        env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                                      range_start=(0, box), sensor_range=14.0, periodic=True), device=cuda)
        env.set_state(positions=pos, headings=head)
        envs.append(env)
        learners.append(MADDPGLearner(N, k, recurrent=True, hidden1=8, hidden2=8, batch_size=8, chunk_size=4,
                                      buffer_capacity=1500, min_size_buffer=8, device=cuda, use_graph=False))
    for t in range(3):
        act = torch.from_numpy(rng.uniform(-1.0, 2.5, (E, N, 2)).astype(np.float32)).to(cuda)
        outs = []
        for i, (env, L) in enumerate(zip(envs, learners)):
            with diag("pf", -1 if i == 0 else 0, default=-1):
                obs, rew, (done, anyd), _ = env.step(act, ring=L.replay_slots(E))
                torch.cuda.synchronize()
            outs.append({"pos": env.positions, "vel": env.velocities, "head": env.headings, "dnn": env.dnn,
                         "idx": env.nn_idx, "rew": rew, "done": done, "any": anyd, "seeds": env.seeds.clone()})
        for key in outs[0]:
            assert torch.equal(outs[0][key], outs[1][key]), f"step {t}: {key}"
    for name in learners[0].replay.bufs:
        assert torch.equal(learners[0].replay.bufs[name], learners[1].replay.bufs[name]), name
