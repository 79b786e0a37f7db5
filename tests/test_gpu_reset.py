"""Device reset at BASELINE densities and auto-reset behind the step.

Reference: every driver re-draws the env after a collision (main.py:24-31, learners/vdn/train_flock.py:92,
learners/maddpg_shared_critic/train_flock.py:98-99,131-134); reset() re-draws the whole swarm until no agent is
closer than collision_distance to its nearest neighbours (gym_flock_v2.py:85-108, Euclidean kNN). At main.py
density that recursion cannot terminate for N >= 256 (about 0.04 N colliding pairs per draw), so the build defines
the result: bounded whole-swarm draws first, then a per-agent repair (VecFlockEnv.reset docstring), valid[] False
only if both fail.
"""
import numpy as np
import pytest
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _min_pair_distance(pos):
    """Smallest Euclidean distance between two agents of each env: [E, N, 2] -> [E] (float64)."""
    p = torch.as_tensor(pos, dtype=torch.float64)
    d = torch.cdist(p, p)
    d.diagonal(dim1=1, dim2=2).fill_(float("inf"))
    return d.amin(dim=(1, 2))


@pytest.mark.parametrize("variant,N", [("v2", 256), ("uw_discrete", 512), ("v2", 1024)])
def test_reset_at_baseline_density(variant, N, cuda):
    """main.py density (box = round(sqrt(250 N))): bounded whole-swarm draws alone never succeed (valid False,
    as the reference's recursion never ends); with the repair stage every env is collision-free under the
    reference's own check, positions in (0, box], headings in the variant's range, and the kNN state matches the
    oracle bitwise on the final positions."""
    E, k = 32, 4
    box = float(round(np.sqrt(250 * N)))
    cd = 2.5
    base = dict(variant=variant, num_envs=E, num_agents=N, k=k, collision_distance=cd, range_start=(0, box),
                sensor_range=14.0, seed=11, max_reset_attempts=16)
    plain = VecFlockEnv(FlockConfig(**base, reset_repair_rounds=0), device=cuda)
    plain.reset()
    assert not plain.valid.any(), "whole-swarm rejection sampling at this density (SURVEY.md 8(d))"
    env = VecFlockEnv(FlockConfig(**base, reset_repair_rounds=64), device=cuda)
    env.reset()
    torch.cuda.synchronize()
    assert env.valid.all()
    pos = env.positions.cpu().numpy()
    assert (pos > 0).all() and (pos <= box).all()
    chk = 4.0 if variant == "uw_discrete" else cd
    assert (_min_pair_distance(pos) >= chk).all()
    dnn, idx = O.knn(pos, k, box, 14.0, periodic=False, clamp=True)
    np.testing.assert_array_equal(env.dnn.cpu().numpy(), dnn)
    if env.nn_idx is not None:
        np.testing.assert_array_equal(env.nn_idx.cpu().numpy(), idx)
    h = env.headings.cpu().numpy()
    top = {"v2": 1.5 * np.pi, "uw_discrete": np.pi / 1.2}[variant]
    assert (h > 0).all() and (h <= top + 1e-6).all()
    assert not env.done.any() and not env.any_done.any()
    env2 = VecFlockEnv(FlockConfig(**base, reset_repair_rounds=64), device=cuda)
    env2.reset()
    assert torch.equal(env.positions, env2.positions) and torch.equal(env.headings, env2.headings)


def _dense_pair(cuda, E=64, N=32, box=40.0, **kw):
    cfg = FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, collision_distance=2.5, range_start=(0, box),
                      sensor_range=14.0, seed=5, max_reset_attempts=64, **kw)
    envs = [VecFlockEnv(cfg, device=cuda) for _ in range(2)]
    g = torch.Generator(device=cuda).manual_seed(2)
    pos = torch.rand(E, N, 2, device=cuda, generator=g) * box
    head = torch.rand(E, N, device=cuda, generator=g) * 4.7
    for e in envs:
        e.set_state(positions=pos, headings=head)
    return envs, g


def test_auto_reset_touches_only_done_envs(cuda):
    """step(auto_reset=True) == step() followed by reset(env_mask=any_done) with the done flags kept: envs without
    a collision are bitwise the plain step's, done envs start a new episode (collision-free, valid), the returned
    done / any_done report the step's termination, and info["final_observation"] holds the terminal observation."""
    (auto, plain), g = _dense_pair(cuda)
    E = auto.E
    seen = torch.zeros(E, dtype=torch.bool, device=cuda)
    for _ in range(6):
        a = torch.stack([torch.rand(E, auto.N, device=cuda, generator=g),
                         torch.rand(E, auto.N, device=cuda, generator=g) * 3 - 1.5], -1).contiguous()
        obs, rew, (done, any_done), info = auto.step(a, auto_reset=True)
        pobs, prew, (pdone, pany), _ = plain.step(a)
        assert torch.equal(done, pdone) and torch.equal(any_done, pany) and torch.equal(rew, prew)
        assert torch.equal(info["final_observation"], pobs["actors"])
        keep = ~pany
        assert torch.equal(auto.positions[keep], plain.positions[keep])
        assert torch.equal(auto.headings[keep], plain.headings[keep])
        assert torch.equal(obs["actors"][keep], pobs["actors"][keep])
        if pany.any():
            seen |= pany
            assert auto.valid[pany].all()
            assert (_min_pair_distance(auto.positions[pany].cpu()) >= 2.5).all()
            assert not torch.equal(auto.positions[pany], plain.positions[pany])
            assert (auto.velocities[pany] == 0).all()
        # continue both from the auto-reset state so later steps compare again
        plain.set_state(positions=auto.positions, headings=auto.headings, velocities=auto.velocities)
        plain._bufs[plain._cur]["dnn"].copy_(auto.dnn)
        plain._bufs[plain._cur]["idx"].copy_(auto.nn_idx)
    assert seen.any(), "the dense swarm must produce collisions"


def test_auto_reset_is_deterministic(cuda):
    (a1, a2), g = _dense_pair(cuda)
    E = a1.E
    for _ in range(5):
        a = torch.stack([torch.rand(E, a1.N, device=cuda, generator=g),
                         torch.rand(E, a1.N, device=cuda, generator=g) * 3 - 1.5], -1).contiguous()
        a1.step(a, auto_reset=True)
        a2.step(a, auto_reset=True)
    for name in ("positions", "headings", "velocities", "dnn", "nn_idx", "reward", "done", "any_done"):
        assert torch.equal(getattr(a1, name), getattr(a2, name)), name


def test_auto_reset_with_fused_replay_insert(cuda):
    """With the replay insert fused into the step (flock_step_v2_store), the stored new observation of a done env
    is its terminal one, and the next step's stored previous observation is the reset one."""
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner

    (env, _), g = _dense_pair(cuda, N=128, box=100.0)
    E, N = env.E, env.N
    L = SharedCriticLearner(N, 4, fc1=16, fc2=8, batch_size=8, buffer_size=4 * E * N, device=cuda)
    for s in range(3):
        a = torch.stack([torch.rand(E, N, device=cuda, generator=g),
                         torch.rand(E, N, device=cuda, generator=g) * 3 - 1.5], -1).contiguous()
        prev = env.dnn.clone()
        obs, rew, (done, any_done), info = env.step(a, ring=L.replay_slots(E * N), auto_reset=True)
        rows = slice(s * E * N, (s + 1) * E * N)
        assert torch.equal(L.replay.bufs["state"][rows], prev.reshape(E * N, 4))
        assert torch.equal(L.replay.bufs["new_state"][rows], info["final_observation"].reshape(E * N, 4))
        assert torch.equal(L.replay.bufs["terminal"][rows], (~done).float().reshape(E * N))


@pytest.mark.parametrize("repair", [0, 64])
def test_single_env_reset_at_density(repair, cuda):
    """The gym surface: reset() at N=256, main.py density. Without repair it raises (the reference's recursion
    overflows: RecursionError); with the default repair it returns a collision-free swarm."""
    from marl_range_flocking_amd.environments.gym_flock_v2 import MultiAgentEnv

    env = MultiAgentEnv(256, 4, 2.5, range_start=(0, 253), sensor_range=14, max_reset_attempts=8)
    env._vec.cfg.reset_repair_rounds = repair
    if repair == 0:
        with pytest.raises(RuntimeError, match="collision-free"):
            env.reset()
    else:
        obs = env.reset()
        assert (obs["actors"] >= 2.5).all()
