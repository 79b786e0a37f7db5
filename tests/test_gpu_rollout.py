"""K gym_flock_uw steps in one call (VecFlockEnv.rollout -> torch.ops.flock.rollout_uw -> flock_rollout_uw; BASELINE
config 2's shape, N = 64 and k = 4, runs all K steps in ONE launch with the env state on chip, other shapes K step
launches). Bar: bitwise equal to K single steps (environments/gym_flock_uw.py:69-81 K times) for every per-step
output (observation memory, reward, done, any_done) and for the state the env is left in; and, free-running from the
reference fixtures' initial state, the reference's own trajectory (tests/golden/env_uw_*.npz) within the step tests'
tolerances."""
import glob
import os

import numpy as np
import pytest
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from parity import allclose_rel, meta

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _pair(cuda, E, N, k=4, box=None, layout="uniform", rigid=False, seed=1):
    box = float(round((250 * N) ** 0.5)) if box is None else box
    cfg = FlockConfig(variant="uw", num_envs=E, num_agents=N, k=k, collision_distance=2.5, range_start=(0, box),
                      sensor_range=14.0, seed=seed, rigid_boundary=rigid)
    envs = [VecFlockEnv(cfg, device=cuda) for _ in range(2)]
    g = torch.Generator(device=cuda).manual_seed(seed)
    if layout == "uniform":
        pos = torch.rand(E, N, 2, device=cuda, generator=g) * box
    elif layout == "dense":  # a crowded corner: collisions, rewards of -5, any_done
        pos = torch.rand(E, N, 2, device=cuda, generator=g) * (box / 6)
    elif layout == "lattice":  # exact distance ties: ambiguous truncated buckets, the exact rescans
        side = int(np.ceil(N ** 0.5))
        ij = torch.stack(torch.meshgrid(torch.arange(side), torch.arange(side), indexing="ij"), -1).reshape(-1, 2)
        pos = (ij[:N].float() * 4.0 + 1.0).to(cuda).expand(E, N, 2).contiguous()
    else:  # the box edges: check_boundary's teleports
        pos = torch.where(torch.rand(E, N, 2, device=cuda, generator=g) < 0.5,
                          torch.rand(E, N, 2, device=cuda, generator=g) * 0.05,
                          box - torch.rand(E, N, 2, device=cuda, generator=g) * 0.05)
    head = torch.rand(E, N, device=cuda, generator=g) * 6.28
    mem = torch.rand(E, N, 4, k, device=cuda, generator=g) * 14.0
    for e in envs:
        e.set_state(positions=pos, headings=head, prev_headings=head + 0.5, obs_memory=mem)
    return envs, g


def _check(envs, actions, out):
    K = actions.shape[0]
    ref, roll = envs
    for t in range(K):
        obs, rew, (done, any_done), _ = ref.step(actions[t])
        for name, a, b in (("obs", obs, out[0][t]), ("reward", rew, out[1][t]), ("done", done, out[2][t]),
                           ("any_done", any_done, out[3][t])):
            assert torch.equal(a, b), f"step {t}: {name}"
    for name in ("positions", "headings", "prev_headings", "velocities", "dnn", "obs_memory", "reward", "done",
                 "any_done"):
        assert torch.equal(getattr(ref, name), getattr(roll, name)), name
    if ref.nn_idx is not None:
        assert torch.equal(ref.nn_idx, roll.nn_idx)
    assert ref.steps == roll.steps  # (the buffer parity may differ: a rollout flips the double buffers once)


@pytest.fixture(params=[2, 4], ids=["spl2", "spl4"])
def spl(request):
    """The one-launch kernel's lanes per agent (flock_set_diag("rollout_spl"); 2 is the default)."""
    from marl_range_flocking_amd import _native

    lib = _native.lib()
    assert lib.flock_set_diag(b"rollout_spl", request.param) == 0
    yield request.param
    lib.flock_set_diag(b"rollout_spl", 2)


@pytest.mark.parametrize("layout", ["uniform", "dense", "lattice", "edges"])
@pytest.mark.parametrize("N,k", [(64, 4), (32, 4), (64, 3)], ids=["config2-one-launch", "N32-steps", "k3-steps"])
def test_rollout_is_bitwise_k_steps(N, k, layout, spl, cuda):
    if spl == 4 and N != 64:
        pytest.skip("the lanes-per-agent knob only changes the one-launch kernel")
    E, K = 48, 7
    envs, g = _pair(cuda, E, N, k, layout=layout, rigid=layout == "edges")
    actions = (torch.rand(K, E, N, 2, device=cuda, generator=g) * 2 - 1)
    actions[1, :, :3] = 0.0  # zero actions: nan_to_num of 0 / 0
    out = envs[1].rollout(actions)
    _check(envs, actions, out)
    # a second call continues from the state the first left (memory buffers, parity)
    actions2 = torch.rand(3, E, N, 2, device=cuda, generator=g) * 2 - 1
    _check(envs, actions2, envs[1].rollout(actions2, out=tuple(o[:3] for o in out)))


def test_rollout_config2_full_size(spl, cuda):
    """BASELINE config 2 (uw, 1024 envs x 64 agents) over K = 12 steps in one launch: bitwise 12 single steps."""
    E, N, K = 1024, 64, 12
    envs, g = _pair(cuda, E, N)
    actions = torch.rand(K, E, N, 2, device=cuda, generator=g) * 2 - 1
    _check(envs, actions, envs[1].rollout(actions))


def test_rollout_empty_and_errors(cuda):
    envs, g = _pair(cuda, 4, 64)
    out = envs[1].rollout(torch.zeros(0, 4, 64, 2, device=cuda))
    assert out[0].shape == (0, 4, 64, 4, 4) and envs[1].steps == 0
    with pytest.raises(RuntimeError):
        envs[1].rollout(torch.zeros(2, 4, 63, 2, device=cuda))
    v2 = VecFlockEnv(FlockConfig(variant="v2", num_envs=2, num_agents=16, k=4), device=cuda)
    with pytest.raises(NotImplementedError):
        v2.rollout(torch.zeros(1, 2, 16, 2, device=cuda))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "env_uw_*.npz"))),
                         ids=lambda p: os.path.basename(p)[:-4])
def test_rollout_matches_reference_trajectory(path, cuda):
    """Free-running from the fixture's initial state with the reference's actions: every step's observation memory,
    reward, dones and the final state within the single-step tests' tolerances (tests/test_gpu_env_parity.py)."""
    z = np.load(path)
    m = meta(z)
    E, N, k = m["E"], m["N"], m["k"]
    env = VecFlockEnv(FlockConfig(variant="uw", num_envs=E, num_agents=N, k=k,
                                  collision_distance=m["collision_distance"], range_start=(0, m["box"]),
                                  sensor_range=m.get("sensor_range", 14.0),
                                  normalize_distance=m.get("normalize_distance", False)), device=cuda)
    env.set_state(positions=z["pos0"], headings=z["head0"], prev_headings=z["prevh0"], velocities=z["vel0"],
                  obs_memory=z["mem0"])
    obs, rew, done, any_done = env.rollout(torch.from_numpy(np.ascontiguousarray(z["actions"])))
    torch.cuda.synchronize()
    for t in range(m["T"]):
        ok, err = allclose_rel(obs[t].cpu().numpy(), z["obs"][t], atol=1e-12)
        assert ok, f"t={t} obs memory rel err {err}"
        np.testing.assert_array_equal(rew[t].cpu().numpy(), z["reward"][t])
        np.testing.assert_array_equal(done[t].cpu().numpy(), z["done"][t])
        np.testing.assert_array_equal(any_done[t].cpu().numpy(), z["any_done"][t])
    ok, err = allclose_rel(env.positions.cpu().numpy(), z["pos"][-1], atol=1e-12)
    assert ok, f"final positions rel err {err}"
    np.testing.assert_array_equal(env.prev_headings.cpu().numpy(), z["prevh"][-1])
