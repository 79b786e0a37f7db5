"""torch.ops.flock on the GPU: torch.library.opcheck of every op (schema / mutation annotations, FakeTensor via the
Meta kernels, AOT dispatch), and VecFlockEnv(launch="torch") bitwise equal to the C-ABI launch-plan path over
multi-step rollouts of all four variants and the device reset."""
import pytest
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def flock():
    from marl_range_flocking_amd import torch_ops

    return torch_ops.load()


def _state(cuda, E=4, N=32, k=4, box=60.0, seed=0):
    g = torch.Generator(device=cuda).manual_seed(seed)
    f = dict(device=cuda)
    return dict(pos=torch.rand(E, N, 2, generator=g, **f) * box, heading=torch.rand(E, N, generator=g, **f) * 4.7,
                action=torch.rand(E, N, 2, generator=g, **f), vel=torch.zeros(E, N, 2, **f),
                dnn=torch.zeros(E, N, k, **f), nn_idx=torch.zeros(E, N, k, dtype=torch.int64, **f),
                reward=torch.zeros(E, N, **f), done=torch.zeros(E, N, dtype=torch.bool, **f),
                any_done=torch.zeros(E, dtype=torch.bool, **f))


# the AOT-dispatch checks are where functionalisation of mutating custom ops is exercised; the schema and fake
# checks cover the annotations and the Meta kernels
TESTS = ("test_schema", "test_faketensor", "test_aot_dispatch_dynamic")


def test_opcheck_step_v2(flock, cuda):
    st = _state(cuda)
    torch.library.opcheck(flock.step_v2.default, (*st.values(), None, 4, 60.0, 14.0, 2.5), test_utils=TESTS)


def test_opcheck_step_uw(flock, cuda):
    st = _state(cuda)
    E, N, k = 4, 32, 4
    mem_in, mem_out = torch.rand(E, N, 4, k, device=cuda), torch.zeros(E, N, 4, k, device=cuda)
    prev = torch.zeros(E, N, device=cuda)
    args = (st["pos"], st["heading"], prev, st["action"], mem_in, mem_out, st["vel"], st["dnn"], None, st["reward"],
            st["done"], st["any_done"], None, k, 60.0, 14.0, 2.5)
    torch.library.opcheck(flock.step_uw.default, args, test_utils=TESTS)


@pytest.mark.parametrize("N", [64, 32], ids=["one-launch", "step-launches"])
def test_opcheck_rollout_uw(flock, cuda, N):
    st = _state(cuda, N=N)
    E, k, K = 4, 4, 3
    mem_in, mem_out = torch.rand(E, N, 4, k, device=cuda), torch.zeros(E, N, 4, k, device=cuda)
    prev = torch.zeros(E, N, device=cuda)
    outs = (torch.zeros(K, E, N, 4, k, device=cuda), torch.zeros(K, E, N, device=cuda),
            torch.zeros(K, E, N, dtype=torch.bool, device=cuda), torch.zeros(K, E, dtype=torch.bool, device=cuda))
    args = (st["pos"], st["heading"], prev, torch.rand(K, E, N, 2, device=cuda), mem_in, mem_out, st["vel"],
            st["dnn"], None, st["reward"], st["done"], st["any_done"], *outs, None, k, 60.0, 14.0, 2.5)
    torch.library.opcheck(flock.rollout_uw.default, args, test_utils=TESTS)


def test_opcheck_step_uw_discrete(flock, cuda):
    st = _state(cuda)
    E, N, k = 4, 32, 4
    ids = torch.randint(0, 10, (E, N), device=cuda)
    from marl_range_flocking_amd.ops import UWD_TABLE

    table = torch.tensor(UWD_TABLE, device=cuda)
    status = torch.zeros(1, dtype=torch.int32, device=cuda)
    args = (st["pos"], st["heading"], torch.zeros(E, N, device=cuda), ids, torch.randn(E, N, 2, device=cuda) * 0.1,
            table, st["vel"], st["dnn"], None, st["reward"], st["done"], st["any_done"], status, None, k, 60.0, 14.0,
            3.0)
    torch.library.opcheck(flock.step_uw_discrete.default, args, test_utils=TESTS)


def test_opcheck_step_flock(flock, cuda):
    st = _state(cuda)
    E, N, k = 4, 32, 4
    vel = torch.nn.functional.normalize(torch.rand(E, N, 2, device=cuda) + 0.1, dim=-1)
    args = (st["pos"], vel, st["action"], torch.rand(E, N, 4, k, device=cuda), torch.zeros(E, N, 4, k, device=cuda),
            st["dnn"], None, st["reward"], st["done"], st["any_done"], None, k, 60.0, 2.5)
    torch.library.opcheck(flock.step_flock.default, args, test_utils=TESTS)


def test_opcheck_knn_and_reset(flock, cuda):
    st = _state(cuda)
    torch.library.opcheck(flock.knn.default, (st["pos"], 4, 60.0), test_utils=TESTS)
    E, N, k = 4, 32, 4
    valid = torch.zeros(E, dtype=torch.bool, device=cuda)
    args = (st["pos"], st["dnn"], st["heading"], torch.zeros(E, N, device=cuda), st["vel"], st["nn_idx"], None,
            valid, None, 0, k, 0.0, 60.0, 60.0, 14.0, 2.5)
    torch.library.opcheck(flock.reset.default, args, test_utils=TESTS)


def test_ops_errors(flock, cuda):
    st = _state(cuda, N=4)
    with pytest.raises(RuntimeError, match="selected index k out of range"):
        flock.step_v2(*st.values(), None, 4, 60.0, 14.0, 2.5)
    st = _state(cuda)
    with pytest.raises(RuntimeError, match="action must be"):
        flock.step_v2(*dict(st, action=st["action"].double()).values(), None, 4, 60.0, 14.0, 2.5)


@pytest.mark.parametrize("variant,N,norm", [("v2", 64, False), ("v2", 256, False), ("uw", 64, False),
                                            ("uw_discrete", 128, False), ("flock", 16, False), ("uw", 64, True),
                                            ("uw_discrete", 128, True), ("flock", 16, True)])
def test_torch_ops_path_is_bitwise_the_plan_path(variant, N, norm, cuda):
    """norm: normalize_distance=True steps and resets through the ops' normalize_distance flag (the full-scan
    kernels, FlockStepExt.normalize_distance / flock_reset_ext2) against the plan path."""
    E, k = 16, 4
    box = float(round((250 * N) ** 0.5))
    cfg = FlockConfig(variant=variant, num_envs=E, num_agents=N, k=k, collision_distance=2.5 if not norm else 0.05,
                      range_start=(0, box), sensor_range=14.0, seed=7, max_reset_attempts=8, normalize_distance=norm)
    envs = [VecFlockEnv(cfg, device=cuda, launch=o) for o in ("plan", "torch")]
    for e in envs:
        e.reset()
    g = torch.Generator(device=cuda).manual_seed(3)
    for _ in range(4):
        if variant == "uw_discrete":
            a = torch.randint(0, 10, (E, N), device=cuda, generator=g)
        elif variant == "v2":
            a = torch.stack([torch.rand(E, N, device=cuda, generator=g),
                             torch.rand(E, N, device=cuda, generator=g) * 3 - 1.5], -1).contiguous()
        else:
            a = (torch.rand(E, N, 2, device=cuda, generator=g) * 2 - 1).contiguous()
        outs = [e.step(a) for e in envs]
        for name in ("positions", "headings", "prev_headings", "velocities", "dnn", "reward", "done", "any_done"):
            assert torch.equal(getattr(envs[0], name), getattr(envs[1], name)), name
        if envs[0].nn_idx is not None:
            assert torch.equal(envs[0].nn_idx, envs[1].nn_idx)
        if envs[0].obs_memory is not None:
            assert torch.equal(envs[0].obs_memory, envs[1].obs_memory)
