"""torch.ops.flock (csrc/flock_torch.cpp) without a GPU: the library loads, the schemas carry the mutation
annotations of SURVEY.md §8(b), the Meta kernels give shapes and the reference's errors, and CPU tensors are refused
(no CPU fallback)."""
import pytest
import torch

from marl_range_flocking_amd import build


@pytest.fixture(scope="module")
def flock():
    build.build()
    from marl_range_flocking_amd import torch_ops

    return torch_ops.load()


def test_schemas_annotate_every_written_buffer(flock):
    s = str(flock.step_v2.default._schema)
    for arg in ("Tensor(a!) pos", "Tensor(b!) heading", "Tensor action", "Tensor(c!) vel", "Tensor(d!) dnn",
                "Tensor(e!)? nn_idx", "Tensor(f!) reward", "Tensor(g!) done", "Tensor(h!) any_done"):
        assert arg in s, arg
    assert s.endswith("-> ()")
    assert "Tensor mem_in" in str(flock.step_uw.default._schema)
    assert "Tensor(c!) mem_out" in str(flock.step_uw.default._schema)
    assert "Tensor action_id" in str(flock.step_uw_discrete.default._schema)
    assert "Tensor(b!) vel" in str(flock.step_flock.default._schema)
    assert str(flock.knn.default._schema).endswith("-> (Tensor dnn, Tensor nn_idx)")
    assert "Tensor? env_mask" in str(flock.reset.default._schema)


def _meta_state(E, N, k):
    m = dict(device="meta")
    return dict(pos=torch.empty(E, N, 2, **m), heading=torch.empty(E, N, **m), action=torch.empty(E, N, 2, **m),
                vel=torch.empty(E, N, 2, **m), dnn=torch.empty(E, N, k, **m),
                nn_idx=torch.empty(E, N, k, dtype=torch.int64, **m), reward=torch.empty(E, N, **m),
                done=torch.empty(E, N, dtype=torch.bool, **m), any_done=torch.empty(E, dtype=torch.bool, **m))


def test_meta_kernels(flock):
    dnn, idx = flock.knn(torch.empty(3, 16, 2, device="meta"), 4, 20.0)
    assert dnn.shape == (3, 16, 4) and idx.shape == (3, 16, 4) and idx.dtype == torch.int64
    st = _meta_state(3, 16, 4)
    flock.step_v2(*st.values(), None, 4, 20.0, 14.0, 2.5)
    with pytest.raises(RuntimeError, match="selected index k out of range"):  # torch.topk, gym_flock_v2.py:147
        flock.knn(torch.empty(3, 4, 2, device="meta"), 4, 20.0)
    bad = dict(st, heading=torch.empty(3, 16, dtype=torch.float64, device="meta"))
    with pytest.raises(RuntimeError, match="heading must be"):
        flock.step_v2(*bad.values(), None, 4, 20.0, 14.0, 2.5)
    bad = dict(st, dnn=torch.empty(3, 16, 5, device="meta"))
    with pytest.raises(RuntimeError, match="dnn must have shape"):
        flock.step_v2(*bad.values(), None, 4, 20.0, 14.0, 2.5)


def test_cpu_tensors_are_refused(flock):
    with pytest.raises(NotImplementedError):
        flock.knn(torch.zeros(2, 8, 2), 4, 10.0)


def test_sc_act_schema_meta_and_refusal(flock):
    """flock::sc_act (choose_action of every agent, csrc/flock_act.hip): mutation annotations, Meta shape checks with
    the op's errors, and no CPU implementation."""
    s = str(flock.sc_act.default._schema)
    for arg in ("Tensor obs", "Tensor actors", "Tensor(a!) actions", "Tensor(b!)? ou_state", "Tensor? noise"):
        assert arg in s, arg
    m = dict(device="meta")
    obs, actors = torch.empty(10, 3, 4, **m), torch.empty(3 * 320, **m)
    act, ou, z = torch.empty(10, 3, 2, **m), torch.empty(10, 3, 2, **m), torch.empty(10, 3, 2, **m)
    flock.sc_act(obs, actors, act, ou, z, 16, 8, 0.2, 0.01, 0.015)
    flock.sc_act(obs, actors, act, None, None, 16, 8, 0.2, 0.01, 0.015)
    with pytest.raises(RuntimeError, match="actions must have shape"):
        flock.sc_act(obs, actors, torch.empty(10, 3, 3, **m), None, None, 16, 8, 0.2, 0.01, 0.015)
    with pytest.raises(RuntimeError, match="fc1 a multiple of 8"):
        flock.sc_act(obs, actors, act, None, None, 12, 8, 0.2, 0.01, 0.015)
    with pytest.raises(RuntimeError, match="ou_state and noise"):
        flock.sc_act(obs, actors, act, ou, None, 16, 8, 0.2, 0.01, 0.015)
    with pytest.raises(NotImplementedError):
        flock.sc_act(torch.zeros(10, 3, 4), torch.zeros(960), torch.zeros(10, 3, 2), None, None, 16, 8, 0.2, 0.01,
                     0.015)
