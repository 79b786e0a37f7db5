"""CPU tests of the C-ABI boundary: libflock_amd.so loads, exports every symbol include/flock_amd.h declares with the
arity the Python binding uses, and rejects bad arguments before touching the GPU (no compute here)."""
import ctypes
import os
import re

import pytest

from marl_range_flocking_amd import _native, build

INCLUDE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
HEADERS = [os.path.join(INCLUDE, h) for h in sorted(os.listdir(INCLUDE)) if h.endswith(".h")]


def header_functions():
    src = "\n".join(open(h).read() for h in HEADERS)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*(?:int|int64_t|const char\*|void|\w+\*)\s+(flock_\w+)\s*\(([^;]*?)\)\s*;", src,
                         flags=re.M | re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else len(args.split(","))
    return out


@pytest.fixture(scope="module")
def lib():
    build.build()
    return _native.lib()


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for name in ("flock_step_v2", "flock_step_uw", "flock_step_uw_discrete", "flock_step_flock", "flock_knn",
                 "flock_reset", "flock_abi_version", "flock_last_error", "flock_adam_step", "flock_soft_update",
                 "flock_grad_norm", "flock_gru_fwd", "flock_gru_bwd", "flock_gather_rows", "flock_scatter_rows",
                 "flock_sc_workspace_floats", "flock_sc_critic_update", "flock_sc_actor_update",
                 "flock_sc_prep_snapshot", "flock_sc_round", "flock_sc_pipeline_create", "flock_sc_pipeline_learn",
                 "flock_sc_pipeline_flush"):
        assert name in fns, name


def test_library_exports_every_declared_symbol_with_binding_arity(lib):
    for name, nargs in header_functions().items():
        assert hasattr(lib, name), f"{name} not exported"
        assert name in _native.SIGNATURES, f"{name} has no Python binding"
        assert len(_native.SIGNATURES[name]) == nargs, f"{name}: header has {nargs} args"


def test_abi_version(lib):
    assert lib.flock_abi_version() == 1


def test_k_out_of_range_rejected_like_torch_topk(lib):
    # N = 4, k = 4: the reference raises "selected index k out of range" (tests/golden/errors.json)
    rc = lib.flock_knn(None, 1, 4, 4, 10.0, 7.0, 1, 1, None, None, None)
    assert rc == -1
    assert lib.flock_last_error().decode() == "selected index k out of range"


def test_limits_and_null_pointers_rejected(lib):
    assert lib.flock_knn(None, 1, 2048, 4, 10.0, 7.0, 1, 1, None, None, None) == -2
    assert lib.flock_knn(None, 1, 64, 16, 10.0, 7.0, 1, 1, None, None, None) == -2
    assert lib.flock_knn(None, 1, 64, 4, 10.0, 7.0, 1, 1, None, None, None) == -3
    rc = lib.flock_reset(None, 0, 1, 64, 4, 0.0, 50.0, 50.0, 14.0, 2.5, 0, 0, 0, 0, *([None] * 9))
    assert rc == -3
    x = ctypes.c_float(0)
    rc = lib.flock_reset(None, 9, 1, 64, 4, 0.0, 50.0, 50.0, 14.0, 2.5, 0, 4, 0, 0, None, ctypes.byref(x), None,
                         None, None, ctypes.byref(x), None, None, None)
    assert rc == -5


def test_empty_batch_is_a_noop(lib):
    assert lib.flock_knn(None, 0, 64, 4, 10.0, 7.0, 1, 1, None, None, None) == 0


def test_ops_refuse_cpu_tensors():
    import torch

    from marl_range_flocking_amd import ops

    with pytest.raises(RuntimeError, match="HIP device"):
        ops.knn(torch.zeros(1, 8, 2), 4, 10.0)


def test_shared_critic_update_struct_and_argument_checks(lib):
    assert ctypes.sizeof(_native.FlockScUpdate) == lib.flock_sc_update_size()
    n = lib.flock_sc_workspace_floats(256, 4, 2, 400, 300)
    assert n >= 256 * (11 * 400 + 14 * 300) and n % 64 == 0
    u = _native.FlockScUpdate(B=16, in_dim=4, n_actions=2, fc1=32, fc2=24, do_adam=1)
    assert lib.flock_sc_critic_update(None, ctypes.byref(u)) == -3  # NULL pointers
    assert lib.flock_sc_actor_update(None, None) == -3
    u.fc1 = 2048
    assert lib.flock_sc_critic_update(None, ctypes.byref(u)) == -2  # beyond the row-kernel limits
    assert "fc1/fc2 <= 1024" in lib.flock_learn_last_error().decode()


def test_shared_critic_round_and_pipeline_argument_checks(lib):
    assert lib.flock_sc_round(None, None, None) == -3
    u = _native.FlockScUpdate(B=16, in_dim=4, n_actions=2, fc1=32, fc2=24, do_adam=1)
    assert lib.flock_sc_round(None, ctypes.byref(u), None) == -3  # NULL pointers, checked before any launch
    rows = _native.FlockScRows()
    assert not lib.flock_sc_pipeline_create(1, ctypes.byref(u), ctypes.byref(rows), ctypes.byref(rows))
    assert "n_slots" in lib.flock_learn_last_error().decode()
    assert lib.flock_sc_pipeline_flush(None, None) == -3
    assert lib.flock_sc_pipeline_mark(None, None, 1) == -3
    assert lib.flock_sc_pipeline_gated_learns(None) == 0
    assert lib.flock_sc_pipeline_comm_stream(None) is None
    assert lib.flock_sc_pipeline_learn(None, None, None, 1, 0, 0, 0) == -3
    assert lib.flock_sc_pipeline_set_dp(None, None, 0, 0, 0, None, None, None) == -3


def test_step_ext_layout_and_launches_option():
    """FlockStepExt mirrors the header ({ring*, seeds*, int launches, int normalize_distance}: 24 bytes on x86-64);
    step_launches < 1 is rejected by FlockConfig and by the ext builder before any launch."""
    from marl_range_flocking_amd import FlockConfig, _native, ops

    assert ctypes.sizeof(_native.FlockStepExt) == 24
    assert [f[0] for f in _native.FlockStepExt._fields_] == ["ring", "seeds", "launches", "normalize_distance"]
    header = open(os.path.join(INCLUDE, "flock_amd.h")).read()
    body = header[header.index("typedef struct FlockStepExt"):header.index("} FlockStepExt;")]
    assert "int launches;" in body and body.index("int launches;") < body.index("int normalize_distance;")
    with pytest.raises(ValueError):
        FlockConfig(step_launches=0).resolved()
    with pytest.raises(ValueError):
        ops._ext(launches=0)
    assert ops._ext() is None and ops._ext(launches=2).launches == 2
    assert ops._ext(normalize=True).normalize_distance == 1
