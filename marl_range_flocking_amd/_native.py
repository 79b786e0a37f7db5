"""Loader for the HIP library (libflock_amd.so, C ABI in include/flock_amd.h).

There is no CPU fallback: if the library is missing or no HIP device is present, every op raises. Build it with
``python -c "import __graft_entry__ as g; g.build()"`` (or ``python -m marl_range_flocking_amd.build``).
"""
import ctypes
import os

PKG = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(PKG, "_build")
LIB_PATH = os.path.join(BUILD_DIR, "libflock_amd.so")  # A/B of builds: copy a variant over it (tools/gpu_ab_swap.sh)

_c_void_p, _c_int, _c_float, _c_u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_uint64

# name -> argtypes (mirrors include/flock_amd.h exactly; checked by tests/test_abi.py)
SIGNATURES = {
    "flock_abi_version": [],
    "flock_last_error": [],
    "flock_set_diag": [ctypes.c_char_p, _c_int],
    "flock_step_v2": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float, _c_float, _c_float,
                      _c_int, _c_int] + [_c_void_p] * 9,
    "flock_step_uw": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float, _c_int]
                     + [_c_void_p] * 12,
    "flock_step_uw_discrete": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float, _c_float,
                               _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_float, _c_u64,
                               _c_u64, _c_void_p, _c_int] + [_c_void_p] * 7,
    "flock_step_flock": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_int] + [_c_void_p] * 10,
    "flock_step_v2_ext": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float, _c_float,
                          _c_float, _c_int, _c_int] + [_c_void_p] * 10,
    "flock_step_uw_ext": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float, _c_int]
                         + [_c_void_p] * 13,
    "flock_step_uw_discrete_ext": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float,
                                   _c_float, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                   _c_float, _c_u64, _c_u64, _c_void_p, _c_int] + [_c_void_p] * 8,
    "flock_rollout_uw": [_c_void_p, _c_int, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float, _c_int]
                        + [_c_void_p] * 17,
    "flock_step_flock_ext": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_int]
                            + [_c_void_p] * 11,
    "flock_knn": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_int, _c_int] + [_c_void_p] * 3,
    "flock_reset": [_c_void_p, _c_int, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float, _c_float,
                    _c_int, _c_int, _c_u64, _c_u64] + [_c_void_p] * 9,
    "flock_reset_ext": [_c_void_p, _c_int, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float,
                        _c_float, _c_int, _c_int, _c_u64, _c_u64] + [_c_void_p] * 9 + [_c_int],
    "flock_reset_ext2": [_c_void_p, _c_int, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float,
                         _c_float, _c_int, _c_int, _c_u64, _c_u64] + [_c_void_p] * 9 + [_c_int, _c_int],
    # learner kernels (include/flock_learn.h)
    "flock_learn_last_error": [],
    "flock_adam_step": [_c_void_p, ctypes.c_int64] + [_c_void_p] * 5 + [_c_float] * 4 + [ctypes.c_int64, _c_void_p,
                                                                                      _c_float, _c_int],
    "flock_adam_step_dev": [_c_void_p, ctypes.c_int64] + [_c_void_p] * 5 + [_c_float] * 4 + [_c_void_p, _c_void_p,
                                                                                          _c_float, _c_int],
    "flock_soft_update": [_c_void_p, ctypes.c_int64, _c_void_p, _c_void_p, _c_float, _c_int],
    "flock_grad_norm": [_c_void_p, ctypes.c_int64, _c_void_p, _c_void_p, _c_int, _c_float, _c_void_p],
    "flock_gru_fwd": [_c_void_p, ctypes.c_int64, _c_int] + [_c_void_p] * 5,
    "flock_gru_bwd": [_c_void_p, ctypes.c_int64, _c_int] + [_c_void_p] * 6,
    "flock_vdn_feat_fwd": [_c_void_p, _c_int, _c_int, _c_int, _c_int, _c_void_p] + [ctypes.c_int64] * 3
                          + [_c_void_p] * 9,
    "flock_vdn_feat_bwd": [_c_void_p, _c_int, _c_int, _c_int, _c_int, _c_void_p] + [ctypes.c_int64] * 3
                          + [_c_void_p] * 11,
    "flock_gru_seq_fwd": [_c_void_p, _c_int, _c_int, _c_int, _c_int] + [_c_void_p] * 4 + [ctypes.c_int64] * 3
    + [_c_void_p] * 2,
    "flock_gru_seq_bwd": [_c_void_p, _c_int, _c_int, _c_int, _c_int] + [_c_void_p] * 5 + [ctypes.c_int64] * 3
    + [_c_void_p] * 3,
    "flock_gru_seq_q_fwd": [_c_void_p] + [_c_int] * 5 + [_c_void_p] * 6 + [ctypes.c_int64] * 3 + [_c_void_p] * 3,
    "flock_gru_seq_q_bwd": [_c_void_p] + [_c_int] * 5 + [_c_void_p] * 6 + [ctypes.c_int64] * 3 + [_c_void_p] * 5,
    "flock_gather_rows": [_c_void_p, ctypes.c_int64, ctypes.c_int64, _c_void_p, _c_void_p, _c_void_p],
    "flock_scatter_rows": [_c_void_p, ctypes.c_int64, ctypes.c_int64, _c_void_p, _c_void_p, _c_void_p],
}


class FlockScRows(ctypes.Structure):
    """Mirror of ``FlockScRows`` (include/flock_learn.h): replay fields of a ring or of its minibatch snapshot."""

    _fields_ = [(n, _c_void_p) for n in ("state", "new_state", "action", "reward", "terminal")]


class FlockScUpdate(ctypes.Structure):
    """Mirror of ``FlockScUpdate`` (include/flock_learn.h): all pointers are device pointers."""

    _fields_ = ([(n, _c_int) for n in ("B", "in_dim", "n_actions", "fc1", "fc2", "do_adam")]
                + [(n, _c_void_p) for n in ("idx", "agent", "ring_state", "ring_new_state", "ring_action",
                                            "ring_reward", "ring_terminal", "critic", "critic_grad",
                                            "critic_exp_avg", "critic_exp_avg_sq", "critic_step", "actors",
                                            "actors_grad", "actors_exp_avg", "actors_exp_avg_sq", "actors_target",
                                            "actor_steps")]
                + [("actor_stride", ctypes.c_int64)]
                + [(n, _c_void_p) for n in ("losses", "workspace", "counters")]
                + [(n, _c_float) for n in ("alpha", "beta", "gamma", "beta1", "beta2", "eps", "tau")]
                + [("update_rate", _c_int), ("critic_view", _c_void_p), ("actor_grad_out", _c_void_p)])


def sc_update(learner, job, dims, hyper):
    """The FlockScUpdate of a torch.ops.flock.sc_round argument list (learner state [13], job [9 or 10], dims [7],
    hyper [7]; csrc/flock_torch_sc.h), for callers of the C ABI (the op-vs-C-ABI tests)."""
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None and t.numel() else None  # noqa: E731
    L = learner
    B, n_in, na, fc1, fc2, rate, do_adam = dims
    u = FlockScUpdate(B=B, in_dim=n_in, n_actions=na, fc1=fc1, fc2=fc2, do_adam=do_adam, idx=p(job[0]),
                      agent=p(job[1]), ring_state=p(job[2]), ring_new_state=p(job[3]), ring_action=p(job[4]),
                      ring_reward=p(job[5]), ring_terminal=p(job[6]), critic=p(L[0]), critic_grad=p(L[1]),
                      critic_exp_avg=p(L[2]), critic_exp_avg_sq=p(L[3]), critic_step=p(L[4]), actors=p(L[5]),
                      actors_grad=p(L[6]), actors_exp_avg=p(L[7]), actors_exp_avg_sq=p(L[8]), actors_target=p(L[9]),
                      actor_steps=p(L[10]), actor_stride=L[5].numel() // L[10].numel(), losses=p(L[11]),
                      workspace=p(job[7]), counters=p(L[12]), update_rate=rate, critic_view=p(job[8]),
                      actor_grad_out=p(job[9]) if len(job) > 9 else None)
    for n, v in zip(("alpha", "beta", "gamma", "beta1", "beta2", "eps", "tau"), hyper):
        setattr(u, n, v)
    return u


def sc_rows(rows):
    """FlockScRows of [state, new_state, action, reward, terminal] tensors."""
    return FlockScRows(*[ctypes.c_void_p(t.data_ptr()) for t in rows])


class FlockRingField(ctypes.Structure):
    """Mirror of ``FlockRingField`` (include/flock_learn.h)."""

    _fields_ = [("src", _c_void_p), ("dst", _c_void_p), ("width", ctypes.c_int64), ("kind", _c_int)]


class FlockRing(ctypes.Structure):
    """Mirror of ``FlockRing`` (include/flock_amd.h): replay-ring targets of flock_step_v2_store."""

    _fields_ = ([(n, _c_void_p) for n in ("state", "action", "reward", "new_state", "terminal", "prev_obs")]
                + [("capacity", ctypes.c_int64), ("start", ctypes.c_int64), ("skip", ctypes.c_int64)]
                + [("actor_state", _c_void_p), ("actor_new_state", _c_void_p), ("group", ctypes.c_int64),
                   ("store_done", _c_int), ("action_ids", _c_int), ("env_done", _c_int)])


class FlockStepExt(ctypes.Structure):
    """Mirror of ``FlockStepExt`` (include/flock_amd.h): optional extras of the *_ext step entry points."""

    _fields_ = [("ring", ctypes.POINTER(FlockRing)), ("seeds", _c_void_p), ("launches", _c_int),
                ("normalize_distance", _c_int)]


for _name in ("flock_step_v2_ext", "flock_step_uw_ext", "flock_step_uw_discrete_ext", "flock_step_flock_ext"):
    SIGNATURES[_name] = SIGNATURES[_name][:-1] + [ctypes.POINTER(FlockStepExt)]

SIGNATURES.update({
    "flock_step_v2_store": SIGNATURES["flock_step_v2"] + [ctypes.POINTER(FlockRing)],
    "flock_ring_store": [_c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _c_int,
                         ctypes.POINTER(FlockRingField)],
    "flock_sc_workspace_floats": [_c_int] * 5,
    "flock_sc_update_size": [],
    "flock_sc_prep_snapshot": [_c_void_p, _c_int, ctypes.c_int64, _c_u64, _c_u64, _c_void_p, _c_void_p,
                               ctypes.c_int64, _c_int, _c_int, _c_void_p, _c_void_p],
    "flock_sc_prep": [_c_void_p, _c_int, ctypes.c_int64, _c_u64, _c_u64, _c_void_p, _c_void_p, ctypes.c_int64],
    "flock_sc_act": [_c_void_p, ctypes.c_int64, _c_int, _c_int, _c_int, _c_int, _c_void_p, _c_void_p, ctypes.c_int64,
                     _c_void_p, _c_void_p, _c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_float],
    "flock_sc_critic_update": [_c_void_p, ctypes.POINTER(FlockScUpdate)],
    "flock_sc_actor_update": [_c_void_p, ctypes.POINTER(FlockScUpdate)],
    "flock_sc_round": [_c_void_p, ctypes.POINTER(FlockScUpdate), ctypes.POINTER(FlockScUpdate)],
    "flock_sc_round_adam": [_c_void_p, ctypes.POINTER(FlockScUpdate), ctypes.POINTER(FlockScUpdate), _c_void_p],
    "flock_sc_pipeline_create": [_c_int, ctypes.POINTER(FlockScUpdate), ctypes.POINTER(FlockScRows),
                                 ctypes.POINTER(FlockScRows)],
    "flock_sc_pipeline_learn": [_c_void_p] * 3 + [ctypes.c_int64, _c_u64, _c_u64, ctypes.c_int64],
    "flock_sc_pipeline_flush": [_c_void_p, _c_void_p],
    "flock_sc_pipeline_set_gate": [_c_void_p, _c_int],
    "flock_sc_pipeline_mark": [_c_void_p, _c_void_p, _c_int],
    "flock_sc_pipeline_comm_stream": [_c_void_p],
    "flock_sc_pipeline_gated_learns": [_c_void_p],
    "flock_sc_pipeline_check": [_c_void_p],
    "flock_sc_pipeline_gated": [_c_void_p],
    "flock_sc_pipeline_set_dp": [_c_void_p, _c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _c_void_p,
                                 _c_void_p, _c_void_p],
    "flock_sc_pipeline_set_dp_actor": [_c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p],
    "flock_sc_pipeline_destroy": [_c_void_p],
})
RESTYPES = {"flock_last_error": ctypes.c_char_p, "flock_learn_last_error": ctypes.c_char_p,
            "flock_sc_workspace_floats": ctypes.c_int64, "flock_sc_update_size": ctypes.c_int64,
            "flock_sc_pipeline_create": _c_void_p, "flock_sc_pipeline_destroy": None,
            "flock_sc_pipeline_comm_stream": _c_void_p, "flock_sc_pipeline_gated_learns": ctypes.c_int64}

_lib = None


class FlockNativeError(RuntimeError):
    pass


def lib():
    """The loaded library with argtypes set. Raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FlockNativeError(
                f"HIP library not built: {LIB_PATH} is missing. Run "
                "`python -c \"import __graft_entry__ as g; g.build()\"` (hipcc --offload-arch=gfx950).")
        L = ctypes.CDLL(LIB_PATH)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = argtypes
            fn.restype = RESTYPES.get(name, ctypes.c_int)
        _lib = L
    return _lib


def check(rc: int, what: str, learn: bool = False):
    if rc != 0:
        msg = (lib().flock_learn_last_error() if learn else lib().flock_last_error()).decode()
        raise RuntimeError(f"{what}: {msg} (code {rc})")
