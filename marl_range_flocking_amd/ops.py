"""Torch-facing wrappers of the C ABI (include/flock_amd.h).

Each function checks device / dtype / shape / contiguity, passes raw device pointers and the current HIP stream to
libflock_amd.so and returns nothing (outputs are written into the tensors given). No host synchronisation happens
here. Errors mirror the reference: ``k + 1 > N`` raises ``RuntimeError("selected index k out of range")`` as
torch.topk does in gym_flock_v2.py:147.
"""
import ctypes

import torch

from . import _native

UWD_TABLE = ((0.2, -1.2), (0.2, -0.5), (0.2, 0.0), (0.2, 0.5), (0.2, 1.2),
             (0.6, -1.2), (0.6, -0.5), (0.6, 0.0), (0.6, 0.5), (0.6, 1.2))  # gym_flock_uw_discrete.py:59-75


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _need(t, name, dtype, shape, device):
    if t is None:
        raise ValueError(f"{name} is required")
    if t.device != device:
        raise ValueError(f"{name} must be on {device}, got {t.device}")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _opt(t, name, dtype, shape, device):
    if t is not None:
        _need(t, name, dtype, shape, device)


def _dims(pos):
    if pos.dim() != 3 or pos.shape[-1] != 2:
        raise ValueError(f"pos must be [E, N, 2], got {tuple(pos.shape)}")
    if pos.device.type != "cuda":
        raise RuntimeError("flock ops run on a HIP device only (no CPU fallback); got " + str(pos.device))
    return pos.shape[0], pos.shape[1], pos.device


def _check_k(N, k):
    if k < 1 or k + 1 > N:
        raise RuntimeError("selected index k out of range")


def flock_ring(ring, prev_obs):
    """The C ABI's FlockRing of a learner's StepRing (learners/core.py) for the launch-plan path: one ctypes struct
    per StepRing, updated in place (start / skip of the step, the previous observation buffer), so a StepPlan that
    recorded a pointer to it sees every step's values."""
    c = ring.__dict__.get("_flock_ring")
    if c is None:
        f, m = ring.fields, ring.meta
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        c = ring._flock_ring = _native.FlockRing(
            state=ptr(f[0]), action=ptr(f[1]), reward=ptr(f[2]), new_state=ptr(f[3]), terminal=ptr(f[4]),
            prev_obs=None, capacity=f[0].shape[0], start=0, skip=0, actor_state=ptr(ring.actor_state),
            actor_new_state=ptr(ring.actor_new_state), group=m[2], store_done=m[3], action_ids=m[4], env_done=m[5])
    c.start, c.skip = ring.meta[0], ring.meta[1]
    c.prev_obs = prev_obs.data_ptr()
    return c


def _ext(ring=None, seeds=None, E=0, N=0, k=0, dev=None, launches=1, normalize=False):
    """FlockStepExt for the *_ext entry points, or None when there is nothing extra."""
    launches = int(launches)
    if launches < 1:
        raise ValueError("launches must be >= 1")
    if ring is None and seeds is None and launches == 1 and not normalize:
        return None
    if seeds is not None:
        _need(seeds, "seeds", torch.int16, (E, N, k), dev)
    return _native.FlockStepExt(ring=ctypes.pointer(ring) if ring is not None else None,
                                seeds=_ptr(seeds) if seeds is not None else None, launches=launches,
                                normalize_distance=int(bool(normalize)))


class StepPlan:
    """A validated step launch over fixed buffers (VecFlockEnv allocates its state once, so every call with the
    same buffer parity passes the same pointers). The first call through a plan checks every tensor and records
    the argument tuple; later calls check only the per-call action tensor and substitute the stream, the action
    pointer, dt and (uw_discrete) the RNG offset: the Python cost of a step drops to about one ctypes call."""

    __slots__ = ("fn", "name", "args", "ext", "i_action", "i_dt", "i_rng", "ring")

    def __init__(self):
        self.fn = None
        self.ring = None

    def record(self, fn, name, args, ext, i_action, i_dt, i_rng=None):
        self.fn, self.name, self.args, self.ext = fn, name, list(args), ext
        self.i_action, self.i_dt, self.i_rng = i_action, i_dt, i_rng

    def launch(self, stream, action, dt, rng_offset=None):
        a = self.args
        a[0] = stream
        a[self.i_action] = ctypes.c_void_p(action.data_ptr())
        a[self.i_dt] = float(dt)
        if self.i_rng is not None:
            a[self.i_rng] = int(rng_offset) & (2**64 - 1)
        rc = self.fn(*a) if self.ext is None else self.fn(*a, ctypes.byref(self.ext))
        _native.check(rc, self.name)


def _planned(plan, pos, action, name, dtype, shape, dt, rng_offset=None):
    """Run a recorded plan (True) after checking the per-call action tensor, or return False."""
    if plan is None or plan.fn is None:
        return False
    _need(action, name, dtype, shape, pos.device)
    plan.launch(_stream(pos), action, dt, rng_offset)
    return True


def _record(plan, lib_fn, name, args, ext, i_action, i_dt, i_rng=None):
    if ext is None:
        _native.check(lib_fn(*args), name)
    else:
        _native.check(lib_fn(*args, ctypes.byref(ext)), name)
    if plan is not None:
        plan.record(lib_fn, name, args, ext, i_action, i_dt, i_rng)


def step_v2(pos, heading, action, vel, dnn, nn_idx, reward, done, any_done, *, k, box, sensor_range,
            collision_distance, dt=0.1, v_min=0.005, v_max=2.5, periodic=True, rigid_boundary=False, ring=None,
            seeds=None, plan=None, launches=1, normalize=False):
    """gym_flock_v2.MultiAgentEnv.step (gym_flock_v2.py:71-83) for E envs; pos/heading updated in place.
    ring (a _native.FlockRing): also write every transition into a replay ring in the same launch
    (flock_step_v2_store; the store_transitions that follows each step in train_flock.py).
    seeds ([E, N, k] int16, rw, optional): compact kNN search seeds (flock_step_v2_ext; see include/flock_amd.h).
    plan (StepPlan, optional): record / replay the validated launch over the same buffers; with a ring, the plan
    holds that FlockRing object (ReplayRing.step_slots updates one object in place) and serves only that ring."""
    if plan is not None and plan.ring is not ring:
        plan.fn = None  # recorded for another ring (or none): record again
    if _planned(plan, pos, action, "action", torch.float32, tuple(pos.shape), dt):
        return
    E, N, dev = _dims(pos)
    _check_k(N, k)
    f32 = torch.float32
    _need(pos, "pos", f32, (E, N, 2), dev)
    _need(heading, "heading", f32, (E, N), dev)
    _need(action, "action", f32, (E, N, 2), dev)
    _need(vel, "vel", f32, (E, N, 2), dev)
    _need(dnn, "dnn", f32, (E, N, k), dev)
    _opt(nn_idx, "nn_idx", torch.int64, (E, N, k), dev)
    _need(reward, "reward", f32, (E, N), dev)
    _need(done, "done", torch.bool, (E, N), dev)
    _need(any_done, "any_done", torch.bool, (E,), dev)
    args = (_stream(pos), E, N, k, float(box), float(sensor_range), float(collision_distance), float(dt),
            float(v_min), float(v_max), int(bool(periodic)), int(bool(rigid_boundary)), _ptr(pos), _ptr(heading),
            _ptr(action), _ptr(vel), _ptr(dnn), _ptr(nn_idx), _ptr(reward), _ptr(done), _ptr(any_done))
    ext = _ext(ring, seeds, E, N, k, dev, launches, normalize)
    L = _native.lib()
    _record(plan, L.flock_step_v2 if ext is None else L.flock_step_v2_ext,
            "flock_step_v2" if ext is None else "flock_step_v2_ext", args, ext, 14, 7)
    if plan is not None:
        plan.ring = ring  # a strong reference: the recorded ext points into it


def step_uw(pos, heading, prev_heading, action, mem_in, mem_out, vel, dnn, nn_idx, reward, done, any_done, *, k, box,
            sensor_range, collision_distance, dt=0.1, rigid_boundary=False, seeds=None, plan=None, launches=1,
            normalize=False):
    """gym_flock_uw.MultiAgentEnv.step (gym_flock_uw.py:69-81); mem_out = rolled 4-frame observation."""
    if _planned(plan, pos, action, "action", torch.float32, tuple(pos.shape), dt):
        return
    E, N, dev = _dims(pos)
    _check_k(N, k)
    f32 = torch.float32
    _need(pos, "pos", f32, (E, N, 2), dev)
    _need(heading, "heading", f32, (E, N), dev)
    _need(prev_heading, "prev_heading", f32, (E, N), dev)
    _need(action, "action", f32, (E, N, 2), dev)
    _need(mem_in, "mem_in", f32, (E, N, 4, k), dev)
    _need(mem_out, "mem_out", f32, (E, N, 4, k), dev)
    _need(vel, "vel", f32, (E, N, 2), dev)
    _need(dnn, "dnn", f32, (E, N, k), dev)
    _opt(nn_idx, "nn_idx", torch.int64, (E, N, k), dev)
    _need(reward, "reward", f32, (E, N), dev)
    _need(done, "done", torch.bool, (E, N), dev)
    _need(any_done, "any_done", torch.bool, (E,), dev)
    args = (_stream(pos), E, N, k, float(box), float(sensor_range), float(collision_distance), float(dt),
            int(bool(rigid_boundary)), _ptr(pos), _ptr(heading), _ptr(prev_heading), _ptr(action), _ptr(mem_in),
            _ptr(mem_out), _ptr(vel), _ptr(dnn), _ptr(nn_idx), _ptr(reward), _ptr(done), _ptr(any_done))
    ext = _ext(None, seeds, E, N, k, dev, launches, normalize)
    L = _native.lib()
    _record(plan, L.flock_step_uw if ext is None else L.flock_step_uw_ext,
            "flock_step_uw" if ext is None else "flock_step_uw_ext", args, ext, 12, 7)


def step_uw_discrete(pos, heading, prev_heading, action_id, noise, table, vel, dnn, nn_idx, reward, done, any_done,
                     status=None, *, k, box, sensor_range, collision_distance, dt=0.1, v_max=2.5, rigid_boundary=False,
                     noise_std=0.1, seed=0, rng_offset=0, seeds=None, plan=None, launches=1, ring=None,
                     normalize=False):
    """gym_flock_uw_discrete.MultiAgentEnv.step (gym_flock_uw_discrete.py:110-122). noise=None → in-kernel
    Philox N(0, noise_std) draws; otherwise noise [E,N,2] is added to the action-table means (parity mode).
    plan (StepPlan, optional; in-kernel noise only): record / replay the validated launch over the same buffers.
    ring (a _native.FlockRing with action_ids / env_done, VDNLearner.replay_slots): also write every env's team
    transition into the VDN replay ring in the same launch (memory.put, learners/vdn/train_flock.py:102)."""
    if plan is not None and plan.ring is not ring:
        plan.fn = None  # recorded for another ring (or none): record again
    if noise is None and _planned(plan, pos, action_id, "action_id", torch.int64, tuple(pos.shape[:2]), dt,
                                  rng_offset):
        return
    E, N, dev = _dims(pos)
    _check_k(N, k)
    f32 = torch.float32
    _need(pos, "pos", f32, (E, N, 2), dev)
    _need(heading, "heading", f32, (E, N), dev)
    _need(prev_heading, "prev_heading", f32, (E, N), dev)
    _need(action_id, "action_id", torch.int64, (E, N), dev)
    _opt(noise, "noise", f32, (E, N, 2), dev)
    if table.dim() != 2 or table.shape[1] != 2:
        raise ValueError("table must be [n_actions, 2]")
    _need(table, "table", f32, tuple(table.shape), dev)
    _need(vel, "vel", f32, (E, N, 2), dev)
    _need(dnn, "dnn", f32, (E, N, k), dev)
    _opt(nn_idx, "nn_idx", torch.int64, (E, N, k), dev)
    _need(reward, "reward", f32, (E, N), dev)
    _need(done, "done", torch.bool, (E, N), dev)
    _need(any_done, "any_done", torch.bool, (E,), dev)
    _opt(status, "status", torch.int32, (1,), dev)
    args = (_stream(pos), E, N, k, float(box), float(sensor_range), float(collision_distance), float(dt),
            float(v_max), int(bool(rigid_boundary)), _ptr(pos), _ptr(heading), _ptr(prev_heading), _ptr(action_id),
            _ptr(noise), float(noise_std), int(seed) & (2**64 - 1), int(rng_offset) & (2**64 - 1), _ptr(table),
            int(table.shape[0]), _ptr(vel), _ptr(dnn), _ptr(nn_idx), _ptr(reward), _ptr(done), _ptr(any_done),
            _ptr(status))
    ext = _ext(ring, seeds, E, N, k, dev, launches, normalize)
    L = _native.lib()
    _record(plan if noise is None else None, L.flock_step_uw_discrete if ext is None else L.flock_step_uw_discrete_ext,
            "flock_step_uw_discrete" if ext is None else "flock_step_uw_discrete_ext", args, ext, 13, 7, 17)
    if plan is not None and noise is None:
        plan.ring = ring  # a strong reference: the recorded ext points into it


def step_flock(pos, vel, action, mem_in, mem_out, dnn, nn_idx, reward, done, any_done, *, k, box, collision_distance,
               dt=0.1, rigid_boundary=False, seeds=None, plan=None, launches=1, normalize=False):
    """gym_flock.MultiAgentEnv.step (gym_flock.py:48-60); vel is the unit-velocity state (rw)."""
    if _planned(plan, pos, action, "action", torch.float32, tuple(pos.shape), dt):
        return
    E, N, dev = _dims(pos)
    _check_k(N, k)
    f32 = torch.float32
    _need(pos, "pos", f32, (E, N, 2), dev)
    _need(vel, "vel", f32, (E, N, 2), dev)
    _need(action, "action", f32, (E, N, 2), dev)
    _need(mem_in, "mem_in", f32, (E, N, 4, k), dev)
    _need(mem_out, "mem_out", f32, (E, N, 4, k), dev)
    _need(dnn, "dnn", f32, (E, N, k), dev)
    _opt(nn_idx, "nn_idx", torch.int64, (E, N, k), dev)
    _need(reward, "reward", f32, (E, N), dev)
    _need(done, "done", torch.bool, (E, N), dev)
    _need(any_done, "any_done", torch.bool, (E,), dev)
    args = (_stream(pos), E, N, k, float(box), float(collision_distance), float(dt), int(bool(rigid_boundary)),
            _ptr(pos), _ptr(vel), _ptr(action), _ptr(mem_in), _ptr(mem_out), _ptr(dnn), _ptr(nn_idx), _ptr(reward),
            _ptr(done), _ptr(any_done))
    ext = _ext(None, seeds, E, N, k, dev, launches, normalize)
    L = _native.lib()
    _record(plan, L.flock_step_flock if ext is None else L.flock_step_flock_ext,
            "flock_step_flock" if ext is None else "flock_step_flock_ext", args, ext, 10, 6)


def knn(pos, k, box, sensor_range=14.0, periodic=True, clamp=True, dnn=None, nn_idx=None):
    """kNN sensing only (gym_flock_v2.py:135-151 periodic, :155-175 Euclidean). Returns (dnn, nn_idx)."""
    E, N, dev = _dims(pos)
    _check_k(N, k)
    _need(pos, "pos", torch.float32, (E, N, 2), dev)
    if dnn is None:
        dnn = torch.empty((E, N, k), dtype=torch.float32, device=dev)
    if nn_idx is None:
        nn_idx = torch.empty((E, N, k), dtype=torch.int64, device=dev)
    _need(dnn, "dnn", torch.float32, (E, N, k), dev)
    _need(nn_idx, "nn_idx", torch.int64, (E, N, k), dev)
    rc = _native.lib().flock_knn(_stream(pos), E, N, k, float(box), float(sensor_range), int(bool(periodic)),
                                 int(bool(clamp)), _ptr(pos), _ptr(dnn), _ptr(nn_idx))
    _native.check(rc, "flock_knn")
    return dnn, nn_idx


VARIANT_IDS = {"v2": 0, "uw": 1, "uw_discrete": 2, "flock": 3}


def reset(variant, pos, dnn, *, k, range_start, box, sensor_range, check_distance, heading=None, prev_heading=None,
          vel=None, nn_idx=None, mem=None, valid=None, env_mask=None, rigid_boundary=False, max_attempts=64, seed=0,
          rng_offset=0, repair_rounds=0, normalize=False):
    """Device-side reset with bounded rejection sampling (reference reset() recursion, e.g. gym_flock_v2.py:85-108);
    repair_rounds > 0: envs whose every draw collided re-draw only their colliding agents (flock_reset_ext).
    normalize: normalize_distance=True (the collision check and observation on positions / max |p|; no repair)."""
    E, N, dev = _dims(pos)
    _check_k(N, k)
    f32 = torch.float32
    _need(pos, "pos", f32, (E, N, 2), dev)
    _need(dnn, "dnn", f32, (E, N, k), dev)
    _opt(heading, "heading", f32, (E, N), dev)
    _opt(prev_heading, "prev_heading", f32, (E, N), dev)
    _opt(vel, "vel", f32, (E, N, 2), dev)
    _opt(nn_idx, "nn_idx", torch.int64, (E, N, k), dev)
    _opt(mem, "mem", f32, (E, N, 4, k), dev)
    _opt(valid, "valid", torch.bool, (E,), dev)
    _opt(env_mask, "env_mask", torch.bool, (E,), dev)
    rc = _native.lib().flock_reset_ext2(
        _stream(pos), VARIANT_IDS[variant], E, N, k, float(range_start[0]), float(range_start[1]), float(box),
        float(sensor_range), float(check_distance), int(bool(rigid_boundary)), int(max_attempts),
        int(seed) & (2**64 - 1), int(rng_offset) & (2**64 - 1), _ptr(env_mask), _ptr(pos), _ptr(heading),
        _ptr(prev_heading), _ptr(vel), _ptr(dnn), _ptr(nn_idx), _ptr(mem), _ptr(valid), int(repair_rounds),
        int(bool(normalize)))
    _native.check(rc, "flock_reset_ext2")
