"""ctypes front-end of the C oracle (oracle/flock_oracle.c). TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this module, and only as the
checker / the timed CPU port. The product path (marl_range_flocking_amd) never imports it.

All functions take and return numpy arrays with a leading env axis E (see flock_oracle.c for layouts), copy their
inputs (the C code updates state in place) and return a dict of the post-step state and outputs.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libflock_oracle.so")

# action dictionary of gym_flock_uw_discrete.py:59-75 (linear, angular means)
UWD_TABLE = np.array([[0.2, -1.2], [0.2, -0.5], [0.2, 0.0], [0.2, 0.5], [0.2, 1.2],
                      [0.6, -1.2], [0.6, -0.5], [0.6, 0.0], [0.6, 0.5], [0.6, 1.2]], dtype=np.float32)

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
    return _lib


def _f(x):
    return np.ascontiguousarray(x, dtype=np.float32)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


_I, _F = ctypes.c_int, ctypes.c_float


class _normalized:
    """normalize_distance=True around one oracle call (oracle_set_normalize; the C switch is process-global)."""

    def __init__(self, on):
        self.on = bool(on)

    def __enter__(self):
        lib().oracle_set_normalize(_I(int(self.on)))

    def __exit__(self, *exc):
        lib().oracle_set_normalize(_I(0))


def knn(pos, k, box, sensor_range=14.0, periodic=True, clamp=True, normalize=False):
    pos = _f(pos)
    E, N = pos.shape[:2]
    dnn = np.zeros((E, N, k), np.float32)
    idx = np.zeros((E, N, k), np.int64)
    with _normalized(normalize):
        rc = lib().oracle_knn(_I(E), _I(N), _I(k), _F(box), _F(sensor_range), _I(int(periodic)), _I(int(clamp)),
                              _p(pos), _p(dnn), _p(idx))
    if rc != 0:
        raise RuntimeError("selected index k out of range")
    return dnn, idx


def _outs(E, N, k):
    return dict(vel=np.zeros((E, N, 2), np.float32), dnn=np.zeros((E, N, k), np.float32),
                idx=np.zeros((E, N, k), np.int64), reward=np.zeros((E, N), np.float32),
                done=np.zeros((E, N), np.uint8), any_done=np.zeros((E,), np.uint8))


def step_v2(pos, heading, action, *, k, box, sensor_range=14.0, cd=2.5, dt=0.1, v_min=0.005, v_max=2.5,
            periodic=True, rigid=False, normalize=False):
    pos, heading, action = _f(pos).copy(), _f(heading).copy(), _f(action)
    E, N = heading.shape
    o = _outs(E, N, k)
    with _normalized(normalize):
        rc = lib().oracle_step_v2(_I(E), _I(N), _I(k), _F(box), _F(sensor_range), _F(cd), _F(dt), _F(v_min),
                              _F(v_max), _I(int(periodic)), _I(int(rigid)), _p(pos), _p(heading), _p(action),
                              _p(o["vel"]), _p(o["dnn"]), _p(o["idx"]), _p(o["reward"]), _p(o["done"]),
                              _p(o["any_done"]))
    if rc != 0:
        raise RuntimeError("selected index k out of range")
    o.update(pos=pos, heading=heading)
    return o


def step_uw(pos, heading, prev_heading, action, mem, *, k, box, sensor_range=14.0, cd=2.5, dt=0.1, rigid=False,
            normalize=False):
    pos, heading, prev = _f(pos).copy(), _f(heading).copy(), _f(prev_heading).copy()
    action, mem = _f(action), _f(mem)
    E, N = heading.shape
    o = _outs(E, N, k)
    mem_out = np.zeros((E, N, 4, k), np.float32)
    with _normalized(normalize):
        rc = lib().oracle_step_uw(_I(E), _I(N), _I(k), _F(box), _F(sensor_range), _F(cd), _F(dt), _I(int(rigid)),
                              _p(pos), _p(heading), _p(prev), _p(action), _p(mem), _p(mem_out), _p(o["vel"]),
                              _p(o["dnn"]), _p(o["idx"]), _p(o["reward"]), _p(o["done"]), _p(o["any_done"]))
    if rc != 0:
        raise RuntimeError("selected index k out of range")
    o.update(pos=pos, heading=heading, prev_heading=prev, obs=mem_out)
    return o


def step_uwd(pos, heading, prev_heading, action, noise, *, k, box, sensor_range=14.0, cd=3.0, dt=0.1, v_max=2.5,
             rigid=False, table=UWD_TABLE, normalize=False):
    pos, heading, prev = _f(pos).copy(), _f(heading).copy(), _f(prev_heading).copy()
    action = np.ascontiguousarray(action, dtype=np.int64)
    noise, table = _f(noise), _f(table)
    E, N = heading.shape
    o = _outs(E, N, k)
    with _normalized(normalize):
        rc = lib().oracle_step_uwd(_I(E), _I(N), _I(k), _F(box), _F(sensor_range), _F(cd), _F(dt), _F(v_max),
                               _I(int(rigid)), _p(pos), _p(heading), _p(prev), _p(action), _p(noise), _p(table),
                               _I(table.shape[0]), _p(o["vel"]), _p(o["dnn"]), _p(o["idx"]), _p(o["reward"]),
                               _p(o["done"]), _p(o["any_done"]))
    if rc == -2:
        raise KeyError("action id outside the action dictionary")
    if rc != 0:
        raise RuntimeError("selected index k out of range")
    o.update(pos=pos, heading=heading, prev_heading=prev, obs=o["dnn"])
    return o


def step_flock(pos, vel, action, mem, *, k, box, cd=2.5, dt=0.1, rigid=False, normalize=False):
    pos, vel, action, mem = _f(pos).copy(), _f(vel).copy(), _f(action), _f(mem)
    E, N = pos.shape[:2]
    o = _outs(E, N, k)
    mem_out = np.zeros((E, N, 4, k), np.float32)
    with _normalized(normalize):
        rc = lib().oracle_step_flock(_I(E), _I(N), _I(k), _F(box), _F(cd), _F(dt), _I(int(rigid)), _p(pos), _p(vel),
                                 _p(action), _p(mem), _p(mem_out), _p(o["dnn"]), _p(o["idx"]), _p(o["reward"]),
                                 _p(o["done"]), _p(o["any_done"]))
    if rc != 0:
        raise RuntimeError("selected index k out of range")
    o.update(pos=pos, vel=vel, obs=mem_out)
    return o
