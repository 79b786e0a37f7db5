"""Loader for the HIP library (libflock_amd.so, C ABI in include/flock_amd.h).

There is no CPU fallback: if the library is missing or no HIP device is present, every op raises. Build it with
``python -c "import __graft_entry__ as g; g.build()"`` (or ``python -m marl_range_flocking_amd.build``).
"""
import ctypes
import os

PKG = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(PKG, "_build")
LIB_PATH = os.path.join(BUILD_DIR, "libflock_amd.so")

_c_void_p, _c_int, _c_float, _c_u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_uint64

# name -> argtypes (mirrors include/flock_amd.h exactly; checked by tests/test_abi.py)
SIGNATURES = {
    "flock_abi_version": [],
    "flock_last_error": [],
    "flock_step_v2": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float, _c_float, _c_float,
                      _c_int, _c_int] + [_c_void_p] * 9,
    "flock_step_uw": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float, _c_int]
                     + [_c_void_p] * 12,
    "flock_step_uw_discrete": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float, _c_float,
                               _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_float, _c_u64,
                               _c_u64, _c_void_p, _c_int] + [_c_void_p] * 7,
    "flock_step_flock": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_int] + [_c_void_p] * 10,
    "flock_knn": [_c_void_p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_int, _c_int] + [_c_void_p] * 3,
    "flock_reset": [_c_void_p, _c_int, _c_int, _c_int, _c_int, _c_float, _c_float, _c_float, _c_float, _c_float,
                    _c_int, _c_int, _c_u64, _c_u64] + [_c_void_p] * 9,
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
    "flock_gather_rows": [_c_void_p, ctypes.c_int64, ctypes.c_int64, _c_void_p, _c_void_p, _c_void_p],
    "flock_scatter_rows": [_c_void_p, ctypes.c_int64, ctypes.c_int64, _c_void_p, _c_void_p, _c_void_p],
}
RESTYPES = {"flock_last_error": ctypes.c_char_p, "flock_learn_last_error": ctypes.c_char_p}

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
