"""torch.ops.flock.*: the step / kNN / reset kernels as PyTorch custom ops (csrc/flock_torch.cpp, libflock_torch.so).

Schemas: every buffer an op writes is a mutable alias argument (``Tensor(a!)``); the ops return
nothing (``knn`` returns (dnn, nn_idx)), enqueue on the current HIP stream and never synchronise; Meta kernels make
them traceable (FakeTensor, torch.compile). ``load()`` loads the library once; there is no CPU implementation.

    torch.ops.flock.step_v2(pos, heading, action, vel, dnn, nn_idx, reward, done, any_done, seeds, k, box,
                            sensor_range, collision_distance, dt, v_min, v_max, periodic, rigid_boundary)
    torch.ops.flock.step_uw / step_uw_discrete / step_flock / knn / reset
"""
import os

import torch

from ._native import BUILD_DIR

LIB = os.path.join(BUILD_DIR, "libflock_torch.so")
_loaded = False


def load():
    """Load libflock_torch.so (registers torch.ops.flock); raises if it has not been built."""
    global _loaded
    if not _loaded:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} is missing: build it with python -m marl_range_flocking_amd.build")
        from . import _native

        _native.lib()  # libflock_amd.so first (libflock_torch.so links it through rpath $ORIGIN)
        torch.ops.load_library(LIB)
        _loaded = True
    return torch.ops.flock

