"""marl_range_flocking_amd — MI355X-native batched flocking-env stepper and MARL learner updates.

Hot path: libflock_amd.so (hand-written HIP for gfx950, C ABI in include/flock_amd.h), driven from Python through
ctypes. ``VecFlockEnv`` is the batched engine; ``environments/`` holds the drop-in gym surfaces of the reference.
"""
from .vec_env import FlockConfig, VecFlockEnv  # noqa: F401

__all__ = ["FlockConfig", "VecFlockEnv"]
