"""Drop-in for environments/gym_flock.py (MultiAgentEnv :18-221): acceleration actions on a unit-velocity state,
Euclidean kNN without range clamp, 4-frame observation memory, collision-only reward.
One HIP launch per step (flock_step_flock, include/flock_amd.h).
"""
from marl_range_flocking_amd.spaces import Box
from marl_range_flocking_amd.environments._base import SingleFlockEnv


class MultiAgentEnv(SingleFlockEnv):
    variant = "flock"

    def __init__(self, agents, k, collision_distance, normalize_distance=False, rigid_boundary=False,
                 range_start=(0, 30), **kw):
        super().__init__(agents, k, collision_distance, normalize_distance, rigid_boundary, range_start,
                         sensor_range=float("inf"), **kw)
        self.action_space = Box(low=-1, high=1, shape=(2,))                 # :40
        self.observation_space = Box(low=0, high=100, shape=(self.k + 2,))  # :41

    def _obs(self):  # _computeObs :86-89
        return self._vec.obs_memory[0].clone()

    def _action(self, action):
        return super()._action(action).float().reshape(self.num_particles, 2)
