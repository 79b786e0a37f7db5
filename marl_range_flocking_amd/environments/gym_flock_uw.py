"""Drop-in for environments/gym_flock_uw.py (MultiAgentEnv :19-369): velocity actions normalised to unit speed,
Euclidean kNN, 4-frame observation memory (N, 4, k), reward = collision + centre of mass + angular terms.
One HIP launch per step (flock_step_uw, include/flock_amd.h).
"""
from marl_range_flocking_amd.spaces import Box
from marl_range_flocking_amd.environments._base import SingleFlockEnv


class MultiAgentEnv(SingleFlockEnv):
    variant = "uw"

    def __init__(self, agents, k, collision_distance, normalize_distance=False, rigid_boundary=False,
                 range_start=(0, 100), sensor_range=7, max_linear_velocity=2.5, desired_distance=15, **kw):
        super().__init__(agents, k, collision_distance, normalize_distance, rigid_boundary, range_start,
                         sensor_range, max_linear_velocity, desired_distance, **kw)
        self.action_space = Box(low=-1, high=1, shape=(2,))                 # :57
        self.observation_space = Box(low=0, high=100, shape=(self.k + 2,))  # :58 (sic: the obs is (N, 4, k))

    def _obs(self):  # _computeObs :120-123 (roll + insert); a snapshot, as copy() of the rolled tensor is
        return self._vec.obs_memory[0].clone()

    def _action(self, action):
        return super()._action(action).float().reshape(self.num_particles, 2)
