"""Drop-in for environments/gym_flock_uw_discrete.py (MultiAgentEnv :19-433): discrete actions index the
10-entry (linear, angular) mean dictionary (:59-75), N(mean, 0.1) noise (drawn in-kernel with Philox, or injected
through ``step(action, noise=...)`` for parity), unit-speed heading kinematics, Euclidean kNN, reward = collision
(-9) + alignment. One HIP launch per step (flock_step_uw_discrete); the reference's N per-agent ``int(act)`` host
syncs (:329-330) are gone.
"""
import torch

from marl_range_flocking_amd.spaces import Box, Discrete
from marl_range_flocking_amd.environments._base import SingleFlockEnv


class MultiAgentEnv(SingleFlockEnv):
    variant = "uw_discrete"

    def __init__(self, agents, k=4, collision_distance=3, normalize_distance=False, rigid_boundary=False,
                 range_start=(0, 100), sensor_range=7, max_linear_velocity=2.5, desired_distance=15, **kw):
        super().__init__(agents, k, collision_distance, normalize_distance, rigid_boundary, range_start,
                         sensor_range, max_linear_velocity, desired_distance, **kw)
        self.collision_temp = collision_distance
        self.action_dictionary = {i: list(v) for i, v in enumerate(
            [[0.2, -1.2], [0.2, -0.5], [0.2, 0], [0.2, 0.5], [0.2, 1.2],
             [0.6, -1.2], [0.6, -0.5], [0.6, 0], [0.6, 0.5], [0.6, 1.2]])}
        n = self.num_particles
        self.action_space = list(Discrete(self.k) for _ in range(n))                                   # :98
        self.observation_space = list(Box(low=0, high=self.sensor_range, shape=(self.k,)) for _ in range(n))  # :99

    def _obs(self):  # _computeObs :170-171
        return self._vec.dnn[0].clone()

    def step(self, action, dt=0.1, noise=None):
        a = torch.as_tensor(action).to(self.device).reshape(1, self.num_particles)
        # action_dictionary[int(act)] raises before any state changes (:329-330): check the ids first (this
        # single-env wrapper synchronises every step anyway; VecFlockEnv reports bad ids through its status flag)
        ids = a if a.dtype == torch.int64 else a.to(torch.int64)
        if bool(((ids < 0) | (ids >= len(self.action_dictionary))).any().item()):
            raise KeyError("action id outside the action dictionary (gym_flock_uw_discrete.py:329)")
        if noise is not None:
            noise = torch.as_tensor(noise, dtype=torch.float32).to(self.device).reshape(1, self.num_particles, 2)
        self._vec.step(a, noise=noise, dt=dt)
        status, all_done = self._vec.status.item(), bool(self._vec.any_done[0].item())
        if status & 1:
            self._vec.status.zero_()
            raise KeyError("action id outside the action dictionary (gym_flock_uw_discrete.py:329)")
        return self._obs(), self._vec.reward[0].reshape(-1, 1).clone(), (self._vec.done[0].clone(), all_done), {}
