"""Drop-in for environments/gym_flock_v2.py (MultiAgentEnv :20-415, make_env :418-429).

Same constructor, spaces, attributes and step/reset return types; the step runs as one HIP launch
(flock_step_v2, include/flock_amd.h). ``periodic`` / ``v_min`` select the learners/maddpg_official_rnn fork
(Euclidean distances, linear-speed floor 0.5) — see gym_flock_v2_rnn.py.
"""
from marl_range_flocking_amd.spaces import Box
from marl_range_flocking_amd.environments._base import SingleFlockEnv


class MultiAgentEnv(SingleFlockEnv):
    variant = "v2"

    def __init__(self, agents, k, collision_distance, normalize_distance=False, rigid_boundary=False,
                 range_start=(0, 100), sensor_range=7, max_linear_velocity=2.5, desired_distance=15, **kw):
        super().__init__(agents, k, collision_distance, normalize_distance, rigid_boundary, range_start,
                         sensor_range, max_linear_velocity, desired_distance, **kw)
        n = self.num_particles
        self.action_space = list(Box(low=-1.5, high=1.5, shape=(2,)) for _ in range(n))  # :58
        self.observation_space = [Box(low=0, high=range_start[1], shape=(n, self.k)),
                                  list(Box(low=0, high=range_start[1], shape=(self.k,)) for _ in range(n))]  # :60

    def _obs(self):  # _computeObs :127-133 — two independent copies, as the reference clones twice
        d = self._vec.dnn[0]
        return {"critic": d.clone(), "actors": d.clone()}

    def _action(self, action):
        return super()._action(action).float().reshape(self.num_particles, 2)


def make_env(args) -> MultiAgentEnv:
    """gym_flock_v2.py:418-429 (normalize_distance forced False, rigid_boundary default, as there)."""
    return MultiAgentEnv(agents=args.nb_agents, k=args.k, collision_distance=args.collision_distance,
                         normalize_distance=False, range_start=args.range_start, sensor_range=args.sensor_range)
