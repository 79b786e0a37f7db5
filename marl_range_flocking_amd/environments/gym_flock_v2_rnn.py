"""Drop-in for the fork learners/maddpg_official_rnn/gym_flock_v2.py (the env main.py resolves when the RNN learner
directory is first on sys.path): step uses Euclidean _computeDistances (:75) and the linear speed is
clamped to [0.5, max_linear_velocity] (:310). Everything else is gym_flock_v2.
"""
from marl_range_flocking_amd.environments import gym_flock_v2 as _v2


class MultiAgentEnv(_v2.MultiAgentEnv):
    def __init__(self, *args, **kw):
        kw.setdefault("periodic", False)
        kw.setdefault("v_min", 0.5)
        super().__init__(*args, **kw)


def make_env(args) -> MultiAgentEnv:
    return MultiAgentEnv(agents=args.nb_agents, k=args.k, collision_distance=args.collision_distance,
                         normalize_distance=False, range_start=args.range_start, sensor_range=args.sensor_range)
