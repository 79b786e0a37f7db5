from marl_range_flocking_amd.learners.dropin import OUActionNoiseGPU, ReplayBuffer  # noqa: F401  (utils.py:6,28)
