from marl_range_flocking_amd.learners.dropin import CriticNetwork  # noqa: F401  (ddpg_network.py:11)
