from marl_range_flocking_amd.learners.dropin import QNet  # noqa: F401  (vdn/net.py:11)
