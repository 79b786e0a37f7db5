from marl_range_flocking_amd.learners.dropin import ReplayBufferVDN  # noqa: F401  (vdn/utils.py:7)
