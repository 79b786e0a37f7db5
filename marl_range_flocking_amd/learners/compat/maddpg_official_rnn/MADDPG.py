from marl_range_flocking_amd.learners.dropin import SuperAgent  # noqa: F401  (MADDPG.py:13, recurrent)
