from marl_range_flocking_amd.learners.dropin import SuperAgentFF as SuperAgent  # noqa: F401  (MADDPG.py:13)
