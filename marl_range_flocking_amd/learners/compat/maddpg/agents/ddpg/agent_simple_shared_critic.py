from marl_range_flocking_amd.learners.dropin import Agent  # noqa: F401  (agent_simple_shared_critic.py:14)
