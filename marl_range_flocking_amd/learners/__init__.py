"""Batched-over-agents MARL learner updates (shared-critic DDPG, recurrent VDN, MADDPG RNN / feed-forward)."""
