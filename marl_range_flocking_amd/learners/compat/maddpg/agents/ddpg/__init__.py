"""maddpg package shim (reference import paths of learners/maddpg_shared_critic)."""
