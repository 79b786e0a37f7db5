from marl_range_flocking_amd.learners.dropin import vdn_train as train  # noqa: F401  (vdn/train_flock.py:16)
