"""Drop-in replacements for the reference's environments/ modules (same module and class names).

Put this directory on sys.path where the reference's ``environments/`` was and ``from gym_flock_v2 import
make_env`` (main.py:6) resolves here.
"""
