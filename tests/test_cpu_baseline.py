"""The timed CPU baseline (oracle/torch_ref.py): the torch-CPU restatement of the reference's
gym_flock_v2 step must reproduce the reference's own golden vectors (tests/golden/env_v2_*.npz, made by running
environments/gym_flock_v2.py here), so the number bench.py reports beside the GPU is the reference's computation;
the calibration record (tests/golden/cpu_calibration.json, oracle/calibrate_cpu.py) states its speed against the
reference itself."""
import glob
import json
import os

import numpy as np
import pytest
import torch

from oracle.torch_ref import V2Env

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "env_v2_N*.npz"))),
                         ids=lambda p: os.path.basename(p)[:-4])
def test_torch_ref_matches_reference_teacher_forced(path):
    z = np.load(path)
    m = json.loads(str(z["meta"]))
    for e in range(m["E"]):
        for t in range(m["T"]):
            pos0 = z["pos0"][e] if t == 0 else z["pos"][t - 1, e]
            head0 = z["head0"][e] if t == 0 else z["head"][t - 1, e]
            env = V2Env(pos0, head0, k=m["k"], box=m["box"], sensor_range=m["sensor_range"],
                        collision_distance=m["collision_distance"])
            obs, rew, (done, all_done), _ = env.step(torch.from_numpy(z["actions"][t, e]), dt=m["dt"])
            np.testing.assert_allclose(env.positions.numpy(), z["pos"][t, e], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(env.headings.numpy(), z["head"][t, e], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(obs["actors"].numpy(), z["dnn"][t, e], rtol=1e-5, atol=1e-6)
            # the restatement ran on the reference's own post-step positions: indices equal up to exact ties
            same = env.nearest_neighbors.numpy() == z["nn_idx"][t, e]
            assert same.mean() > 0.99
            np.testing.assert_array_equal(rew.numpy()[:, 0], z["reward"][t, e])
            np.testing.assert_array_equal(done.numpy(), z["done"][t, e])
            assert all_done == bool(z["any_done"][t, e])


def test_calibration_record_is_present():
    c = json.load(open(os.path.join(GOLD, "cpu_calibration.json")))
    assert c["rows"] and all(0.5 < r["ratio_restatement_over_reference"] < 2.0 for r in c["rows"])
