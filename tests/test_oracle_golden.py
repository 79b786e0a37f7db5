"""Pin the CPU oracle (oracle/flock_oracle.c) against golden vectors produced by the reference itself.

Fixtures: tests/golden/env_*.npz, sense_*.npz, errors.json (generator: tests/golden/gen_golden_env.py, which imports
/root/reference on torch CPU). Each step is teacher-forced: the oracle steps from the reference's own state at t-1,
so every step is compared without accumulated drift; a free-running rollout is checked separately.
"""
import glob
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from parity import RTOL, allclose_rel, d2_rows, knn_mismatch, knn_positions, meta

GOLD = os.path.join(os.path.dirname(__file__), "golden")
ENV_FIXTURES = sorted(glob.glob(os.path.join(GOLD, "env_*.npz")))


def oracle_step(m, z, t, pos, head, prev, vel, mem):
    v, k = m["variant"], m["k"]
    kw = dict(k=k, box=m["box"], cd=m["collision_distance"], normalize=m.get("normalize_distance", False))
    if v in ("v2", "v2fork"):
        return O.step_v2(pos, head, z["actions"][t], sensor_range=m["sensor_range"], v_min=m["v_min"],
                         periodic=(v == "v2"), **kw)
    if v == "uw":
        return O.step_uw(pos, head, prev, z["actions"][t], mem, sensor_range=m["sensor_range"], **kw)
    if v == "uwd":
        return O.step_uwd(pos, head, prev, z["actions"][t], z["noise"][t], sensor_range=m["sensor_range"], **kw)
    return O.step_flock(pos, vel, z["actions"][t], mem, **kw)


@pytest.mark.parametrize("path", ENV_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_matches_reference_teacher_forced(path):
    z = np.load(path)
    m = meta(z)
    v = m["variant"]
    pos, head, prev, vel, mem = z["pos0"], z["head0"], z["prevh0"], z["vel0"], z["mem0"]
    for t in range(m["T"]):
        o = oracle_step(m, z, t, pos, head, prev, vel, mem)
        ok, err = allclose_rel(o["pos"], z["pos"][t])
        assert ok, f"t={t} positions rel err {err}"
        ok, err = allclose_rel(o["vel"], z["vel"][t], atol=1e-12)
        assert ok, f"t={t} velocities rel err {err}"
        if v != "flock":
            ok, err = allclose_rel(o["heading"], z["head"][t])
            assert ok, f"t={t} headings rel err {err}"
        ok, err = allclose_rel(o["dnn"], z["dnn"][t], atol=1e-12)
        assert ok, f"t={t} dnn rel err {err}"
        if v in ("v2", "v2fork"):
            D = d2_rows(knn_positions(z["pos"][t], m), m["box"], periodic=(v == "v2"))
            _, _, bad = knn_mismatch(z["nn_idx"][t], o["idx"], D)
            assert not bad, f"t={t} neighbour indices differ beyond ties at rows {bad[:5]}"
        np.testing.assert_array_equal(o["reward"], z["reward"][t])
        np.testing.assert_array_equal(o["done"].astype(bool), z["done"][t])
        np.testing.assert_array_equal(o["any_done"].astype(bool), z["any_done"][t])
        if v in ("uw", "flock"):
            ok, err = allclose_rel(o["obs"], z["obs"][t], atol=1e-12)
            assert ok, f"t={t} obs memory rel err {err}"
        if v in ("uw", "uwd"):
            np.testing.assert_array_equal(o["prev_heading"], z["prevh"][t])
        # teacher forcing: continue from the reference's state
        pos, head, vel, prev = z["pos"][t], z["head"][t], z["vel"][t], z["prevh"][t]
        if v in ("uw", "flock"):
            mem = z["obs"][t]


@pytest.mark.parametrize("path", [p for p in ENV_FIXTURES if "_N8_" in p], ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_free_running_20_steps(path):
    """No teacher forcing: 20 chained steps (config-1 length) stay within tolerance of the reference."""
    z = np.load(path)
    m = meta(z)
    v = m["variant"]
    pos, head, prev, vel, mem = z["pos0"], z["head0"], z["prevh0"], z["vel0"], z["mem0"]
    for t in range(m["T"]):
        o = oracle_step(m, z, t, pos, head, prev, vel, mem)
        pos, vel = o["pos"], o["vel"]
        head = o.get("heading", head)
        prev = o.get("prev_heading", prev)
        if v in ("uw", "flock"):
            mem = o["obs"]
    ok, err = allclose_rel(pos, z["pos"][-1], rtol=1e-4)
    assert ok, f"free-running drift {err}"


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "sense_*.npz"))),
                         ids=lambda p: os.path.basename(p)[:-4])
@pytest.mark.parametrize("periodic", [True, False], ids=["periodic", "euclid"])
def test_oracle_knn_matches_reference(path, periodic):
    z = np.load(path)
    m = meta(z)
    dnn, idx = O.knn(z["pos"], m["k"], m["box"], m["sensor_range"], periodic=periodic)
    tag = "per" if periodic else "euc"
    ok, err = allclose_rel(dnn, z[f"{tag}_dnn"], atol=1e-12)
    assert ok, err
    D = z[f"{tag}_D"] if f"{tag}_D" in z else np.sqrt(d2_rows(z["pos"], m["box"], periodic))
    exact, ties, bad = knn_mismatch(z[f"{tag}_idx"], idx, D)
    assert not bad, bad[:5]
    if m.get("lattice"):
        assert ties > 0, "lattice fixture is expected to exercise tie resolution"


def test_oracle_k_out_of_range_raises_like_reference():
    with open(os.path.join(GOLD, "errors.json")) as f:
        err = json.load(f)["k_plus_1_gt_N"]
    pos = np.random.default_rng(0).uniform(0, 10, size=(1, err["N"], 2))
    with pytest.raises(RuntimeError, match="selected index k out of range"):
        O.knn(pos, err["k"], 10.0)
    assert err["message"] == "selected index k out of range"


def test_oracle_uwd_unknown_action_raises():
    pos = np.random.default_rng(0).uniform(0, 50, size=(1, 8, 2))
    with pytest.raises(KeyError):
        O.step_uwd(pos, np.zeros((1, 8)), np.zeros((1, 8)), np.full((1, 8), 12), np.zeros((1, 8, 2)), k=4, box=50)
