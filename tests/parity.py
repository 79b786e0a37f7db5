"""Parity helpers shared by the oracle-vs-reference and GPU-vs-oracle tests.

Tolerance rules (north_star): neighbour indices bit-exact, except that two index lists may differ by
swapping neighbours whose distances are tied within a few ulp (the reference's torch.topk tie order is
implementation-defined); float32 state within rtol 1e-5.
"""
import json

import numpy as np

RTOL = 1e-5  # north_star: "within 1e-5 rtol on float32 positions/velocities"
TIE_ULP = 4  # near-tie window for index permutations


def meta(z):
    return json.loads(str(z["meta"]))


def d2_rows(pos, box, periodic):
    """[E,N,N] squared distances with the reference op order (gym_flock_v2.py:137-144), float32."""
    p = np.asarray(pos, np.float32)
    dx = (p[:, :, None, 0] - p[:, None, :, 0]).astype(np.float32)
    dy = (p[:, :, None, 1] - p[:, None, :, 1]).astype(np.float32)
    if periodic:
        half = np.float32(box) * np.float32(0.5)
        dx, dy = np.abs(dx), np.abs(dy)
        dx = np.where(dx > half, np.float32(box) - dx, dx).astype(np.float32)
        dy = np.where(dy > half, np.float32(box) - dy, dy).astype(np.float32)
    return (dx * dx).astype(np.float32) + (dy * dy).astype(np.float32)


def knn_positions(pos, m):
    """The positions the kNN ranks: pos / max |p| per env under normalize_distance (gym_flock_uw.py:127-133)."""
    p = np.asarray(pos, np.float32)
    if not m.get("normalize_distance", False):
        return p
    mag = np.sqrt((p[..., 0] * p[..., 0]).astype(np.float32) + (p[..., 1] * p[..., 1]).astype(np.float32))
    return (p / mag.max(-1)[:, None, None]).astype(np.float32)


def knn_mismatch(ref_idx, our_idx, D, tie_ulp=TIE_ULP):
    """Compare two [E,N,k] index arrays given distances D [E,N,N] (any monotone distance works).

    Returns (n_exact_rows, n_tie_rows, bad_rows) where bad_rows lists (e, i) whose lists differ by more than a
    permutation of near-tied neighbours.
    """
    ref_idx = np.asarray(ref_idx)
    our_idx = np.asarray(our_idx)
    exact = (ref_idx == our_idx).all(-1)
    bad = []
    ties = 0
    for e, i in zip(*np.nonzero(~exact)):
        dr = D[e, i, ref_idx[e, i]].astype(np.float64)
        do = D[e, i, our_idx[e, i]].astype(np.float64)
        tol = tie_ulp * np.spacing(np.maximum(np.abs(dr), np.abs(do)).astype(np.float32)).astype(np.float64)
        if np.all(np.abs(dr - do) <= tol):
            ties += 1
        else:
            bad.append((int(e), int(i)))
    return int(exact.sum()), ties, bad


def allclose_rel(a, b, rtol=RTOL, atol=0.0):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    both_nan = np.isnan(a) & np.isnan(b)
    ok = np.isclose(a, b, rtol=rtol, atol=atol) | both_nan
    return bool(ok.all()), (np.nanmax(np.abs(a - b) / np.maximum(np.abs(b), 1e-30)) if a.size else 0.0)


def _knn_exact(pos, k, box, sr, periodic, clamp, gdnn, gidx, normalize=False):
    """GPU kNN (distances and indices) bitwise equal to the C oracle's exact (d2, j) order on the same positions."""
    from oracle import oracle as O

    dnn, idx = O.knn(pos, k, box, sr, periodic=periodic, clamp=clamp, normalize=normalize)
    np.testing.assert_array_equal(gidx, idx)
    np.testing.assert_array_equal(gdnn, dnn)
