"""Compact encoding for the production-shape learner fixtures (test infrastructure only; nothing here ships).

At the reference's default layer sizes (400/300) a full dump of every initial / final parameter and every consumed
gradient would be tens of MB per learner. The ``*_prod.npz`` fixtures therefore keep:
  * the initial parameters as a recipe, not data: every parameter of every network is overwritten, before the
    reference's update runs, with ``init_value(tag, name, shape)`` (a seeded numpy draw), and the test rebuilds the same
    values from the (tag, name, shape) list stored in the fixture's metadata;
  * the final parameters at up to ``S`` seeded sample positions per tensor (``sample_index``), every position of the
    small tensors;
  * instead of the gradients, one bit per sampled position saying whether every gradient the optimizer consumed there
    was well-conditioned (``|g| > 1e-6`` or exactly 0, the SURVEY.md §8(c) rule for comparing post-Adam parameters).
The generators (``gen_golden_learn_*.py --prod``) and the GPU tests share these functions, so both sides see the same
numbers.
"""
import zlib

import numpy as np

S = 512  # sampled positions per large tensor


def _rng(*key):
    return np.random.default_rng([zlib.crc32("/".join(map(str, key)).encode()), 7])


def init_value(tag, name, shape, seed=0):
    """Deterministic f32 initial value of parameter ``name`` of network ``tag`` (nn.Linear-like U(+-1/sqrt(fan_in));
    LayerNorm weights 1 + U(+-0.1), LayerNorm biases U(+-0.1)). Target networks ("target" in tag) are the online
    network's value plus 0.01 * N(0, 1), so target and online networks differ as they do during training."""
    shape = tuple(int(s) for s in shape)
    base = tag.replace("target_", "")
    r = _rng(seed, base, name)
    if (name.startswith("bn") or ".ln" in name or name.startswith("ln")) and name.endswith("weight"):
        v = (1.0 + r.uniform(-0.1, 0.1, shape)).astype(np.float32)
    elif name.startswith("bn") or name.startswith("ln"):
        v = r.uniform(-0.1, 0.1, shape).astype(np.float32)
    else:
        fan = shape[-1] if len(shape) > 1 else max(shape[0], 1)
        b = 1.0 / np.sqrt(fan)
        v = r.uniform(-b, b, shape).astype(np.float32)
    if tag.startswith("target"):
        v = (v + (0.01 * _rng(seed, tag, name, "perturb").standard_normal(shape)).astype(np.float32)).astype(
            np.float32)
    return v


def rebuild(specs, seed=0):
    """specs: [[tag, name, shape], ...] (fixture metadata) -> {tag: {name: ndarray}} in spec order."""
    out = {}
    for tag, name, shape in specs:
        out.setdefault(tag, {})[name] = init_value(tag, name, shape, seed)
    return out


def sample_index(tag, name, size, s=S):
    """Sorted flat positions compared for tensor ``name`` of network ``tag`` (all of them when size <= s)."""
    if size <= s:
        return np.arange(size)
    return np.sort(_rng("sample", tag, name).choice(size, s, replace=False))


def well_conditioned(grads, shape):
    """Positions where every consumed gradient is |g| > 1e-6 or exactly 0 (no gradients: all positions)."""
    m = np.ones(shape, bool)
    for g in grads:
        g = np.asarray(g)
        m &= (np.abs(g) > 1e-6) | (g == 0)
    return m


def encode(tag, params, grads_by_name=None, s=S):
    """{name: final value} (+ {name: [consumed grads]}) -> fixture entries of network ``tag`` (``s`` samples per
    tensor, recorded in the fixture's meta as "samples")."""
    out = {}
    for name, v in params.items():
        v = np.asarray(v, np.float32)
        idx = sample_index(tag, name, v.size, s)
        out[f"final/{tag}/{name}"] = v.reshape(-1)[idx]
        if grads_by_name is not None:
            m = well_conditioned(grads_by_name.get(name, []), v.shape).reshape(-1)[idx]
            out[f"mask/{tag}/{name}"] = np.packbits(m)
    return out


def decode_mask(z, tag, name, n):
    key = f"mask/{tag}/{name}"
    if key not in z.files:
        return None
    return np.unpackbits(z[key])[:n].astype(bool)


def check(z, tag, name, got, lr, n_steps, rtol=1e-4, atol=1e-6, s=S):
    """Compare a final tensor ``got`` with the fixture's samples: well-conditioned positions within rtol / atol,
    the others within the Adam step bound 2 * lr per step (lr * g / (|g| + eps) is sign-unstable for tiny g);
    networks without a mask (never updated by an optimizer) bitwise."""
    got = np.asarray(got, np.float32).reshape(-1)
    idx = sample_index(tag, name, got.size, s)
    want = z[f"final/{tag}/{name}"]
    g = got[idx]
    mask = decode_mask(z, tag, name, idx.size)
    if mask is None:
        np.testing.assert_array_equal(g, want, err_msg=f"{tag} {name}")
        return
    g64, w64 = g.astype(np.float64), want.astype(np.float64)
    err = np.abs(g64 - w64)
    bad = mask & (err > atol + rtol * np.abs(w64))
    assert not bad.any(), f"{tag} {name}: {bad.sum()} / {mask.sum()} off, max err {err[mask].max()}"
    loose = ~mask & (err > 2.0 * lr * max(1, n_steps) + atol)
    assert not loose.any(), f"{tag} {name}: ill-conditioned elements beyond the Adam step bound: {err[~mask].max()}"
