"""CPU tests of learner helpers that need no GPU (learners/core.py)."""
import torch

from marl_range_flocking_amd.learners.core import linear_t


def test_linear_t_is_differentiable_without_gradient_views():
    """linear_t on trainable parameters under autograd and with no gW / gb views (the public path): the functional
    GEMM forms, so the backward reaches W, b and x; under no_grad the out= forms give the same values."""
    g = torch.Generator().manual_seed(0)
    x = torch.rand(5, 3, generator=g, requires_grad=True)
    W = torch.rand(2, 4, 3, generator=g, requires_grad=True)
    b = torch.rand(2, 4, generator=g, requires_grad=True)
    y = linear_t(x, W, b)
    ref = torch.einsum("aoi,ri->aor", W, x) + b[..., None]
    torch.testing.assert_close(y, ref)
    (y * torch.arange(y.numel()).reshape(y.shape)).sum().backward()
    xr, Wr, br = (t.detach().clone().requires_grad_() for t in (x, W, b))
    (torch.einsum("aoi,ri->aor", Wr, xr) + br[..., None]).mul(torch.arange(y.numel()).reshape(y.shape)).sum().backward()
    for got, want in ((x.grad, xr.grad), (W.grad, Wr.grad), (b.grad, br.grad)):
        torch.testing.assert_close(got, want)
    with torch.no_grad():
        torch.testing.assert_close(linear_t(x, W, b), ref)
        torch.testing.assert_close(linear_t(x, W), ref - b[..., None])


def test_replay_ring_pending_copy_is_copied_back_on_first_access():
    """ReplayRing.set_pending_copy (a loop's ring copies, SharedCriticBench.run_steps): the copy's rows replace the
    ring's at the next access of bufs, once; later writes to the copy are not seen."""
    from marl_range_flocking_amd.learners.core import ReplayRing

    ring = ReplayRing(6, {"state": (4,), "reward": ()}, "cpu")
    src = {"state": torch.arange(24, dtype=torch.float32).reshape(6, 4), "reward": torch.full((6,), 2.0)}
    ring.set_pending_copy(src)
    assert ring._pending is not None
    b = ring.bufs
    assert ring._pending is None
    assert torch.equal(b["state"], src["state"]) and torch.equal(b["reward"], src["reward"])
    src["reward"].fill_(7.0)  # the copy is a buffer of its own: the ring does not alias it
    assert torch.equal(ring.bufs["reward"], torch.full((6,), 2.0))
    try:
        ring.set_pending_copy({"state": src["state"]})
    except AssertionError:
        pass
    else:
        raise AssertionError("a pending copy must name every field")
