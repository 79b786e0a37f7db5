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
