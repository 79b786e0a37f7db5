"""Learner updates at the BASELINE configs' own shapes, against independent plain-PyTorch fp32 restatements of the
reference loops (tests/reference_torch.py, autograd gradients):

  config 4  VDN train() with 512 agents (learners/vdn/train_flock.py:16-43; B 32, chunk 10)
  config 5  RNN-MADDPG train() with 1024 agents at hidden 400/300 (learners/maddpg_official_rnn/MADDPG.py:78-150;
            B 128, chunk 10): 0.9 G critic parameters

These shapes are too large for a reference fixture (the reference's per-agent Python loops would take hours on the
container's CPU); the production-shape fixtures at 64 / 16 agents (test_gpu_learners.py::*_prod) pin the same code
paths against the reference itself. Tolerances: losses rtol 1e-4; gradients rtol 1e-3 with atol
1e-4 x the tensor's largest |g| (two summation orders over up to 2448-wide dot products); post-Adam parameters
rtol 1e-4 where every |g| > 1e-6, the Adam step bound elsewhere; frozen actors and target soft updates bitwise.

At config 5 the critic's fce gradient sums B x C = 1280 products of O(10) inputs with heavy cancellation, so a
fixed rtol is the wrong yardstick there: the restatement also runs in float64 and the build's gradients must be as
close to it as the plain fp32 restatement's are (max and L2 error each within 4x the fp32 restatement's, per
tensor); post-Adam parameters are then compared where |g| exceeds both 1e-6 and 4x the largest fp32 gradient error
(no Adam sign flips possible there).
"""
import numpy as np
import pytest
import torch

import reference_torch as R

pytestmark = pytest.mark.gpu


def _adam_reference(params, grads, lr, clip=None):
    """torch.optim.Adam (single-tensor path, the reference's optimizer) on copies of params, after an optional
    clip_grad_norm_(clip)."""
    ps = [torch.nn.Parameter(p.detach().clone()) for p in params]
    for p, g in zip(ps, grads):
        p.grad = g.detach().clone()
    if clip is not None:
        torch.nn.utils.clip_grad_norm_(ps, clip, norm_type=2)
    opt = torch.optim.Adam(ps, lr=lr, foreach=False)
    opt.step()
    return [p.detach() for p in ps]


def _post_adam_close(got, want, g, lr, what, thresh=1e-6, g_err=0.0):
    """Adam's first step is lr * g / (|g| + eps): where |g| > thresh, the parameters agree within rtol 1e-4 plus
    what a gradient error g_err can move that ratio (eps * g_err / g^2, times lr); elsewhere within the step bound."""
    well = g.abs() > thresh
    err = (got - want).abs()
    tol = 1e-6 + 1e-4 * want.abs() + lr * 2e-8 * g_err / g.double().square().clamp_min(1e-300)
    bad = well & (err > tol)
    assert not bad.any(), f"{what}: {int(bad.sum())} of {int(well.sum())} off, max {float(err[well].max())}"
    assert float(err.max()) <= 2 * lr + 1e-6, f"{what}: beyond the Adam step bound"


def _grad_close(got, want, what):
    scale = float(want.abs().max())
    torch.testing.assert_close(got, want, rtol=1e-3, atol=1e-4 * max(scale, 1e-30), msg=lambda m: f"{what}: {m}")


def test_vdn_train_config4_shape(cuda):
    """VDN, 512 agents (BASELINE config 4's swarm), one update iteration through the HIP-graph path."""
    from marl_range_flocking_amd.learners.vdn import VDNLearner

    A, K, NA, B, C, T, lr, gamma = 512, 4, 4, 32, 10, 60, 1e-3, 0.99
    g = torch.Generator(device=cuda).manual_seed(4)
    s_all = torch.rand(T, A, K, device=cuda, generator=g) * 7
    s2_all = torch.rand(T, A, K, device=cuda, generator=g) * 7
    a_all = torch.randint(0, NA, (T, A), device=cuda, generator=g)
    r_all = torch.where(torch.rand(T, A, device=cuda, generator=g) < 0.05, -8.9, 0.1)
    d_all = (torch.rand(T, device=cuda, generator=g) < 0.15).float()
    L = VDNLearner(A, K, NA, lr=lr, gamma=gamma, batch_size=B, chunk_size=C, update_iter=1, grad_clip_norm=5.0,
                   buffer_limit=64, device=cuda, use_graph=True)
    with torch.no_grad():  # a target network that differs from q
        L.q.P.target.add_(0.01 * torch.randn(L.q.P.target.shape, device=cuda, generator=g))
    L.put(s_all, a_all, r_all, s2_all, d_all)
    P0 = {n: L.q.P.view(L.q.P.data, n).detach().clone().requires_grad_(True) for n in L.q.P.shapes}
    T0 = {n: L.q.P.view(L.q.P.target, n).detach().clone() for n in L.q.P.shapes}
    starts = torch.randint(0, T - C, (B,), device=cuda, generator=g)
    L.train(starts=starts[None])
    torch.cuda.synchronize()

    idx = starts[:, None] + torch.arange(C, device=cuda)[None]
    loss = R.vdn_loss(P0, T0, s_all[idx], a_all[idx].float(), r_all[idx], s2_all[idx], d_all[idx][..., None], gamma)
    grads = torch.autograd.grad(loss, list(P0.values()))
    np.testing.assert_allclose(L.loss.item(), loss.item(), rtol=1e-4)
    norm = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(x) for x in grads]))
    np.testing.assert_allclose(L.norm.out[0].item(), norm.item(), rtol=1e-4)
    for n, gr in zip(P0, grads):
        _grad_close(L.q.P.view(L.q.P.grad, n), gr, f"grad {n}")
    new = _adam_reference(list(P0.values()), grads, lr, clip=5.0)
    for n, want, gr in zip(P0, new, grads):
        _post_adam_close(L.q.P.view(L.q.P.data, n), want, gr, lr, n)


def test_maddpg_rnn_train_config5_shape(cuda):
    """RNN-MADDPG with 1024 agents at hidden 400/300 (BASELINE config 5's learner): one train() through the
    HIP-graph path against the reference loop restated in plain PyTorch."""
    from marl_range_flocking_amd.learners.maddpg import CRITIC_JOINED, MADDPGLearner

    N, K, B, C, T, lr, gamma, tau = 1024, 4, 128, 10, 150, 3e-3, 0.99, 0.001
    L = MADDPGLearner(N, K, recurrent=True, hidden1=400, hidden2=300, batch_size=B, chunk_size=C,
                      buffer_capacity=160, min_size_buffer=B, device=cuda, use_graph=True, seed=3)
    g = torch.Generator(device=cuda).manual_seed(5)
    with torch.no_grad():  # targets that differ from the online networks
        for fp in (L.actors, L.critics):
            fp.target.add_(0.01 * torch.randn(fp.target.shape, device=cuda, generator=g))
    obs = torch.rand(T + 1, N, K, device=cuda, generator=g) * 14
    act = torch.rand(T, N, 2, device=cuda, generator=g) * 2.5 - 1
    rew = torch.where(torch.rand(T, N, device=cuda, generator=g) < 0.05, -5.0, 0.01)
    done = (torch.rand(T, N, device=cuda, generator=g) < 0.02).float()
    L.add_record(obs[:-1], obs[1:], act, obs[:-1], obs[1:], rew, done)  # one record per row of the leading dim

    def snap(fp, buf, joined):
        d = {n: fp.view(buf, n).detach().clone() for n in fp.shapes}
        if joined:
            for ref, parts in CRITIC_JOINED.items():
                d[ref] = torch.cat([d.pop(p) for p in parts], -1)
        return d

    Pc = snap(L.critics, L.critics.data, True)
    Ptc = snap(L.critics, L.critics.target, True)
    Pa, Pta = snap(L.actors, L.actors.data, False), snap(L.actors, L.actors.target, False)
    starts = torch.randperm(T - C, device=cuda, generator=g)[:B]
    assert L.train(starts=starts) is not None
    torch.cuda.synchronize()
    got = snap(L.critics, L.critics.data, True)
    got_grad = snap(L.critics, L.critics.grad, True)
    got_target = snap(L.critics, L.critics.target, True)

    idx = starts[:, None] + torch.arange(C, device=cuda)[None]                       # [B, C]
    names = list(Pc)

    def restated(dtype):
        cast = lambda d: {n: v.to(dtype) for n, v in d.items()}  # noqa: E731
        P = {n: v.requires_grad_(True) for n, v in cast(Pc).items()}
        o, a = obs.to(dtype), act.to(dtype)
        total, closs, aloss = R.maddpg_rnn_loss(
            P, cast(Ptc), cast(Pa), cast(Pta), o[:-1][idx], o[1:][idx], o[:-1][idx].permute(2, 0, 1, 3),
            o[1:][idx].permute(2, 0, 1, 3), a[idx].permute(2, 0, 1, 3), rew.to(dtype)[idx][..., None],
            done.to(dtype)[idx][..., None], gamma)
        gr = torch.autograd.grad(total, [P[n] for n in names])
        return [closs.mean().item(), aloss.mean().item()], dict(zip(names, gr))

    losses64, g64 = restated(torch.float64)
    np.testing.assert_allclose(L.losses.cpu().numpy(), losses64, rtol=1e-4)
    losses32, g32 = restated(torch.float32)
    grads = {}
    for n in names:
        e32 = (g32.pop(n).double() - g64[n])
        e_build = got_grad[n].double() - g64[n]
        tiny = 1e-12 * float(g64[n].abs().max())
        assert float(e_build.abs().max()) <= 4 * float(e32.abs().max()) + tiny, f"critic grad {n}: max error"
        assert float(e_build.norm()) <= 4 * float(e32.norm()) + tiny, f"critic grad {n}: L2 error"
        grads[n] = (g64[n], 4 * float(e32.abs().max()))
    new = dict(zip(names, _adam_reference([Pc[n].double() for n in names], [grads[n][0] for n in names], lr)))
    for n in names:
        gref, err = grads[n]
        _post_adam_close(got[n].double(), new[n], gref, lr, f"critic {n}", thresh=max(1e-6, err), g_err=err)
        # update_target_networks (net.py:74-78) from the learner's own post-Adam parameters: same op order
        assert torch.equal(got_target[n], Ptc[n] * (1.0 - tau) + got[n] * tau), f"target critic {n}"
    for n in L.actors.shapes:  # the actors get no gradient (Q6): frozen, their targets soft-updated
        assert torch.equal(L.actors.view(L.actors.data, n), Pa[n]), f"actor {n}"
        assert torch.equal(L.actors.view(L.actors.target, n), Pta[n] * (1.0 - tau) + Pa[n] * tau), f"target actor {n}"
