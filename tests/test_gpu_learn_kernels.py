"""GPU numerics of the learner HIP kernels against plain PyTorch fp32 references of the same ops."""
import numpy as np
import pytest
import torch

from marl_range_flocking_amd.learners.core import FlatParams, GradNorm, ReplayRing, gru_cell, gru_cell_gi, gru_seq

pytestmark = pytest.mark.gpu


def test_fused_adam_matches_torch_adam(cuda):
    torch.manual_seed(0)
    shapes = {"w": (37, 53), "b": (53,)}
    fp = FlatParams(shapes, cuda, agents=5)
    ref = [torch.nn.Parameter(torch.randn(5, *s, device=cuda)) for s in shapes.values()]
    for (n, p), r in zip(fp.params.items(), ref):
        with torch.no_grad():
            p.copy_(r)
    opt = torch.optim.Adam(ref, lr=3e-3, foreach=False)
    for step in range(6):
        grads = [torch.randn_like(r) * (10.0 ** (step - 3)) for r in ref]
        for r, g in zip(ref, grads):
            r.grad = g.clone()
        opt.step()
        fp.zero_grad()
        for p, g in zip(fp.params.values(), grads):
            p.grad.copy_(g)
        fp.adam_step(3e-3)
        for p, r in zip(fp.params.values(), ref):
            torch.testing.assert_close(p.detach(), r.detach(), rtol=2e-6, atol=1e-7)


def test_fused_adam_soft_update_and_per_agent(cuda):
    shapes = {"w": (8, 4)}
    fp = FlatParams(shapes, cuda, agents=3, agent_major=True, target=True)
    with torch.no_grad():
        fp.data.uniform_(-1, 1)
        fp.target.uniform_(-1, 1)
    p0, t0 = fp.data.clone(), fp.target.clone()
    fp.grad.normal_()
    fp.adam_step(1e-3, agent=1, tau=0.01, target_mode=0)
    lo, hi = fp.agent_range(1)
    assert torch.equal(fp.data[:lo], p0[:lo]) and torch.equal(fp.data[hi:], p0[hi:])
    exp_t = t0[lo:hi] * (1 - 0.01) + fp.data[lo:hi] * 0.01
    torch.testing.assert_close(fp.target[lo:hi], exp_t, rtol=1e-6, atol=1e-7)
    assert fp.agent_steps == [0, 1, 0]
    # mode 1 self update (shared critic is its own target)
    c = fp.data.clone()
    fp.soft_update(0.001, mode=1, self_update=True)
    torch.testing.assert_close(fp.data, 0.001 * c + 0.999 * c, rtol=0, atol=0)


def test_fused_adam_vector_path_is_bitwise_the_scalar_path_at_grid_stride_sizes(cuda):
    """The float4 path (two per thread and iteration over the grid stride, csrc/flock_learn.hip adam_kernel) against
    the scalar one (unaligned views) at sizes past one and two grid strides of 2048 x 256 float4, with a tail; the
    target soft update on."""
    from marl_range_flocking_amd.learners.core import _ops

    for n in (4 * 2048 * 256 * 2 + 4 * 77 + 3, 4 * 2048 * 256 * 3 - 4 * 5 + 1):
        g0 = torch.Generator(device=cuda).manual_seed(n)
        base = [torch.rand(n + 1, device=cuda, generator=g0) for _ in range(5)]
        base[3] *= 1e-3  # v >= 0
        vec = [b[:n].clone() for b in base]      # 16-B aligned: adam_kernel<true>
        sca = [torch.empty(n + 1, device=cuda) for _ in range(5)]
        for s_, b in zip(sca, base):
            s_[1:].copy_(b[:n])
        sca = [s_[1:] for s_ in sca]            # 4-B aligned only: adam_kernel<false>
        for bufs in (vec, sca):
            step = torch.zeros(1, dtype=torch.int64, device=cuda)
            p, g, m, v, t = bufs
            for _ in range(2):
                step.add_(1)
                _ops().adam_step(p, g, m, v, step, None, t, 3e-3, 0.9, 0.999, 1e-8, 0.01, 0)
        for a, b in zip(vec, sca):
            assert torch.equal(a, b)


def test_grad_norm_and_clip_scale(cuda):
    g = torch.randn(1_000_003, device=cuda) * 0.01
    out = GradNorm(cuda)(g, 5.0)
    n = torch.linalg.vector_norm(g)
    torch.testing.assert_close(out[0], n, rtol=1e-5, atol=0)
    torch.testing.assert_close(out[1], torch.clamp(5.0 / (n + 1e-6), max=1.0), rtol=1e-5, atol=0)
    out = GradNorm(cuda)(g * 1e4, 5.0)
    torch.testing.assert_close(out[1], 5.0 / (torch.linalg.vector_norm(g * 1e4) + 1e-6), rtol=1e-5, atol=0)


@pytest.mark.parametrize("A,B,IN,H", [(1, 5, 7, 32), (6, 128, 32, 32), (3, 64, 16, 20)])
def test_gru_cell_matches_torch_grucell(A, B, IN, H, cuda):
    torch.manual_seed(A * 100 + B)
    cells = [torch.nn.GRUCell(IN, H).to(cuda) for _ in range(A)]
    x = torch.randn(A, B, IN, device=cuda, requires_grad=True)
    h = torch.randn(A, B, H, device=cuda, requires_grad=True)
    Wih = torch.stack([c.weight_ih for c in cells]).detach().requires_grad_()
    Whh = torch.stack([c.weight_hh for c in cells]).detach().requires_grad_()
    bih = torch.stack([c.bias_ih for c in cells]).detach().requires_grad_()
    bhh = torch.stack([c.bias_hh for c in cells]).detach().requires_grad_()
    out = gru_cell(x, h, Wih, Whh, bih, bhh)
    ref = torch.stack([cells[a](x[a], h[a]) for a in range(A)])
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-6)
    go = torch.randn_like(out)
    gx, gh, gw = torch.autograd.grad(out, (x, h, Wih), go)
    rx, rh = torch.autograd.grad(ref, (x, h), go, retain_graph=True)
    rw = torch.stack([torch.autograd.grad(ref, cells[a].weight_ih, go, retain_graph=True)[0] for a in range(A)])
    torch.testing.assert_close(gx, rx, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(gh, rh, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(gw, rw, rtol=1e-4, atol=1e-5)


def test_replay_ring_scatter_gather_wraps(cuda):
    ring = ReplayRing(10, {"s": (3,), "d": ()}, cuda)
    rows = [torch.arange(i * 3, i * 3 + 12, dtype=torch.float32, device=cuda).view(4, 3) for i in range(4)]
    for r in rows:
        ring.store({"s": r, "d": r[:, 0]})
    allrows = torch.cat(rows)  # 16 rows into capacity 10: positions (i mod 10), last write wins
    expect = torch.zeros(10, 3, device=cuda)
    for i in range(16):
        expect[i % 10] = allrows[i]
    assert torch.equal(ring.bufs["s"], expect)
    idx = torch.tensor([[0, 9], [3, 3]], device=cuda)
    got = ring.gather("s", idx)
    assert got.shape == (2, 2, 3) and torch.equal(got, expect[idx])
    assert torch.equal(ring.gather("d", idx), expect[idx][..., 0])
    assert len(ring) == 10 and ring.counter == 16


@pytest.mark.parametrize("cap,n,steps", [(64, 16, 7), (1000, 96, 13), (37, 5, 11)], ids=["vec", "vec-wrap", "scalar"])
def test_ring_store_fused_matches_row_copies(cap, n, steps, cuda):
    """flock_ring_store (all fields, one launch; float4 and scalar paths; bool -> 1 - x) against a python ring."""
    ring = ReplayRing(cap, {"s": (4,), "a": (2,), "r": (1,), "t": ()}, cuda)
    ref = {k: torch.zeros(cap, w, device=cuda) for k, w in (("s", 4), ("a", 2), ("r", 1), ("t", 1))}
    g = torch.Generator(device=cuda).manual_seed(0)
    pos = 0
    for _ in range(steps):
        s = torch.randn(n, 4, device=cuda, generator=g)
        a = torch.randn(n, 2, device=cuda, generator=g)
        r = torch.randn(n, 1, device=cuda, generator=g)
        d = torch.rand(n, device=cuda, generator=g) < 0.3
        ring.store({"s": s, "a": a, "r": r, "t": d}, one_minus=("t",))
        for i in range(n):
            p = (pos + i) % cap
            ref["s"][p], ref["a"][p], ref["r"][p] = s[i], a[i], r[i]
            ref["t"][p] = 1.0 - d[i].float()
        pos += n
    for k in ref:
        assert torch.equal(ring.bufs[k].reshape(cap, -1), ref[k]), k
    assert ring.counter == n * steps


@pytest.mark.parametrize("A,C,B,per_agent", [(3, 10, 32, False), (5, 10, 128, True), (2, 1, 7, True), (4, 4, 200, False),
                                             (2, 3, 16, True), (3, 5, 8, False), (512, 10, 32, False),
                                             (2, 3, 1000, True), (3, 4, 700, False)])
def test_gru_seq_matches_per_step_grucell(A, C, B, per_agent, cuda):
    """flock_gru_seq_fwd/_bwd (one launch per chunk) against the per-step loop the learners used before: gru_cell
    per step (hidden GEMM + gate kernel) with the done reset between steps, fp32 autograd, same inputs. B = 700 and
    1000: more rows than one block's LDS holds (the union batch of agent-sharded critics at 8 ranks): row chunks of
    640 in the forward launch, 256-row backward launches adding their dW / db sums in order."""
    g = torch.Generator(device=cuda).manual_seed(A * 100 + B)
    H = 32
    gi = torch.randn(A, C, B, 3 * H, device=cuda, generator=g, requires_grad=True)
    W = (0.3 * torch.randn(A, 3 * H, H, device=cuda, generator=g)).requires_grad_()
    b = (0.3 * torch.randn(A, 3 * H, device=cuda, generator=g)).requires_grad_()
    if per_agent:   # MADDPG: a done flag per agent, strided view [C, A, B]
        keep = (torch.rand(B, C, A, device=cuda, generator=g) > 0.2).permute(1, 2, 0)
    else:           # VDN: one flag per batch row, expanded over agents
        keep = (torch.rand(C, B, device=cuda, generator=g) > 0.2).unsqueeze(1).expand(C, A, B)
    hs = gru_seq(gi, W, b, keep)
    h = torch.zeros(A, B, H, device=cuda)
    ref = []
    for t in range(C):
        h = gru_cell_gi(gi[:, t], h, W, b)
        ref.append(h)
        h = torch.where(keep[t].unsqueeze(-1), h, 0.0)
    ref = torch.stack(ref, 1)
    torch.testing.assert_close(hs, ref, rtol=1e-5, atol=1e-6)
    dout = torch.randn(A, C, B, H, device=cuda, generator=g)
    d1 = torch.autograd.grad(hs, (gi, W, b), dout)
    d2 = torch.autograd.grad(ref, (gi, W, b), dout)
    for x, y, name in zip(d1, d2, ("dgi", "dW_hh", "db_hh")):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5, msg=name)
    with torch.no_grad():  # no saved gates without grad
        torch.testing.assert_close(gru_seq(gi, W, b, keep), ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("fused_bwd", [True, False], ids=["vdn_feat_bwd", "autograd_bwd"])
@pytest.mark.parametrize("A,C,B,n", [(3, 2, 5, 4), (8, 10, 32, 4), (512, 10, 32, 4), (4, 3, 70, 9)])
def test_vdn_feat_matches_torch_linear_chain(A, C, B, n, fused_bwd, cuda):
    """flock_vdn_feat_fwd (one launch: Linear(n,64)-ReLU-Linear(64,32)-ReLU-(x W_ih^T + b_ih), learners/vdn/net.py:19-33)
    against plain PyTorch fp32 nn.functional on the same per-agent weights, forward and every weight gradient, with
    the input read in place through the replay gather's permuted layout; the backward as one flock_vdn_feat_bwd
    launch or as the batched-GEMM autograd chain. Tolerance: fp32 reassociation only (rtol 1e-5 / atol 1e-5 of the
    output scale; gradients rtol 1e-4); rows = 70 and 320 cover partial 64-row blocks."""
    from marl_range_flocking_amd.learners.core import vdn_feat

    g = torch.Generator(device=cuda).manual_seed(A * 7 + B)
    r = lambda *s: (torch.rand(*s, device=cuda, generator=g) * 2 - 1)  # noqa: E731
    raw = r(B, C, A, n)                       # the replay gather's [B, C, A, n]
    x = raw.permute(2, 1, 0, 3)               # [A, C, B, n] view (unit feature stride), as VDNLearner passes it
    W = [r(A, 64, n) * 0.5, r(A, 64) * 0.5, r(A, 32, 64) * 0.2, r(A, 32) * 0.2, r(A, 96, 32) * 0.3, r(A, 96) * 0.3]
    Wf = [w.clone().requires_grad_(True) for w in W]
    Wt = [w.clone().requires_grad_(True) for w in W]
    gi = vdn_feat(x, *Wf, fused_bwd=fused_bwd)
    xr = x.reshape(A, C * B, n)
    y = torch.relu(torch.baddbmm(Wt[1].unsqueeze(1), xr, Wt[0].transpose(1, 2)))
    y = torch.relu(torch.baddbmm(Wt[3].unsqueeze(1), y, Wt[2].transpose(1, 2)))
    ref = torch.baddbmm(Wt[5].unsqueeze(1), y, Wt[4].transpose(1, 2))
    torch.testing.assert_close(gi, ref, rtol=1e-5, atol=1e-5 * float(ref.abs().max()))
    up = r(A, C * B, 96)
    (gi * up).sum().backward()
    (ref * up).sum().backward()
    for name, a_, b_ in zip(("W1", "b1", "W2", "b2", "Wi", "bi"), Wf, Wt):
        torch.testing.assert_close(a_.grad, b_.grad, rtol=1e-4, atol=1e-5 * float(b_.grad.abs().max()), msg=name)
    with torch.no_grad():  # the target network's path: gi only (no saved activations)
        torch.testing.assert_close(vdn_feat(x, *W), ref.detach(), rtol=1e-5, atol=1e-5 * float(ref.abs().max()))


@pytest.mark.parametrize("fused_bwd", [True, False], ids=["vdn_feat_bwd", "autograd_bwd"])
def test_direct_grad_views_equal_returned_grads(fused_bwd, cuda):
    """vdn_feat(grads=...) and gru_seq(gW=, gb=) write their weight gradients into given views of a flat buffer in
    the backward (VDNLearner: grads_into(direct=...), no autograd copy into the flat grad buffer): bitwise the
    gradients the same launches return to autograd, and autograd sees no gradient for those leaves."""
    from marl_range_flocking_amd.learners.core import gru_seq, vdn_feat

    A, C, B, n, H = 16, 10, 32, 4, 32
    g = torch.Generator(device=cuda).manual_seed(5)
    r = lambda *s: (torch.rand(*s, device=cuda, generator=g) * 2 - 1)  # noqa: E731
    x = r(B, C, A, n).permute(2, 1, 0, 3)
    W = [r(A, 64, n) * 0.5, r(A, 64) * 0.5, r(A, 32, 64) * 0.2, r(A, 32) * 0.2, r(A, 96, 32) * 0.3, r(A, 96) * 0.3,
         r(A, 3 * H, H) * 0.3, r(A, 3 * H) * 0.3]
    keep = torch.rand(C, A, B, device=cuda, generator=g) > 0.1
    up = r(A, C, B, H)

    def run(direct):
        P = [w.clone().requires_grad_(True) for w in W]
        flat = torch.full((sum(w.numel() for w in W),), float("nan"), device=cuda)
        views, off = [], 0
        for w in W:
            views.append(flat[off:off + w.numel()].view(w.shape))
            off += w.numel()
        gi = vdn_feat(x, *P[:6], fused_bwd=fused_bwd, grads=views[:6] if direct else None).view(A, C, B, 3 * H)
        hs = gru_seq(gi, P[6], P[7], keep, gW=views[6] if direct else None, gb=views[7] if direct else None)
        grads = torch.autograd.grad((hs * up).sum(), P, allow_unused=True)
        if direct:
            assert all(gr is None for gr in grads)
            return views
        return grads

    for name, a_, b_ in zip(("W1", "b1", "W2", "b2", "Wi", "bi", "W_hh", "b_hh"), run(True), run(False)):
        assert torch.equal(a_, b_), name


@pytest.mark.parametrize("A,C,B,NA", [(3, 10, 32, 10), (512, 10, 32, 10), (4, 3, 8, 2), (2, 5, 32, 16)])
def test_gru_seq_q_matches_gru_seq_and_linear(A, C, B, NA, cuda):
    """flock_gru_seq_q_fwd / _bwd (recurrence + VDN's q head Linear(32, NA) in one launch each way) against gru_seq
    followed by the batched torch Linear of the same weights: q, and the gradients of gi, W_hh, b_hh, W_q, b_q.
    Tolerance: fp32 reassociation of the q dot products / weight-gradient sums (rtol 1e-5 forward, 1e-4 grads)."""
    from marl_range_flocking_amd.learners.core import gru_seq, gru_seq_q

    g = torch.Generator(device=cuda).manual_seed(A + NA)
    H = 32
    r = lambda *s: torch.randn(*s, device=cuda, generator=g)  # noqa: E731
    W = [r(A, C, B, 3 * H), 0.3 * r(A, 3 * H, H), 0.3 * r(A, 3 * H), 0.3 * r(A, NA, H), 0.3 * r(A, NA)]
    keep = torch.rand(C, A, B, device=cuda, generator=g) > 0.15
    P1 = [w.clone().requires_grad_(True) for w in W]
    P2 = [w.clone().requires_grad_(True) for w in W]
    q1 = gru_seq_q(P1[0], P1[1], P1[2], P1[3], P1[4], keep)
    hs = gru_seq(P2[0], P2[1], P2[2], keep)
    q2 = torch.baddbmm(P2[4].unsqueeze(1), hs.reshape(A, C * B, H), P2[3].transpose(1, 2)).view(A, C, B, NA)
    torch.testing.assert_close(q1, q2, rtol=1e-5, atol=1e-5)
    up = r(A, C, B, NA)
    d1 = torch.autograd.grad((q1 * up).sum(), P1)
    d2 = torch.autograd.grad((q2 * up).sum(), P2)
    for name, a_, b_ in zip(("gi", "W_hh", "b_hh", "W_q", "b_q"), d1, d2):
        torch.testing.assert_close(a_, b_, rtol=1e-4, atol=1e-5 * float(b_.abs().max()), msg=name)
    with torch.no_grad():  # the target network's call (no saved states)
        torch.testing.assert_close(gru_seq_q(*W, keep), q2.detach(), rtol=1e-5, atol=1e-5)


def test_vdn_forward_seq_large_batch_falls_back(cuda):
    """forward_seq at a batch the fused q-head backward's LDS cannot hold (B = 256, NA = 10) takes gru_seq + the
    batched q GEMMs instead of failing; same q as the fused path at a small batch slice (tolerance: fp32
    reassociation of the q head)."""
    from marl_range_flocking_amd.learners.vdn import BatchedQNet

    g = torch.Generator(device=cuda).manual_seed(3)
    net = BatchedQNet(4, 4, 10, device=cuda, generator=g)
    x = torch.rand(4, 10, 256, 4, device=cuda, generator=g)
    keep = torch.rand(10, 256, device=cuda, generator=g) > 0.1
    P = net.P.new_leaves()
    q, names = net.forward_seq(x, keep, P, direct_grads=True)
    assert names == net.DIRECT[:8]  # fused feature chain, unfused q head
    q_small = net.forward_seq(x[:, :, :32].contiguous(), keep[:, :32], P)
    torch.testing.assert_close(q[:, :, :32], q_small, rtol=1e-5, atol=1e-5)
