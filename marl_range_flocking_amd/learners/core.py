"""Batched-over-agents learner building blocks on MI355X.

* ``FlatParams``: every parameter of every agent copy of one network lives in ONE flat f32 buffer (with flat grad,
  Adam moment and optional target buffers), exposed as per-layer stacked leaf tensors [A, out, in] that alias it.
  One ``flock_adam_step`` launch then updates all agents (the reference steps one torch.optim.Adam per agent).
* ``blinear`` / ``blayer_norm``: per-agent Linear / LayerNorm over a leading agent axis; the GEMMs are batched
  rocBLAS/hipBLASLt GEMMs (torch.bmm / baddbmm), f32 in and out (gfx950 has no xf32/TF32 path to fall into).
* ``gru_cell``: nn.GRUCell with the gate GEMMs batched and the elementwise part in flock_gru_fwd/bwd.
* ``ReplayRing``: device-resident ring of named row tensors with HIP row scatter (insert) / gather (sample).
"""
import math
from collections import OrderedDict

import warnings

import torch

# agent-major stacked views are strided; their grads alias the same strides on purpose
warnings.filterwarnings("ignore", message="grad and param do not obey the gradient layout contract")


def _ops():
    """torch.ops.flock (csrc/flock_torch*.cpp): every learner kernel below launches through these custom ops."""
    from .. import torch_ops

    return torch_ops.load()


def _require_cuda(t):
    if t.device.type != "cuda":
        raise RuntimeError("learner kernels run on a HIP device only (no CPU fallback)")


class FlatParams:
    """Stacked parameters of ``agents`` copies of one network, aliasing ONE flat f32 buffer.

    shapes: name -> per-agent shape. Each name is exposed as a leaf Parameter [agents, *shape] whose grad aliases the
    flat grad buffer. Layouts: layer-major (default; every stacked tensor contiguous — batched training of all
    agents) or agent-major (each agent's parameters contiguous — per-agent Adam steps, as the shared-critic learner
    updates one actor per learn() call; per-agent leaf views come from agent_params(i)).
    """

    def __init__(self, shapes, device, agents=1, agent_major=False, target=False, adam=True, agent_pad=1):
        self.shapes = OrderedDict((k, tuple(v)) for k, v in shapes.items())
        self.device = torch.device(device)
        self.agents = int(agents)
        self.agent_major = agent_major
        # agent_pad: each agent's block rounded up to a multiple of agent_pad floats (zero padding, never a
        # parameter), so every agent's slice starts equally aligned (the fused kernels use 16-B vector loads)
        raw = sum(math.prod(s) for s in self.shapes.values())
        self.per_agent = -(-raw // agent_pad) * agent_pad
        n = self.per_agent * self.agents
        self.numel = n
        z = lambda: torch.zeros(n, dtype=torch.float32, device=self.device)  # noqa: E731
        self.data, self.grad = z(), z()
        self.exp_avg = z() if adam else None
        self.exp_avg_sq = z() if adam else None
        self.target = z() if target else None
        self.step_count = 0
        self.agent_steps = [0] * self.agents
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=self.device)  # for graph-captured steps
        self.offsets = OrderedDict()
        off = 0
        for name, shp in self.shapes.items():
            m = math.prod(shp)
            self.offsets[name] = (off, m)
            off += m
        self.params = OrderedDict()
        for name in self.shapes:
            p = torch.nn.Parameter(self.view(self.data, name))
            p.grad = self.view(self.grad, name)
            self.params[name] = p
        self._agent_params = {}
        self.writers = []  # OverlappedTrain updates that write this buffer on a stream of their own

    def sync_writers(self):
        """The current stream waits for every pending overlapped update of these parameters (OverlappedTrain): called
        by the host-side readers and writers (export / load / hard_update_target, the learners' acting and
        state-dict methods), so mixing train_overlapped() with them never races."""
        for w in self.writers:
            w.sync()

    def view(self, buf, name, agent=None):
        """Stacked [agents, *shape] view of ``buf`` (data / grad / target / moments) for ``name``."""
        off, m = self.offsets[name]
        shp = self.shapes[name]
        if self.agent_major:
            v = buf.view(self.agents, self.per_agent)[:, off:off + m].view(self.agents, *shp)
        else:
            v = buf[self.agents * off:self.agents * (off + m)].view(self.agents, *shp)
        return v if agent is None else v[agent:agent + 1]

    def __getitem__(self, name):
        return self.params[name]

    def new_leaves(self, squeeze=False):
        """A fresh set of leaf Parameters aliasing the same data/grad storage. Graph-captured updates use their own
        set, so an autograd graph a caller keeps alive on ``params`` (e.g. a grad-enabled forward outside the
        learner) never shares AccumulateGrad nodes with the captured backward (that combination crashed HIP graph
        capture on ROCm 7.2). squeeze (single network): leaves without the agent axis, so no select/unsqueeze
        (and no zero-fill + copy in their backward) enters the graph."""
        d = OrderedDict()
        for name in self.shapes:
            v = self.view(self.data, name)
            g = self.view(self.grad, name)
            if squeeze:
                assert self.agents == 1
                v, g = v[0], g[0]
            p = torch.nn.Parameter(v)
            p.grad = g
            d[name] = p
        return d

    def grads_into(self, loss, leaves, direct=()):
        """Gradients of ``loss`` w.r.t. ``leaves`` written straight into the flat grad buffer with one multi-tensor
        copy (instead of zero-fill + one AccumulateGrad add per parameter). ``direct``: names whose gradient the
        backward itself writes into the grad view (linear_t with grad views): neither copied nor zeroed."""
        names = list(leaves)
        grads = torch.autograd.grad(loss, [leaves[n] for n in names], allow_unused=True)
        dst, src = [], []
        for n, g in zip(names, grads):
            view = leaves[n].grad
            if n in direct:
                assert g is None, f"{n}: written by its backward, yet autograd produced a gradient too"
                continue
            if g is None:
                view.zero_()
            else:
                dst.append(view)
                src.append(g)
        if dst:
            torch._foreach_copy_(dst, src)

    def target_view(self, name, agent=None):
        return self.view(self.target, name, agent)

    def agent_params(self, i):
        """Leaf Parameters [1, *shape] of agent i (agent-major layout), grads aliasing the flat grad buffer."""
        assert self.agent_major
        if i not in self._agent_params:
            d = OrderedDict()
            for name in self.shapes:
                p = torch.nn.Parameter(self.view(self.data, name, i))
                p.grad = self.view(self.grad, name, i)
                d[name] = p
            self._agent_params[i] = d
        return self._agent_params[i]

    def agent_range(self, i):
        assert self.agent_major
        return i * self.per_agent, (i + 1) * self.per_agent

    def parameters(self):
        return list(self.params.values())

    def zero_grad(self, agent=None):
        if agent is None:
            self.grad.zero_()
        else:
            a, b = self.agent_range(agent)
            self.grad[a:b].zero_()

    def adam_step(self, lr, betas=(0.9, 0.999), eps=1e-8, grad_scale=None, tau=None, target_mode=0, agent=None):
        """torch.optim.Adam.step() for every agent in one launch (or agent i's slice, agent-major), optionally
        fused with the target soft update."""
        _require_cuda(self.data)
        if agent is None:
            self.step_count += 1
            lo, hi, step = 0, self.numel, self.step_count
        else:
            self.agent_steps[agent] += 1
            (lo, hi), step = self.agent_range(agent), self.agent_steps[agent]
        sl = lambda t: None if t is None else t[lo:hi]  # noqa: E731
        st = self.__dict__.get("_host_step")
        if st is None:
            st = self._host_step = torch.zeros(1, dtype=torch.int64, device=self.device)
        st.fill_(step)
        _ops().adam_step(sl(self.data), sl(self.grad), sl(self.exp_avg), sl(self.exp_avg_sq), st, grad_scale,
                         sl(self.target) if tau is not None else None, float(lr), float(betas[0]), float(betas[1]),
                         float(eps), float(tau or 0.0), int(target_mode))

    def adam_step_dev(self, lr, betas=(0.9, 0.999), eps=1e-8, grad_scale=None, tau=None, target_mode=0):
        """Adam step with the step count kept on the device (step_dev += 1 then the update): HIP-graph capturable."""
        self.step_dev.add_(1)
        _ops().adam_step(self.data, self.grad, self.exp_avg, self.exp_avg_sq, self.step_dev, grad_scale,
                         self.target if tau is not None else None, float(lr), float(betas[0]), float(betas[1]),
                         float(eps), float(tau or 0.0), int(target_mode))

    def state_tensors(self):
        return [t for t in (self.data, self.exp_avg, self.exp_avg_sq, self.target, self.step_dev) if t is not None]

    def soft_update(self, tau, mode=0, agent=None, self_update=False):
        """target <- mode 0: t*(1-tau)+p*tau, mode 1: tau*p+(1-tau)*t. self_update: params <- soft(params, params)
        (the shared critic is its own target, agent_simple_shared_critic.py:63,76,172-178)."""
        lo, hi = (0, self.numel) if agent is None else self.agent_range(agent)
        dst = self.data if self_update else self.target
        _ops().soft_update(dst[lo:hi], self.data[lo:hi], float(tau), int(mode))

    def hard_update_target(self):
        self.sync_writers()
        self.target.copy_(self.data)

    def load(self, name, value, agent=None, target=False):
        """Copy a per-agent (agent=i) or stacked value into params (or the target copy)."""
        self.sync_writers()
        dst = self.view(self.target if target else self.data, name)
        v = torch.as_tensor(value, dtype=torch.float32).to(self.device)
        with torch.no_grad():
            if agent is None:
                dst.copy_(v.reshape(dst.shape))
            else:
                dst[agent].copy_(v.reshape(dst[agent].shape))

    def export(self, name, agent=None, target=False):
        self.sync_writers()
        v = self.view(self.target if target else self.data, name)
        return v.detach().clone() if agent is None else v[agent].detach().clone()


class GradNorm:
    """clip_grad_norm_ without a host sync: out[0] = ||g||, out[1] = clip coefficient (feed to adam_step)."""

    def __init__(self, device, max_parts=2048):
        self.partial = torch.zeros(max_parts, dtype=torch.float64, device=device)
        self.out = torch.zeros(2, dtype=torch.float32, device=device)
        self.max_parts = max_parts

    def __call__(self, grad, max_norm):
        _ops().grad_norm(grad, self.partial, self.out, float(max_norm))
        return self.out


def blinear(x, W, b=None):
    """Per-agent Linear: x [A,B,in] (or [B,in] shared by all agents), W [A,out,in], b [A,out] -> [A,B,out].
    A single network (W [out,in]) is a plain F.linear on 2-D activations; A == 1 stacked also goes through F.linear
    (one GEMM with the bias epilogue) instead of a batched GEMM."""
    if W.dim() == 2:
        return torch.nn.functional.linear(x, W, b)
    if W.shape[0] == 1:
        x2 = x if x.dim() == 2 else x[0]
        return torch.nn.functional.linear(x2, W[0], None if b is None else b[0]).unsqueeze(0)
    if x.dim() == 2:
        return shared_linear(x, W, b)
    Wt = W.transpose(1, 2)
    if b is None:
        return torch.bmm(x, Wt)
    return torch.baddbmm(b.unsqueeze(1), x, Wt)


def shared_linear(x, W, b=None):
    """Every agent's Linear applied to ONE input shared by all agents: x [..., in], W [A,out,in] -> [A, ..., out].
    One GEMM against the agent-stacked weight viewed as [A*out, in] (its weight gradient is then one GEMM landing in
    W's own layout); the result is a permuted view."""
    A, out, n_in = W.shape
    y = torch.nn.functional.linear(x, W.reshape(A * out, n_in), None if b is None else b.reshape(A * out))
    lead = x.shape[:-1]
    y = y.view(*lead, A, out)
    return y.movedim(-2, 0)


class _LinearTInto(torch.autograd.Function):
    """linear_t with its weight / bias gradients written by the backward itself into given views of the flat grad
    buffer (one GEMM + one row sum; no gradient tensor for autograd to return and no copy into the flat buffer
    afterwards). The shared input gets no gradient (replay rows / detached actions). Each parameter must enter ONE
    such call per update (the backward overwrites its view)."""

    @staticmethod
    def forward(ctx, x, W, b, gW, gb):
        ctx.save_for_backward(x)
        ctx.g = (gW, gb)
        return _linear_t(x, W, b)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        gW, gb = ctx.g
        A, out, n_in = gW.shape
        d2 = dy.reshape(A * out, x.shape[0])
        torch.mm(d2, x, out=gW.view(A * out, n_in))
        if gb is not None:
            torch.sum(d2, 1, out=gb.view(A * out))
        return None, None, None, None, None


def _linear_t(x, W, b):
    A, out, n_in = W.shape
    W2 = W.reshape(A * out, n_in)
    if torch.is_grad_enabled() and (x.requires_grad or W.requires_grad or (b is not None and b.requires_grad)):
        # under autograd without gradient views: the functional forms (out= ops are not differentiable)
        y = W2 @ x.t() if b is None else torch.addmm(b.reshape(A * out, 1), W2, x.t())
        return y.view(A, out, x.shape[0])
    y = torch.empty((A, out, x.shape[0]), dtype=x.dtype, device=x.device)  # a base tensor (in-place safe)
    if b is None:
        torch.mm(W2, x.t(), out=y.view(A * out, -1))
    else:
        torch.addmm(b.reshape(A * out, 1), W2, x.t(), out=y.view(A * out, -1))
    return y


def linear_t(x, W, b=None, gW=None, gb=None):
    """Every agent's Linear on ONE input shared by all agents, TRANSPOSED: x [rows, in], W [A, out, in], b [A, out]
    -> y^T [A, out, rows] (contiguous) = one GEMM [A*out, in] x [in, rows] against the agent-stacked weight, so a
    per-agent consumer reads it without a layout copy (bmm takes the transposed operand) and its weight gradient
    [A*out, rows] x [rows, in] lands in W's own layout. gW / gb (views of the flat grad buffer): the backward writes
    the gradients there itself (grads_into(direct=...))."""
    if gW is not None and torch.is_grad_enabled():
        return _LinearTInto.apply(x, W, b, gW, gb)
    return _linear_t(x, W, b)


def blayer_norm(x, w, b, eps=1e-5):
    """Per-agent LayerNorm over the last dim: normalise, then w[A,F], b[A,F] affine."""
    if w.dim() == 1:
        return torch.nn.functional.layer_norm(x, (x.shape[-1],), w, b, eps=eps)
    if w.shape[0] == 1:  # one network: the fused affine LayerNorm kernel (forward and backward)
        return torch.nn.functional.layer_norm(x, (x.shape[-1],), w[0], b[0], eps=eps)
    y = torch.nn.functional.layer_norm(x, (x.shape[-1],), eps=eps)
    return torch.addcmul(b.unsqueeze(1), y, w.unsqueeze(1))


class _GRUCellFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gi, gh, h):
        gi, gh, h = gi.contiguous(), gh.contiguous(), h.contiguous()
        H = h.shape[-1]
        rows = h.numel() // H
        hout = torch.empty_like(h)
        ws = torch.empty(rows * 4 * H, dtype=h.dtype, device=h.device)
        _ops().gru_cell_fwd(gi, gh, h, hout, ws)
        ctx.save_for_backward(h, ws)
        ctx.H = H
        return hout

    @staticmethod
    def backward(ctx, dhout):
        h, ws = ctx.saved_tensors
        H = ctx.H
        rows = h.numel() // H
        dhout = dhout.contiguous()
        dgi = torch.empty(*h.shape[:-1], 3 * H, dtype=h.dtype, device=h.device)
        dgh = torch.empty_like(dgi)
        dh = torch.empty_like(h)
        _ops().gru_cell_bwd(dhout, h, ws, dgi, dgh, dh)
        return dgi, dgh, dh


def gru_cell(x, h, W_ih, W_hh, b_ih, b_hh):
    """nn.GRUCell for A agents at once: x [A,B,in] (or shared [B,in]), h [A,B,H] -> h' [A,B,H]."""
    return gru_cell_gi(blinear(x, W_ih, b_ih), h, W_hh, b_hh)


class _GRUSeqFn(torch.autograd.Function):
    """A chunk of GRUCell steps for A networks in one launch each way (flock_gru_seq_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, gi, W_hh, b_hh, keep, save, gW=None, gb=None):
        A, C, B, G = gi.shape
        H = G // 3
        gi, W_hh, b_hh = gi.contiguous(), W_hh.contiguous(), b_hh.contiguous()
        k8 = keep.view(torch.uint8) if keep.dtype == torch.bool else keep
        hs = torch.empty((A, C, B, H), dtype=gi.dtype, device=gi.device)
        ws = torch.empty((A, C, B, 4 * H), dtype=gi.dtype, device=gi.device) if save else None
        _ops().gru_seq_fwd(gi, W_hh, b_hh, k8, hs, ws)
        if save:
            ctx.save_for_backward(hs, ws, W_hh, k8)
            ctx.g = (gW, gb)
        return hs

    @staticmethod
    def backward(ctx, dhs):
        hs, ws, W_hh, k8 = ctx.saved_tensors
        A, C, B, H = hs.shape
        dhs = dhs.contiguous()
        gW, gb = ctx.g
        direct = gW is not None
        dgi = torch.empty((A, C, B, 3 * H), dtype=hs.dtype, device=hs.device)
        dW = gW if direct else torch.empty_like(W_hh)
        db = gb if direct else torch.empty((A, 3 * H), dtype=hs.dtype, device=hs.device)
        _ops().gru_seq_bwd(dhs, hs, ws, W_hh, k8, dgi, dW, db)
        if direct:  # written into the flat grad buffer's views (grads_into(direct=...))
            return dgi, None, None, None, None, None, None
        return dgi, dW, db, None, None, None, None


def gru_seq(gi, W_hh, b_hh, keep, gW=None, gb=None):
    """GRUCell recurrence of A networks over a chunk of C steps from a zero hidden state: gi [A,C,B,3H] (every
    step's x W_ih^T + b_ih), W_hh [A,3H,H], b_hh [A,3H], keep [C,A,B] bool (False: reset the hidden state after
    that step; may be an expanded view) -> hs [A,C,B,H], each step's output before its reset. gW / gb (contiguous
    [A,3H,H] / [A,3H] views of a flat grad buffer, both or neither): the backward writes W_hh's and b_hh's gradients
    there itself instead of returning them (each parameter in ONE such call per update: the backward overwrites)."""
    assert keep.dim() == 3 and keep.shape == (gi.shape[1], gi.shape[0], gi.shape[2])
    save = torch.is_grad_enabled() and any(t.requires_grad for t in (gi, W_hh, b_hh))
    if (gW is None) != (gb is None) or (gW is not None and not (gW.is_contiguous() and gb.is_contiguous() and
                                                                 gW.shape == W_hh.shape and gb.shape == b_hh.shape)):
        raise ValueError("gru_seq: gW / gb must both be given, contiguous and shaped like W_hh / b_hh")
    return _GRUSeqFn.apply(gi, W_hh, b_hh, keep, save, gW, gb)


class _GRUSeqQFn(torch.autograd.Function):
    """gru_seq with VDN's q head fused (flock_gru_seq_q_fwd / _bwd): returns q [A,C,B,NA] = hs W_q^T + b_q of every
    step's GRU output; the backward takes dq in place of dhs and also yields dW_q, db_q. g: optional grad views of
    (W_hh, b_hh, W_q, b_q) that the backward writes itself (grads_into(direct=...))."""

    @staticmethod
    def forward(ctx, gi, W_hh, b_hh, Wq, bq, keep, save, g=None):
        A, C, B, G = gi.shape
        H, NA = G // 3, Wq.shape[1]
        gi, W_hh, b_hh, Wq, bq = (t.contiguous() for t in (gi, W_hh, b_hh, Wq, bq))
        k8 = keep.view(torch.uint8) if keep.dtype == torch.bool else keep
        f = dict(dtype=gi.dtype, device=gi.device)
        hs = torch.empty((A, C, B, H), **f) if save else None
        ws = torch.empty((A, C, B, 4 * H), **f) if save else None
        q = torch.empty((A, C, B, NA), **f)
        _ops().gru_seq_q_fwd(gi, W_hh, b_hh, Wq, bq, k8, hs, ws, q)
        if save:
            ctx.save_for_backward(hs, ws, W_hh, Wq, k8)
            ctx.g = g
        return q

    @staticmethod
    def backward(ctx, dq):
        hs, ws, W_hh, Wq, k8 = ctx.saved_tensors
        A, C, B, H = hs.shape
        f = dict(dtype=hs.dtype, device=hs.device)
        dgi = torch.empty((A, C, B, 3 * H), **f)
        if ctx.g is not None:
            gW, gb, gWq, gbq = ctx.g
            _ops().gru_seq_q_bwd(dq.contiguous(), hs, ws, W_hh, Wq, k8, dgi, gW, gb, gWq, gbq)
            return dgi, None, None, None, None, None, None, None
        dW, db = torch.empty_like(W_hh), torch.empty((A, 3 * H), **f)
        dWq, dbq = torch.empty_like(Wq), torch.empty((A, Wq.shape[1]), **f)
        _ops().gru_seq_q_bwd(dq.contiguous(), hs, ws, W_hh, Wq, k8, dgi, dW, db, dWq, dbq)
        return dgi, dW, db, dWq, dbq, None, None, None


def gru_seq_q(gi, W_hh, b_hh, Wq, bq, keep, grads=None):
    """gru_seq followed by every agent's q head Linear(H, NA) on every step's output, in one launch each way: gi
    [A,C,B,3H], W_hh [A,3H,H], b_hh [A,3H], Wq [A,NA,H] (NA <= 16), bq [A,NA], keep [C,A,B] -> q [A,C,B,NA] (the
    GRU outputs are not returned). grads: optional contiguous views (gW_hh, gb_hh, gW_q, gb_q) shaped like the
    parameters that the backward writes itself."""
    assert keep.dim() == 3 and keep.shape == (gi.shape[1], gi.shape[0], gi.shape[2])
    if not (Wq.dim() == 3 and 1 <= Wq.shape[1] <= 16 and Wq.shape[2] == W_hh.shape[2]):
        raise ValueError("gru_seq_q: W_q must be [A, NA <= 16, H]")
    if grads is not None:
        grads = tuple(grads)
        if len(grads) != 4 or any(not g.is_contiguous() or g.shape != p.shape
                                  for g, p in zip(grads, (W_hh, b_hh, Wq, bq))):
            raise ValueError("gru_seq_q: grads must be four contiguous views shaped like W_hh, b_hh, W_q, b_q")
    save = torch.is_grad_enabled() and any(t.requires_grad for t in (gi, W_hh, b_hh, Wq, bq))
    return _GRUSeqQFn.apply(gi, W_hh, b_hh, Wq, bq, keep, save, grads)


class _VdnFeatFn(torch.autograd.Function):
    """The VDN QNet feature chain Linear(n_obs,64)-ReLU-Linear(64,32)-ReLU plus the GRUCell input side of every chunk
    step, A agents in ONE launch (flock_vdn_feat_fwd; learners/vdn/net.py:19-33). The backward is the chain rule on
    the saved post-ReLU activations as batched GEMMs (the weight gradients land in each parameter's own layout)."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, Wi, bi, save, fused_bwd=True, grads=None):
        A, C, B, n = x.shape
        R = C * B
        if x.stride(3) != 1:
            x = x.contiguous()
        W1, b1, W2, b2, Wi, bi = (t.contiguous() for t in (W1, b1, W2, b2, Wi, bi))
        dev, f32 = x.device, x.dtype
        gi = torch.empty((A, R, Wi.shape[1]), dtype=f32, device=dev)
        y1 = torch.empty((A, R, W1.shape[1]), dtype=f32, device=dev) if save else None
        y2 = torch.empty((A, R, W2.shape[1]), dtype=f32, device=dev) if save else None
        _ops().vdn_feat_fwd(x, W1, b1, W2, b2, Wi, bi, y1, y2, gi)
        if save:
            ctx.save_for_backward(x, W2, Wi, y1, y2)
            ctx.fused_bwd = bool(fused_bwd)
            ctx.grads = grads
        return gi

    @staticmethod
    def backward(ctx, dgi):
        x, W2, Wi, y1, y2 = ctx.saved_tensors
        A, C, B, n = x.shape
        if ctx.fused_bwd:  # one launch: flock::vdn_feat_bwd (MFMA, the weight gradients accumulated over all rows)
            if ctx.grads is not None:  # straight into the flat grad buffer's views (grads_into(direct=...))
                _ops().vdn_feat_bwd(x, W2, Wi, y1, y2, dgi.contiguous(), *ctx.grads)
                return (None,) * 10
            f = dict(dtype=x.dtype, device=x.device)
            dW1, db1 = torch.empty(A, 64, n, **f), torch.empty(A, 64, **f)
            dW2, db2 = torch.empty(A, 32, 64, **f), torch.empty(A, 32, **f)
            dWi, dbi = torch.empty(A, 96, 32, **f), torch.empty(A, 96, **f)
            _ops().vdn_feat_bwd(x, W2, Wi, y1, y2, dgi.contiguous(), dW1, db1, dW2, db2, dWi, dbi)
            return None, dW1, db1, dW2, db2, dWi, dbi, None, None, None
        dWi = torch.bmm(dgi.transpose(1, 2), y2)
        dbi = dgi.sum(1)
        dz2 = torch.bmm(dgi, Wi).masked_fill_(y2 <= 0, 0.0)     # ReLU backward on the output (y > 0 iff z > 0)
        dW2 = torch.bmm(dz2.transpose(1, 2), y1)
        db2 = dz2.sum(1)
        dz1 = torch.bmm(dz2, W2).masked_fill_(y1 <= 0, 0.0)
        dW1 = torch.bmm(dz1.transpose(1, 2), x.reshape(A, C * B, n))
        db1 = dz1.sum(1)
        if ctx.grads is not None:
            for g, v in zip(ctx.grads, (dW1, db1, dW2, db2, dWi, dbi)):
                g.copy_(v)
            return (None,) * 10
        return None, dW1, db1, dW2, db2, dWi, dbi, None, None, None


def vdn_feat(x, W1, b1, W2, b2, Wi, bi, fused_bwd=True, grads=None):
    """x [A,C,B,n_obs] (any strides with a unit feature stride, e.g. the replay gather's permuted view) -> gi
    [A, C*B, 96] = relu(relu(x W1^T + b1) W2^T + b2) Wi^T + bi per agent (hidden sizes 64 / 32, n_obs <= 16).
    fused_bwd: the backward as one flock::vdn_feat_bwd launch (False: batched GEMMs + masks + sums, the A/B
    baseline). grads: (gW1, gb1, gW2, gb2, gWi, gbi), contiguous views of a flat grad buffer shaped like the
    parameters: the backward writes the six gradients there itself instead of returning them."""
    A, n = x.shape[0], x.shape[3]
    if not (W1.shape == (A, 64, n) and W2.shape == (A, 32, 64) and Wi.shape == (A, 96, 32) and 1 <= n <= 16):
        raise ValueError("vdn_feat: the QNet feature chain n_obs -> 64 -> 32 -> 3 x 32 (n_obs <= 16)")
    if grads is not None:
        grads = tuple(grads)
        if len(grads) != 6 or any(not g.is_contiguous() or g.shape != p.shape
                                  for g, p in zip(grads, (W1, b1, W2, b2, Wi, bi))):
            raise ValueError("vdn_feat: grads must be six contiguous views shaped like W1, b1, W2, b2, Wi, bi")
    save = torch.is_grad_enabled() and any(t.requires_grad for t in (W1, b1, W2, b2, Wi, bi))
    return _VdnFeatFn.apply(x, W1, b1, W2, b2, Wi, bi, save, fused_bwd, grads)


def gru_cell_gi(gi, h, W_hh, b_hh):
    """gru_cell from precomputed input-side gate pre-activations gi = x W_ih^T + b_ih [A,B,3H] (a recurrence can
    compute them for every step at once)."""
    gh = blinear(h, W_hh, b_hh)
    return _GRUCellFn.apply(gi, gh, h)


class StepRing:
    """The replay-ring targets of one env step that writes its transitions itself (flock::step_v2_store /
    step_uw_discrete_store, include/flock_amd.h FlockRing): the ring field tensors [state, action, reward, new_state,
    terminal] (+ the record's actor_state / actor_new_state copies) and meta = [start, skip, group, store_done,
    action_ids, env_done]. The launch-plan path builds the C ABI's FlockRing from it (ops.flock_ring)."""

    def __init__(self, fields, actor_state, actor_new_state, group, store_done, action_ids, env_done):
        self.fields, self.actor_state, self.actor_new_state = list(fields), actor_state, actor_new_state
        self.meta = [0, 0, int(group), int(bool(store_done)), int(bool(action_ids)), int(bool(env_done))]

    def set_start(self, start, skip):
        self.meta[0], self.meta[1] = int(start), int(skip)

    @property
    def start(self):
        return self.meta[0]

    @property
    def skip(self):
        return self.meta[1]


class ReplayRing:
    """Device-resident ring buffer of named row tensors (``fields``: name -> row shape). ``aliases`` {name: target}:
    fields whose every row is, by the caller's construction, the target field's row (gym_flock_v2's critic and actor
    observations are the same dnn rows): one buffer serves both names, written once."""

    def __init__(self, capacity, fields, device, aliases=None):
        self.capacity = int(capacity)
        self.device = torch.device(device)
        self.fields = OrderedDict((k, tuple(v)) for k, v in fields.items())
        self.aliases = dict(aliases or {})
        for a, t in self.aliases.items():
            assert a in self.fields and t in self.fields and t not in self.aliases and self.fields[a] == self.fields[t]
        self._bufs = OrderedDict()
        for k, v in self.fields.items():
            if k not in self.aliases:
                self._bufs[k] = torch.zeros((self.capacity, *v), dtype=torch.float32, device=self.device)
        for a, t in self.aliases.items():
            self._bufs[a] = self._bufs[t]
        self._bufs = OrderedDict((k, self._bufs[k]) for k in self.fields)
        self.counter = 0

    @property
    def bufs(self):
        """name -> [capacity, *row] tensor."""
        return self._bufs

    def __len__(self):
        return min(self.counter, self.capacity)

    def _width(self, name):
        return math.prod(self.fields[name])

    def store(self, rows: dict, one_minus=()):
        """Append n rows per field (all fields the same n) at positions counter..counter+n-1 (mod capacity), every
        field in ONE flock_ring_store launch. rows[name]: [n, *row_shape] (u8 / bool / int64 converted to f32 by the
        kernel, other dtypes by torch); a name in
        ``one_minus`` takes a bool / 0-1 tensor [n] and stores 1 - x (the reference's terminal = 1 - done)."""
        n = next(iter(rows.values())).shape[0]
        if n > self.capacity:  # only the last `capacity` rows survive
            rows = {k: v[n - self.capacity:] for k, v in rows.items()}
            self.counter += n - self.capacity
            n = self.capacity
        if n == 0:
            return
        srcs, dsts, kinds = [], [], []
        for name, val in rows.items():
            if name in self.aliases:  # written through its target field
                continue
            w = self._width(name)
            val = torch.as_tensor(val, device=self.device)
            kind = 0
            if name in one_minus:
                if val.dtype in (torch.bool, torch.uint8):
                    src, kind = val.reshape(n).contiguous(), 1
                else:
                    src = (1.0 - val.reshape(n).float()).contiguous()
            else:
                src = val.reshape(n, -1)
                assert src.shape[1] == w, (name, src.shape, w)
                if src.dtype in (torch.bool, torch.uint8):  # converted in the store kernel
                    src, kind = src.contiguous(), 2
                elif src.dtype == torch.int64:
                    src, kind = src.contiguous(), 3
                else:
                    src = src.float().contiguous()
            srcs.append(src)
            dsts.append(self.bufs[name])
            kinds.append(kind)
        _require_cuda(self.bufs[next(iter(rows))])
        _ops().ring_store(srcs, dsts, kinds, self.counter % self.capacity)
        self.counter += n

    def step_slots(self, n, state, action, reward, new_state, terminal, actor_state=None, actor_new_state=None,
                   group=1, store_done=False, action_ids=False, env_done=False):
        """Reserve the next n rows for an env step that writes them itself (VecFlockEnv.step(ring=...) ->
        flock_step_v2_store) and return the kernel's FlockRing: same rows and counter as store() (when n exceeds
        the capacity only the last `capacity` rows are kept). Field names map the kernel's targets to this ring's
        fields; group = agents per row (1, or N for one row per env); store_done: store done (else 1 - done);
        action_ids: the step's action ids stored as f32 (uw_discrete); env_done: one terminal flag per env row."""
        skip = max(0, n - self.capacity)
        # one StepRing per field mapping, updated in place (ops.flock_ring builds its FlockRing for the launch-plan
        # path, which keeps a pointer to it)
        key = (state, action, reward, new_state, terminal, actor_state, actor_new_state, group, bool(store_done),
               bool(action_ids), bool(env_done))
        rings = self.__dict__.setdefault("_rings", {})
        ring = rings.get(key)
        if ring is None:
            b = self.bufs
            ring = rings[key] = StepRing([b[state], b[action], b[reward], b[new_state], b[terminal]],
                                         None if actor_state is None else b[actor_state],
                                         None if actor_new_state is None else b[actor_new_state], group,
                                         store_done, action_ids, env_done)
        ring.set_start((self.counter + skip) % self.capacity, skip)
        self.counter += n
        return ring

    def scatter(self, name, idx, rows):
        """Write rows at arbitrary positions idx (HIP row scatter)."""
        idx = idx.to(device=self.device, dtype=torch.int64).contiguous()
        src = rows.to(device=self.device, dtype=torch.float32).reshape(idx.numel(), -1).contiguous()
        _ops().scatter_rows(src, idx, self.bufs[name])

    def gather(self, name, idx, out=None):
        """rows idx (any shape of int64 indices) -> [*idx.shape, *row_shape]."""
        idx = idx.to(device=self.device, dtype=torch.int64).contiguous()
        w = self._width(name)
        if out is None:
            out = torch.empty((*idx.shape, *self.fields[name]), dtype=torch.float32, device=self.device)
        _ops().gather_rows(self.bufs[name], idx, out)
        return out


class OverlappedTrain:
    """A learner's train() beside the env steps that follow it (the random-action exploration regime, where the next
    steps do not read the networks): the rows the update samples are copied out of the replay ring on the caller's
    (env) stream — one row gather per field, ordered before the env kernels that overwrite ring rows — and the update
    itself, the learner's own graph-captured code re-captured over this snapshot, runs on a stream of its own. Results
    are bitwise those of train() on the same draws (the same kernels on the same rows). ``sync()`` makes the caller's
    stream wait for the update (before anything reads the networks; bench.py's finish()); ``writes``: the FlatParams
    the update writes, which then sync on it before their host-side reads and writes (FlatParams.sync_writers)."""

    def __init__(self, ring, n_rows, writes=()):
        self.ring = ring
        self.snap = ReplayRing(n_rows, ring.fields, ring.device, aliases=ring.aliases)
        self.snap.counter = n_rows
        # a stream created once per device in C++ (not torch's pool: a pool stream may share the env stream's hardware
        # queue, and the update would then run behind the env steps instead of beside them)
        from .. import torch_ops

        torch_ops.load()
        h = torch.classes.flock.ScPipeline.side_stream(ring.device.index or 0)
        self.stream = torch.cuda.ExternalStream(h, device=ring.device)
        self.done = torch.cuda.Event()
        self.pending = False
        self.graph = None
        for fp in writes:
            fp.writers.append(self)

    def snapshot(self, idx):
        """Rows idx (int64, n_rows in all, any shape) of every field into snapshot rows 0..n_rows-1 in idx's order, on
        the current stream, after the previous update has finished reading the snapshot."""
        cur = torch.cuda.current_stream(self.ring.device)
        if self.pending:
            cur.wait_event(self.done)
        flat = idx.reshape(-1)
        assert flat.numel() == self.snap.capacity
        for name in self.ring.fields:
            if name not in self.ring.aliases:
                self.ring.gather(name, flat, out=self.snap.bufs[name])

    def launch(self, fn):
        """Run fn (enqueues the update) on the update stream, after the current stream's work so far."""
        cur = torch.cuda.current_stream(self.ring.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            fn()
            self.done.record(self.stream)
        self.pending = True

    def sync(self):
        if self.pending:
            torch.cuda.current_stream(self.ring.device).wait_event(self.done)
            self.pending = False


def capture_graph(fn, device, state, warmup=2):
    """Capture ``fn`` (a learner update on static tensors) into a HIP graph. ``state``: tensors the warm-up runs
    mutate (parameters, moments, step counters) — snapshotted and restored so capture has no side effect."""
    snap = [t.clone() for t in state]
    s = torch.cuda.Stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        for _ in range(warmup):
            fn()
    torch.cuda.current_stream(device).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    with torch.no_grad():
        for t, v in zip(state, snap):
            t.copy_(v)
    return g


def uniform_(t, bound, generator=None):
    with torch.no_grad():
        t.uniform_(-bound, bound, generator=generator)
    return t
