"""Recurrent VDN (reference: learners/vdn/), batched over agents on MI355X.

Reference behaviour kept:
  * QNet (learners/vdn/net.py:11-61): per agent Linear(n_obs,64)-ReLU-Linear(64,32)-ReLU-GRUCell(32,32)-Linear(32,|A|),
    nn.Linear / nn.GRUCell default initialisation, ``sample_action`` epsilon-greedy with ONE coin per batch row (:52-58);
  * train() (learners/vdn/train_flock.py:16-43): update_iter x [sample B chunk starts with replacement, run q and
    q_target over the chunk, sum_q = sum_agents Q(s, a), target = sum r + gamma * sum_agents max Q'(s') * (1 - done),
    loss = sum over steps of smooth_l1, reset hidden rows where done], then clip_grad_norm_(5) and Adam(lr);
  * ReplayBufferVDN (utils.py:7-69): deque of whole-swarm transitions, oldest dropped at buffer_limit, chunk starts
    uniform in [0, len - chunk).
What changes: every agent's network is one slice of stacked [A, ...] tensors (batched GEMMs on hipBLASLt, GRU
elementwise in flock_gru_fwd/bwd), one Adam launch for all agents with the clip coefficient read from device
memory (flock_grad_norm: no host sync), the replay ring is device-resident, and one update iteration replays as a
HIP graph.
"""
import math

import torch
import torch.nn.functional as F

from .. import dist
from .core import (gru_seq_q, FlatParams, GradNorm, OverlappedTrain, ReplayRing, blinear, capture_graph, gru_cell,
                   gru_seq, vdn_feat)

HX = 32


def qnet_shapes(n_obs, n_actions, hx=HX, recurrent=True):
    s = {"feat1.weight": (64, n_obs), "feat1.bias": (64,), "feat2.weight": (hx, 64), "feat2.bias": (hx,)}
    if recurrent:
        s.update({"gru.weight_ih": (3 * hx, hx), "gru.weight_hh": (3 * hx, hx), "gru.bias_ih": (3 * hx,),
                  "gru.bias_hh": (3 * hx,)})
    s.update({"q.weight": (n_actions, hx), "q.bias": (n_actions,)})
    return s


def reference_key(name, i):
    """Our stacked name -> the reference QNet state_dict key of agent i (learners/vdn/net.py:19-25)."""
    layer, kind = name.split(".")
    return {"feat1": f"agent_feature_{i}.0.{kind}", "feat2": f"agent_feature_{i}.2.{kind}",
            "gru": f"agent_gru_{i}.{kind}", "q": f"agent_q_{i}.{kind}"}[layer]


class BatchedQNet:
    def __init__(self, n_agents, n_obs, n_actions, recurrent=True, device="cuda", generator=None):
        self.n_agents, self.n_obs, self.n_actions, self.recurrent = n_agents, n_obs, n_actions, recurrent
        self.hx_size = HX
        # forward_seq's feature chain as one fused launch (False: batched GEMMs + ReLU passes, the A/B baseline)
        self.fused_features = True
        # with fused_features: the GRU recurrence and the q head as one launch each way (False: gru_seq + batched
        # GEMM q head, the A/B baseline)
        self.fused_qhead = n_actions <= 16
        self.device = torch.device(device)
        self.P = FlatParams(qnet_shapes(n_obs, n_actions, HX, recurrent), self.device, agents=n_agents)
        with torch.no_grad():  # nn.Linear / nn.GRUCell defaults: U(+-1/sqrt(fan_in)), GRU U(+-1/sqrt(hidden))
            for name, shp in self.P.shapes.items():
                layer = name.split(".")[0]
                fan = HX if layer == "gru" else self.P.shapes[layer + ".weight"][1]
                b = 1.0 / math.sqrt(fan)
                self.P.view(self.P.data, name).uniform_(-b, b, generator=generator)

    def params(self, target=False):
        buf = self.P.target if target else None
        return self.P.params if buf is None else {n: self.P.view(buf, n) for n in self.P.shapes}

    def forward_am(self, x, h, P=None):
        """Agent-major forward: x [A,B,n_obs], h [A,B,H] -> q [A,B,n_actions], h' (QNet.forward net.py:27-37)."""
        P = self.P.params if P is None else P
        y = F.relu(blinear(x, P["feat1.weight"], P["feat1.bias"]))
        y = F.relu(blinear(y, P["feat2.weight"], P["feat2.bias"]))
        if self.recurrent:
            y = gru_cell(y, h, P["gru.weight_ih"], P["gru.weight_hh"], P["gru.bias_ih"], P["gru.bias_hh"])
            h = y
        return blinear(y, P["q.weight"], P["q.bias"]), h

    # parameters whose gradients forward_seq(..., direct_grads=True)'s backward writes into the flat grad buffer
    DIRECT = ("feat1.weight", "feat1.bias", "feat2.weight", "feat2.bias", "gru.weight_ih", "gru.bias_ih",
              "gru.weight_hh", "gru.bias_hh", "q.weight", "q.bias")

    def forward_seq(self, x, keep, P=None, direct_grads=False):
        """A whole chunk, agent-major: x [A,C,B,n_obs], keep [C,B] (False: the hidden state is reset after that
        step, train_flock.py:34-36) -> q [A,C,B,n_actions] from zero initial hidden states. The feature layers, the
        GRU input GEMM and the q head do not depend on the recurrence, so each runs ONCE over all C steps (one
        batched GEMM of C*B rows per agent); the recurrence itself (hidden GEMM, gates, resets) is one gru_seq
        launch. Same per-step math as forward_am. direct_grads (fused feature chain only): the backward writes the
        gradients of DIRECT (without the q head's unless fused_qhead) into self.P.grad's views itself; returns
        (q, the names it writes) for grads_into(direct=...)."""
        P = self.P.params if P is None else P
        A, C, B, n = x.shape
        fused = self.recurrent and n <= 16 and self.fused_features
        G = {k: self.P.view(self.P.grad, k) for k in self.DIRECT} if (direct_grads and fused) else None
        if fused:
            # feat1-ReLU-feat2-ReLU and the GRU input side of every step in one launch (flock_vdn_feat_fwd)
            gi = vdn_feat(x, P["feat1.weight"], P["feat1.bias"], P["feat2.weight"], P["feat2.bias"],
                          P["gru.weight_ih"], P["gru.bias_ih"],
                          grads=None if G is None else [G[k] for k in self.DIRECT[:6]]).view(A, C, B, -1)
        else:
            y = F.relu(blinear(x.reshape(A, C * B, n), P["feat1.weight"], P["feat1.bias"]))
            y = F.relu(blinear(y, P["feat2.weight"], P["feat2.bias"]))
            if self.recurrent:
                gi = blinear(y, P["gru.weight_ih"], P["gru.bias_ih"]).view(A, C, B, -1)
        NA = self.n_actions
        # the fused backward's LDS: B (5 H + NA) + 9 NA H floats of 160 KB (B <= 224 at NA = 10); else gru_seq + GEMMs
        qfits = B * (5 * self.hx_size + NA) + 9 * NA * self.hx_size <= 40960
        if fused and self.fused_qhead and qfits:  # recurrence + q head in one launch each way (flock_gru_seq_q_*)
            q = gru_seq_q(gi, P["gru.weight_hh"], P["gru.bias_hh"], P["q.weight"], P["q.bias"],
                          keep.unsqueeze(1).expand(C, A, B),
                          grads=None if G is None else [G[k] for k in self.DIRECT[6:]])
            return (q, self.DIRECT if G is not None else ()) if direct_grads else q
        if self.recurrent:  # the whole chunk's recurrence in one launch each way (flock_gru_seq_fwd / _bwd)
            hs = gru_seq(gi, P["gru.weight_hh"], P["gru.bias_hh"], keep.unsqueeze(1).expand(C, A, B),
                         gW=None if G is None else G["gru.weight_hh"], gb=None if G is None else G["gru.bias_hh"])
            y = hs.view(A, C * B, self.hx_size)
        q = blinear(y, P["q.weight"], P["q.bias"]).view(A, C, B, -1)  # (its gradients go through autograd)
        return (q, self.DIRECT[:8] if G is not None else ()) if direct_grads else q

    def __call__(self, obs, hidden):
        """Reference layout: obs [B,A,n_obs], hidden [B,A,H] -> (q [B,A,n_actions], hidden [B,A,H])."""
        self.P.sync_writers()  # an overlapped train() still writing these parameters
        q, h = self.forward_am(obs.transpose(0, 1), hidden.transpose(0, 1))
        return q.transpose(0, 1), h.transpose(0, 1)

    def init_hidden(self, batch_size=1):
        return torch.zeros((batch_size, self.n_agents, HX), device=self.device)

    @torch.no_grad()
    def sample_action(self, obs, hidden, epsilon, generator=None):
        """net.py:52-58: one exploration coin per batch row; returns float action ids [B, A]."""
        out, hidden = self(obs, hidden)
        B = out.shape[0]
        mask = torch.rand((B,), device=self.device, generator=generator) <= epsilon
        rnd = torch.randint(0, out.shape[2], (B, out.shape[1]), device=self.device, generator=generator)
        action = torch.where(mask[:, None], rnd, out.argmax(dim=2)).float()
        return action, hidden

    def load_reference_state_dict(self, sd, target=False):
        for name in self.P.shapes:
            for i in range(self.n_agents):
                self.P.load(name, sd[reference_key(name, i)], agent=i, target=target)

    def state_dict(self):
        """Reference key names (so learners/vdn/test_flock.py-style loaders can read it)."""
        out = {}
        self.P.sync_writers()
        for name in self.P.shapes:
            v = self.P.view(self.P.data, name).detach().cpu()
            for i in range(self.n_agents):
                out[reference_key(name, i)] = v[i].clone()
        return out


class VDNLearner:
    def __init__(self, n_agents, n_obs, n_actions, lr=1e-3, gamma=0.99, batch_size=32, chunk_size=10,
                 update_iter=10, grad_clip_norm=5.0, buffer_limit=50_000, recurrent=True, device="cuda", seed=0,
                 use_graph=True, dist_group=None):
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device).manual_seed(seed)
        self.q = BatchedQNet(n_agents, n_obs, n_actions, recurrent, self.device, self.gen)
        self.q.P.target = torch.zeros_like(self.q.P.data)  # q_target lives in the target slot of the same buffer
        self.sync_target()
        self.A, self.n_obs, self.n_actions = n_agents, n_obs, n_actions
        self.lr, self.gamma, self.B, self.grad_clip_norm = lr, gamma, batch_size, grad_clip_norm
        self.chunk = chunk_size if recurrent else 1
        self.update_iter = update_iter
        self.replay = ReplayRing(buffer_limit, {"s": (n_agents, n_obs), "a": (n_agents,), "r": (n_agents,),
                                                "s_prime": (n_agents, n_obs), "done": ()}, self.device)
        self.norm = GradNorm(self.device)
        self.static_idx = torch.zeros((batch_size, self.chunk), dtype=torch.int64, device=self.device)
        self.loss = torch.zeros((), device=self.device)
        self.use_graph = use_graph
        self.graph = None
        self.train_leaves = self.q.P.new_leaves()
        self.group = dist_group
        self.distributed = dist.active(dist_group)
        if self.distributed:  # identical replicas: rank 0's initial parameters everywhere
            dist.sync_params(self.q.P, group=dist_group)

    def attach(self, q, q_target, ring, lr=1e-3, gamma=0.99, batch_size=32, chunk_size=10, update_iter=10,
               grad_clip_norm=5.0, use_graph=True, seed=0):
        """Build the update engine over EXISTING networks (q, q_target: BatchedQNet) and replay ring — the
        reference's train(q, q_target, memory, ...) signature (learners/dropin.py)."""
        self.device = q.device
        self.gen = torch.Generator(device=self.device).manual_seed(seed)
        self.q, self.q_target = q, q_target
        self.A, self.n_obs, self.n_actions = q.n_agents, q.n_obs, q.n_actions
        self.lr, self.gamma, self.B, self.grad_clip_norm = lr, gamma, batch_size, grad_clip_norm
        self.chunk = chunk_size if q.recurrent else 1
        self.update_iter = update_iter
        self.replay = ring
        self.norm = GradNorm(self.device)
        self.static_idx = torch.zeros((batch_size, self.chunk), dtype=torch.int64, device=self.device)
        self.loss = torch.zeros((), device=self.device)
        self.use_graph, self.graph = use_graph, None
        self.train_leaves = q.P.new_leaves()
        self.group, self.distributed = None, False
        return self

    def target_params(self):
        qt = getattr(self, "q_target", None)
        if qt is None:
            return self.q.params(target=True)
        return {n: qt.P.view(qt.P.data, n) for n in qt.P.shapes}

    def sync_target(self):
        """q_target.load_state_dict(q.state_dict()) (train_flock.py:84, :114-115)."""
        self.q.P.hard_update_target()

    def put(self, s, a, r, s_prime, done):
        """memory.put((s, a, r, s', [int(all_done)])) (train_flock.py:102); also accepts a batch of transitions
        (one per env) with a leading dim."""
        s = torch.as_tensor(s, device=self.device, dtype=torch.float32)
        if s.dim() == 2:
            s, a, r, s_prime = s[None], torch.as_tensor(a)[None], torch.as_tensor(r)[None], torch.as_tensor(s_prime)[None]
            done = torch.as_tensor(done, dtype=torch.float32).reshape(1)
        n = s.shape[0]
        # action ids (int64) and done flags (u8 / bool) are converted to f32 inside the one store launch
        self.replay.store({"s": s, "a": torch.as_tensor(a, device=self.device).reshape(n, self.A),
                           "r": torch.as_tensor(r, device=self.device).float().reshape(n, self.A),
                           "s_prime": torch.as_tensor(s_prime, device=self.device).float(),
                           "done": torch.as_tensor(done, device=self.device).reshape(n)})

    def replay_slots(self, n_envs):
        """Reserve the next n_envs rows for a uw_discrete env step that writes its team transitions itself
        (VecFlockEnv.step(ring=...)): the row memory.put((s, a, r, s', [all_done])) of every env
        (train_flock.py:102): previous obs, action ids as f32, rewards, new obs, the env's any_done."""
        return self.replay.step_slots(n_envs, "s", "a", "r", "s_prime", "done", group=self.A, store_done=True,
                                      action_ids=True, env_done=True)

    def size(self):
        return len(self.replay)

    def _iteration(self):
        self._fwd_bwd()
        self._step()

    def _fwd_bwd(self):
        """Loss and backward of one update iteration on static tensors (train_flock.py:18-41); capturable."""
        A, B, C = self.A, self.B, self.chunk
        idx = self.static_idx
        s = self.replay.gather("s", idx).permute(1, 2, 0, 3)          # [C, A, B, n_obs]
        a = self.replay.gather("a", idx).permute(1, 2, 0).long()       # [C, A, B]
        r = self.replay.gather("r", idx).permute(1, 0, 2)             # [C, B, A]
        s2 = self.replay.gather("s_prime", idx).permute(1, 2, 0, 3)
        done = self.replay.gather("done", idx).t()                      # [C, B]
        Pq, Pt = self.train_leaves, self.target_params()
        keep = done == 0                                                # hidden[done_mask] = 0 (:34-36)
        # agent-major whole-chunk tensors [A, C, B, ...] (one GEMM per layer for all steps, BatchedQNet.forward_seq)
        q_out, direct = self.q.forward_seq(s.permute(1, 0, 2, 3), keep, Pq, direct_grads=True)  # [A, C, B, n_act]
        q_a = q_out.gather(3, a.permute(1, 0, 2).unsqueeze(-1)).squeeze(-1)
        sum_q = q_a.sum(dim=0)                                          # [C, B]
        with torch.no_grad():
            qp = self.q.forward_seq(s2.permute(1, 0, 2, 3), keep, Pt)
            max_q = qp.max(dim=3)[0]                                    # [A, C, B]
            target_q = r.sum(dim=2)                                     # [C, B]
            target_q = target_q + self.gamma * max_q.sum(dim=0) * (1 - done)
        # loss += smooth_l1_loss(sum_q_t, target_q_t) over the chunk steps (:29): per-step means, summed in order
        per_step = F.smooth_l1_loss(sum_q, target_q, reduction="none").mean(dim=1)
        steps = per_step.unbind(0)  # one backward node (a stack) instead of C select_backward zero-fill + copy pairs
        loss = steps[0]
        for t in range(1, C):
            loss = loss + steps[t]
        self.q.P.grads_into(loss, Pq, direct=direct)
        with torch.no_grad():
            self.loss.copy_(loss.detach())

    def _step(self):
        scale = self.norm(self.q.P.grad, self.grad_clip_norm)           # clip_grad_norm_(5) (:42)
        self.q.P.adam_step_dev(self.lr, grad_scale=scale[1:])          # Adam (:43)

    def sample_starts(self):
        n = len(self.replay)
        return torch.randint(0, n - self.chunk, (self.B,), device=self.device, generator=self.gen)

    def train_overlapped(self, starts=None):
        """train() beside the env steps that follow (core.OverlappedTrain): the update_iter x B x C sampled rows of
        all iterations are copied out of the ring on the current stream, the iterations run on a stream of their own;
        bitwise train() on the same draws. Single-process graph path only (data-parallel: train())."""
        if self.distributed or not self.use_graph:
            return self.train(starts)
        U, B, C = self.update_iter, self.B, self.chunk
        ov = self.__dict__.get("_ov")
        if ov is None:
            ov = self._ov = OverlappedTrain(self.replay, U * B * C, writes=(self.q.P,))
            ov.idx_all = torch.arange(U * B * C, device=self.device).view(U, B, C)
            ov.static_idx = torch.zeros((B, C), dtype=torch.int64, device=self.device)
        n = len(self.replay)
        base = self.replay.counter - n
        ar = torch.arange(C, device=self.device)
        st = torch.stack([self.sample_starts() if starts is None else torch.as_tensor(starts[it], device=self.device)
                          for it in range(U)])  # the same draws, in the same order, as train()
        ov.snapshot((base + st[:, :, None] + ar[None, None, :]) % self.replay.capacity)
        if ov.graph is None:  # _iteration over the snapshot rows: the same code, its own graph
            saved = self.replay, self.static_idx
            self.replay, self.static_idx = ov.snap, ov.static_idx
            try:
                ov.graph = capture_graph(self._iteration, self.device,
                                         self.q.P.state_tensors() + [self.loss, self.norm.out])
            finally:
                self.replay, self.static_idx = saved

        def run():
            for it in range(U):
                ov.static_idx.copy_(ov.idx_all[it])
                ov.graph.replay()
        ov.launch(run)
        return self.loss

    def sync(self):
        """The current stream waits for an overlapped train() (before anything reads the networks)."""
        ov = self.__dict__.get("_ov")
        if ov is not None:
            ov.sync()

    def train(self, starts=None):
        """train(q, q_target, memory, optimizer, gamma, batch_size, update_iter, chunk_size) for every agent at
        once. starts: optional [update_iter, B] logical chunk starts (parity tests); returns the last loss."""
        self.sync()  # after a train_overlapped(): its update must land first (same stream order as serial trains)
        n = len(self.replay)
        base = self.replay.counter - n  # logical index 0 = oldest row still in the ring
        ar = torch.arange(self.chunk, device=self.device)
        for it in range(self.update_iter):
            st = self.sample_starts() if starts is None else torch.as_tensor(starts[it], device=self.device)
            self.static_idx.copy_((base + st[:, None] + ar[None, :]) % self.replay.capacity)
            fn = self._fwd_bwd if self.distributed else self._iteration
            if self.use_graph:
                if self.graph is None:
                    self.graph = capture_graph(fn, self.device,
                                               self.q.P.state_tensors() + [self.loss, self.norm.out])
                self.graph.replay()
            else:
                fn()
            if self.distributed:  # one RCCL all-reduce of the whole flat gradient, then identical steps
                dist.allreduce_mean_(self.q.P.grad, self.group)
                self._step()
        return self.loss
