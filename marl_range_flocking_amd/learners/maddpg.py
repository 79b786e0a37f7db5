"""MADDPG learners (reference: learners/maddpg_official_rnn/ and learners/maddpg_official/), batched over agents.

Reference behaviour kept:
  * networks (maddpg_official_rnn/net.py:14-146; maddpg_official/net.py:14-115): RNN actor fce(k->32)-GRUCell(32)-
    fc1-ReLU-fc2-ReLU-[(tanh(linear)+1)/2, 1.5 tanh(angular)]; RNN critic fce(N*k->32)-GRUCell-fc1-ReLU-
    fc2([h, a_1..a_N])-ReLU-fc3; feed-forward variants without fce/GRU and a tanh actor head; fanin_init on fc1/fc2
    (U(+-1/sqrt(size[0]))), heads U(+-3e-3), everything else the torch defaults;
  * SuperAgent.train() (rnn MADDPG.py:78-150, ff MADDPG.py:67-108): per agent y_i = r_i + gamma Q'_i(s', mu'(s'))
    (1 - d_i) on the last chunk step, critic MSE, actor loss -mean Q_i(s, mu(s).detach()) with the critic hidden state
    AFTER the last step (Q8); the detach means the actors never receive a gradient (Q6): their Adam steps are no-ops
    and they stay bitwise frozen, while the actor loss does add to the critic gradient; hidden states reset to zero
    where an agent is done; Adam(3e-3) on each critic; soft updates t*(1-tau) + p*tau of both targets;
  * the replay's raw ``actors_action.reshape(B, C, 2N)`` of an [N, B, C, 2] tensor (MADDPG.py:86; ff :75), which
    interleaves agents and batch rows, is reproduced (``reference_action_layout=True``) for parity;
  * ReplayBufferMaddpg (memory_rnn.py:8-99; memory.py:8-99): rows at counter % capacity; minibatch starts drawn
    without replacement from [0, min(counter, capacity) - chunk); chunks are physical row runs (no wrap);
  * OrnsteinUhlenbeckProcess (utils.py:32-55): ONE process shared by all agents and sampled agent after agent (Q9).
What changes: all N actors / critics / targets are stacked [N, ...] slices of flat buffers; every layer of every
agent is one batched GEMM; the GRU elementwise work is flock_gru_fwd/bwd; the N critic Adam steps + target critic
soft updates are ONE flock_adam_step launch; the update replays as one HIP graph; the N sequential OU samples are a
closed-form prefix scan.

Multi-GPU: data-parallel replicas all-reduce the critics' flat gradient (907 M floats at config 5,
3.6 GB per update), or, with agent_shard=True, each rank owns the critics and target actors of N / world agents:
the ranks' sampled minibatches are all-gathered into the union batch (~2 x 21 MB of observations per rank at
config 5), every rank runs its agents' actor heads and critics on it, and the [B', 2] action columns of the actor
heads are all-gathered (every critic reads every agent's action). Per-agent results equal the replicated update on
the union batch; no gradient crosses xGMI.
"""
import math

import torch
import torch.nn.functional as F

from .. import dist
from .core import (FlatParams, OverlappedTrain, ReplayRing, _ops, blinear, capture_graph, gru_cell, gru_seq, linear_t,
                   shared_linear)

HR = 32  # hidden_rnn (net.py:15,100)


def actor_shapes(k, h1, h2, recurrent, n_actions=2):
    if recurrent:
        return {"fce.weight": (HR, k), "fce.bias": (HR,), "gru.weight_ih": (3 * HR, HR), "gru.weight_hh": (3 * HR, HR),
                "gru.bias_ih": (3 * HR,), "gru.bias_hh": (3 * HR,), "fc1.weight": (h1, HR), "fc1.bias": (h1,),
                "fc2.weight": (h2, h1), "fc2.bias": (h2,), "linear_speed.weight": (1, h2), "linear_speed.bias": (1,),
                "angular_speed.weight": (1, h2), "angular_speed.bias": (1,)}
    return {"fc1.weight": (h1, k), "fc1.bias": (h1,), "fc2.weight": (h2, h1), "fc2.bias": (h2,),
            "fc3.weight": (n_actions, h2), "fc3.bias": (n_actions,)}


def critic_shapes(n_agents, k, h1, h2, recurrent, n_actions=2):
    s = {}
    if recurrent:
        s.update({"fce.weight": (HR, n_agents * k), "fce.bias": (HR,), "gru.weight_ih": (3 * HR, HR),
                  "gru.weight_hh": (3 * HR, HR), "gru.bias_ih": (3 * HR,), "gru.bias_hh": (3 * HR,),
                  "fc1.weight": (h1, HR), "fc1.bias": (h1,)})
    else:
        s.update({"fc1.weight": (h1, n_agents * k), "fc1.bias": (h1,)})
    # fc2.weight [h2, h1 + 2N] is kept as its two column blocks (the fc1-output part and the all-agents action
    # part) so each gets its own gradient GEMM (a sliced leaf costs a zero-filled full-size gradient per use);
    # load_reference_state / state_dict split and join it (CRITIC_JOINED)
    s.update({"fc2.weight_h": (h2, h1), "fc2.weight_a": (h2, n_actions * n_agents), "fc2.bias": (h2,),
              "fc3.weight": (1, h2), "fc3.bias": (1,)})
    return s


CRITIC_JOINED = {"fc2.weight": ("fc2.weight_h", "fc2.weight_a")}  # reference name -> stored column blocks


def reference_names(fp):
    """Parameter names in the reference state_dict order (stored column blocks joined back)."""
    out = []
    for n in fp.shapes:
        ref = next((r for r, parts in CRITIC_JOINED.items() if n in parts), n)
        if ref not in out:
            out.append(ref)
    return out


def _init(fp, generator):
    """fanin_init (net.py:9-12) on fc1/fc2 weights, U(+-3e-3) on head weights, torch defaults elsewhere."""
    with torch.no_grad():
        for name, shp in fp.shapes.items():
            layer, kind = name.split(".")
            if layer == "gru":
                b = 1.0 / math.sqrt(HR)
                fp.view(fp.data, name).uniform_(-b, b, generator=generator)
                continue
            kind = "weight" if kind.startswith("weight") else kind
            if layer + ".weight" in fp.shapes:
                w = fp.shapes[layer + ".weight"]
            else:  # column blocks of one joined weight: [out, sum of the blocks' in]
                parts = CRITIC_JOINED[layer + ".weight"]
                w = (fp.shapes[parts[0]][0], sum(fp.shapes[q][1] for q in parts))
            if kind == "weight" and layer in ("fc1", "fc2"):
                b = 1.0 / math.sqrt(w[0])
            elif kind == "weight" and layer in ("fc3", "linear_speed", "angular_speed"):
                b = 3e-3
            else:
                b = 1.0 / math.sqrt(w[1])
            fp.view(fp.data, name).uniform_(-b, b, generator=generator)


def actor_gru(P, x, h):
    """The recurrent actor's GRU step only: x [A,B,k], h [A,B,32] -> h' (the action head is not evaluated)."""
    return gru_cell(blinear(x, P["fce.weight"], P["fce.bias"]), h, P["gru.weight_ih"], P["gru.weight_hh"],
                    P["gru.bias_ih"], P["gru.bias_hh"])


def actor_head(P, h):
    """The recurrent actor after its GRU: h [A,B,32] -> actions [A,B,2]."""
    y = F.relu(blinear(h, P["fc1.weight"], P["fc1.bias"]))
    y = F.relu(blinear(y, P["fc2.weight"], P["fc2.bias"]))
    lin = (torch.tanh(blinear(y, P["linear_speed.weight"], P["linear_speed.bias"])) + 1) / 2  # :65-66
    ang = torch.tanh(blinear(y, P["angular_speed.weight"], P["angular_speed.bias"])) * 1.5       # :69-70
    return torch.cat([lin, ang], dim=-1)


def actor_forward(P, x, h, recurrent):
    """x [A,B,k], h [A,B,32] -> actions [A,B,2], h'."""
    if recurrent:
        h = actor_gru(P, x, h)
        return actor_head(P, h), h
    y = F.relu(blinear(x, P["fc1.weight"], P["fc1.bias"]))
    y = F.relu(blinear(y, P["fc2.weight"], P["fc2.bias"]))
    return torch.tanh(blinear(y, P["fc3.weight"], P["fc3.bias"])), h


def actor_seq(P, x, keep):
    """The recurrent actors' GRU over a whole chunk: x [A,C,B,k], keep [C,A,B] -> hidden outputs [A,C,B,32]
    (each step's, before its done reset). fce and the GRU input GEMM run once for all steps; the recurrence is one
    gru_seq launch."""
    A, C, B, k = x.shape
    y = blinear(x.reshape(A, C * B, k), P["fce.weight"], P["fce.bias"])
    gi = blinear(y, P["gru.weight_ih"], P["gru.bias_ih"]).view(A, C, B, 3 * HR)
    return gru_seq(gi, P["gru.weight_hh"], P["gru.bias_hh"], keep)


def critic_seq(P, x, keep, G=None):
    """The recurrent critics' GRU over a whole chunk: x [C,B,N*k] shared by every critic, keep [C,A,B] ->
    (hidden outputs [A,C,B,32], fce outputs [A,C,B,32] (a transposed view)). fce is one GEMM [A*32, N*k] x
    [N*k, C*B] for every agent and step (linear_t; its weight gradient one GEMM, written into G's views when given),
    the GRU input GEMM one batched GEMM reading it transposed, the recurrence one gru_seq."""
    C, B, _ = x.shape
    G = G or {}
    fxT = linear_t(x.reshape(C * B, -1), P["fce.weight"], P["fce.bias"], G.get("fce.weight"), G.get("fce.bias"))
    A = fxT.shape[0]
    fx = fxT.transpose(1, 2)                                            # [A, C*B, 32], no copy
    gi = blinear(fx, P["gru.weight_ih"], P["gru.bias_ih"]).view(A, C, B, 3 * HR)
    return gru_seq(gi, P["gru.weight_hh"], P["gru.bias_hh"], keep), fx.view(A, C, B, HR)


def critic_gru(P, fx, h):
    """One GRUCell step of the recurrent critics from their fce output fx [A,B,32]: h [A,B,32] -> h'."""
    return gru_cell(fx, h, P["gru.weight_ih"], P["gru.weight_hh"], P["gru.bias_ih"], P["gru.bias_hh"])


def critic_head(P, y, a, G=None):
    """fc2(cat([y, a])) -> ReLU -> fc3: y [A,B,h1] (post-ReLU fc1 output), a [B,2N] shared -> q [A,B,1].
    fc2 runs as its two column blocks (same math, no [A,B,h1+2N] concat), TRANSPOSED so that no GEMM output needs
    a layout copy: z^T [A,h2,B] = W_a a^T + b (one GEMM over every agent, linear_t; gradients into G's views when
    given) + W_h y^T (batched, in place), q^T [A,1,B] = W3 ReLU(z^T) + b3."""
    G = G or {}
    zT = linear_t(a, P["fc2.weight_a"], P["fc2.bias"], G.get("fc2.weight_a"), G.get("fc2.bias"))
    zT = zT.baddbmm_(P["fc2.weight_h"], y.transpose(1, 2))
    qT = torch.baddbmm(P["fc3.bias"].unsqueeze(-1), P["fc3.weight"], F.relu(zT))
    return qT.transpose(1, 2)


def critic_forward(P, x, a, h, recurrent):
    """One reference critic call (net.py:100-146 / :80-115): x [B, N*k] and a [B, 2N] shared by every agent's
    critic; h [A,B,32] -> q [A,B,1], h'."""
    if recurrent:
        y = h = critic_gru(P, shared_linear(x, P["fce.weight"], P["fce.bias"]), h)
        y = F.relu(blinear(y, P["fc1.weight"], P["fc1.bias"]))
    else:
        y = F.relu(shared_linear(x, P["fc1.weight"], P["fc1.bias"]))
    return critic_head(P, y, a), h


class SharedOU:
    """OrnsteinUhlenbeckProcess shared by all agents, sampled agent after agent (utils.py:32-55, MADDPG.py:18,29),
    for E independent envs at once: the N sequential samples are a closed-form prefix scan (float64)."""

    def __init__(self, size, theta, mu, sigma, sigma_min, dt, device, generator, n_steps_annealing=1000,
                 anneal_per_sample=False):
        self.size, self.theta, self.mu, self.dt = size, theta, mu, dt
        self.sigma, self.sigma_min = sigma, sigma_min
        self.m = -float(sigma - sigma_min) / float(n_steps_annealing) if sigma_min is not None else 0.0
        self.c = sigma
        self.n_steps = 0
        self.sample_sigma = sigma
        self.anneal_per_sample = anneal_per_sample  # maddpg_official samples with current_sigma and n_steps += 1
        self.device, self.gen = device, generator
        self.x = None

    @property
    def current_sigma(self):
        smin = self.sigma_min if self.sigma_min is not None else self.sigma
        return max(smin, self.m * float(self.n_steps) + self.c)

    def reset_states(self):
        self.x = None

    def update_sigma(self):
        self.sample_sigma = self.current_sigma
        self.n_steps += 1

    def sample(self, n, envs=1):
        """n sequential samples for each of ``envs`` processes -> [envs, n, size]."""
        if self.x is None or self.x.shape[0] != envs:
            self.x = torch.zeros((envs, self.size), dtype=torch.float64, device=self.device)
        a = 1.0 - self.theta * self.dt
        if self.anneal_per_sample:
            sig = torch.tensor([self.current_sigma] * n, dtype=torch.float64, device=self.device)
            self.n_steps += n
        else:
            sig = torch.full((n,), self.sample_sigma, dtype=torch.float64, device=self.device)
        z = torch.randn((envs, n, self.size), generator=self.gen, device=self.device).double()
        b = self.theta * self.mu * self.dt + sig.view(1, n, 1) * math.sqrt(self.dt) * z
        j = torch.arange(1, n + 1, dtype=torch.float64, device=self.device).view(1, n, 1)
        u = torch.cumsum(b * a ** (-j), dim=1)
        x = a ** j * (self.x[:, None, :] + u)
        self.x = x[:, -1]
        return x.float()


class MADDPGLearner:
    """SuperAgent (both flavours) for N agents: batched acting, device replay, one-launch updates."""

    def __init__(self, n_agents, k, recurrent=True, n_actions=2, hidden1=400, hidden2=300, actor_lr=3e-3,
                 critic_lr=3e-3, gamma=0.99, tau=0.001, batch_size=128, chunk_size=10, buffer_capacity=45_000,
                 min_size_buffer=8_000, ou_theta=0.15, ou_mu=0.0, ou_sigma=0.2, ou_sigma_min=0.001, device="cuda",
                 seed=0, use_graph=True, reference_action_layout=True, dist_group=None, agent_shard=False,
                 shared_obs=False):
        self.device = torch.device(device)
        # shared_obs: every record's actor observations ARE its critic observations (gym_flock_v2's "actors" and
        # "critic" are the same dnn rows, gym_flock_v2.py:110-125, and main.py:34-41 stores both): the replay ring keeps
        # one buffer for each pair (ReplayRing aliases), which the env kernel's fused insert writes once (bitwise the
        # same records and minibatches; 32 B per agent-step less to write at config 5)
        self.shared_obs = bool(shared_obs)
        self._shared_obs_bad = None  # device flag: a shared_obs record whose actor / critic observations differed
        self.gen = torch.Generator(device=self.device).manual_seed(seed)
        self.N, self.k, self.recurrent, self.h1 = n_agents, k, recurrent, hidden1
        self.actor_lr, self.critic_lr, self.gamma, self.tau = actor_lr, critic_lr, gamma, tau
        self.B, self.C = batch_size, (chunk_size if recurrent else 1)
        self.min_size_buffer = min_size_buffer
        self.reference_action_layout = reference_action_layout
        self.actors = FlatParams(actor_shapes(k, hidden1, hidden2, recurrent, n_actions), self.device, n_agents,
                                 target=True, adam=False)  # the actors never get a gradient (Q6)
        self.critics = FlatParams(critic_shapes(n_agents, k, hidden1, hidden2, recurrent, n_actions), self.device,
                                  n_agents, target=True)
        _init(self.actors, self.gen)
        _init(self.critics, self.gen)
        self.actors.hard_update_target()    # agent.py:37-38
        self.critics.hard_update_target()
        self.group = dist_group
        self.distributed = dist.active(dist_group)
        self.shard = bool(agent_shard) and self.distributed
        if self.shard:
            # this rank's agents [a0, a0 + na): their critics (params, targets, Adam) only; the actors stay whole
            # (frozen, Q6: every rank acts for all agents of its envs), their targets are advanced for [a0, a0 + na)
            W, r = torch.distributed.get_world_size(dist_group), torch.distributed.get_rank(dist_group)
            if not recurrent:
                raise NotImplementedError("agent_shard is built for the recurrent MADDPG (config 5)")
            if n_agents % W:
                raise ValueError(f"agent_shard needs n_agents ({n_agents}) divisible by the world size ({W})")
            self.na, self.a0 = n_agents // W, r * (n_agents // W)
            dist.sync_params(self.critics, group=dist_group)
            full = self.critics
            self.critics = FlatParams(full.shapes, self.device, self.na, target=True)
            with torch.no_grad():
                for n in full.shapes:
                    for buf, dst in ((full.data, self.critics.data), (full.target, self.critics.target)):
                        self.critics.view(dst, n).copy_(full.view(buf, n)[self.a0:self.a0 + self.na])
            del full
        self.replay = ReplayRing(buffer_capacity, {
            "state": (n_agents, k), "next_state": (n_agents, k), "actor_state": (n_agents, k),
            "actor_next_state": (n_agents, k), "action": (n_agents, n_actions), "reward": (n_agents,),
            "done": (n_agents,)}, self.device,
            aliases={"actor_state": "state", "actor_next_state": "next_state"} if self.shared_obs else None)
        self.n_games = 0
        self.random_process = SharedOU(n_actions, ou_theta, ou_mu, ou_sigma, ou_sigma_min if recurrent else None,
                                       1e-2, self.device, self.gen, anneal_per_sample=not recurrent)
        self.critic_leaves = self.critics.new_leaves()
        self.static_idx = torch.zeros((self.B, self.C), dtype=torch.int64, device=self.device)
        self.losses = torch.zeros(2, device=self.device)
        self.use_graph = use_graph
        self.graph = None
        if self.distributed:
            dist.sync_params(self.actors, group=dist_group)
            if not self.shard:
                dist.sync_params(self.critics, group=dist_group)

    # ---------------------------------------------------------------- acting
    def init_hidden(self, envs=1):
        return torch.zeros((self.N, envs, HR), device=self.device)

    @torch.no_grad()
    def get_actions(self, actor_states, hidden=None, test=False):
        """actor_states [N, k] (one env) or [E, N, k]; hidden [N, E, 32] -> (actions like actor_states[..., :2],
        hidden'). Noise: the shared OU process, sampled agent after agent (agent.py:53-64)."""
        single = actor_states.dim() == 2
        self.sync()  # an overlapped train() still writing the networks
        x = actor_states.reshape(-1, self.N, self.k).transpose(0, 1)  # [N, E, k]
        E = x.shape[1]
        if hidden is None:
            hidden = self.init_hidden(E)
        P = {n: self.actors.view(self.actors.data, n) for n in self.actors.shapes}
        mu, h = actor_forward(P, x, hidden, self.recurrent)
        mu = mu.transpose(0, 1)  # [E, N, 2]
        if not test:
            mu = mu + self.random_process.sample(self.N, E)
        return (mu[0] if single else mu), h

    def reset_random_process(self):
        self.random_process.reset_states()

    def update_random_process(self):
        self.random_process.update_sigma()

    # ---------------------------------------------------------------- replay
    @property
    def buffer_counter(self):
        return self.replay.counter

    def check_buffer_size(self):
        return self.replay.counter >= self.B and self.replay.counter >= self.min_size_buffer

    def add_record(self, actor_states, actor_next_states, actions, state, next_state, reward, done):
        """ReplayBufferMaddpg.add_record (memory_rnn.py:53-67); a leading env dim stores one record per env."""
        st = torch.as_tensor(state, device=self.device, dtype=torch.float32)
        n = 1 if st.dim() == 2 else st.shape[0]
        f = lambda t, *shape: torch.as_tensor(t, device=self.device, dtype=torch.float32).reshape(n, *shape)  # noqa
        N, k = self.N, self.k
        if self.shared_obs:
            # one device-side check per record, OR-ed into a flag read at the next train() (check_shared_obs): no host
            # sync on the per-step store path
            bad = ((f(actor_states, N, k) != f(state, N, k)).any()
                   | (f(actor_next_states, N, k) != f(next_state, N, k)).any())
            self._shared_obs_bad = bad if self._shared_obs_bad is None else self._shared_obs_bad | bad
        self.replay.store({"state": f(state, N, k), "next_state": f(next_state, N, k),
                           "actor_state": f(actor_states, N, k), "actor_next_state": f(actor_next_states, N, k),
                           "action": f(actions, N, 2), "reward": f(reward, N), "done": f(done, N)})

    def check_shared_obs(self):
        """Raise if a record stored since the last check had actor observations that differ from its critic
        observations (shared_obs=True keeps one copy of them). One host read; train() calls it."""
        bad, self._shared_obs_bad = self._shared_obs_bad, None
        if bad is not None and bool(bad):
            raise ValueError("shared_obs: a record's actor observations must equal its critic observations")

    def replay_slots(self, n_envs):
        """Reserve the next n_envs records for an env step that writes them itself (VecFlockEnv.step(ring=...)):
        the record add_record(obs, next_obs, actions, obs, next_obs, reward, done) of every env, one ring row per
        env (critic and actor observations are the same dnn rows here, as main.py:34-41 passes for v2)."""
        if self.shared_obs:  # the actor fields alias state / next_state: the kernel writes them once
            return self.replay.step_slots(n_envs, "state", "action", "reward", "next_state", "done", group=self.N,
                                          store_done=True)
        return self.replay.step_slots(n_envs, "state", "action", "reward", "next_state", "done",
                                      actor_state="actor_state", actor_new_state="actor_next_state", group=self.N,
                                      store_done=True)

    # ---------------------------------------------------------------- update
    @staticmethod
    def _direct_grads(Pc, names=("fce.weight", "fce.bias", "fc2.weight_a", "fc2.bias")):
        """The critic parameters whose shared-input GEMMs (linear_t) write their gradients straight into the flat
        grad buffer: the two largest blocks (fce [A,32,N*k], fc2's action block [A,h2,2N]: ~85 % of the critic
        parameters at config 5) and their biases. Each enters exactly one linear_t call per update."""
        return {n: Pc[n].grad for n in names if n in Pc}

    def _update(self):
        self._fwd_bwd()
        self._step()

    def _fwd_bwd(self):
        N, B, C, k = self.N, self.B, self.C, self.k
        idx = self.static_idx
        tidx = idx.t().contiguous()                                             # [C, B]: chunk step major
        S = self.replay.gather("state", tidx).reshape(C, B, N * k)
        S2 = self.replay.gather("next_state", tidx).reshape(C, B, N * k)
        AS = self.replay.gather("actor_state", idx).permute(2, 1, 0, 3)        # [N, C, B, k]
        AS2 = self.replay.gather("actor_next_state", idx).permute(2, 1, 0, 3)
        act = self.replay.gather("action", tidx)                                # [C, B, N, 2]
        if self.reference_action_layout:  # actors_action [N,B,C,2].reshape(B,C,2N) (MADDPG.py:86)
            act = act.permute(2, 1, 0, 3).contiguous().reshape(B, C, 2 * N).transpose(0, 1)
        else:
            act = act.reshape(C, B, 2 * N)
        R = self.replay.gather("reward", idx)                                   # [B, C, N]
        D = self.replay.gather("done", idx)
        Pa = {n: self.actors.view(self.actors.data, n) for n in self.actors.shapes}
        Pta = {n: self.actors.view(self.actors.target, n) for n in self.actors.shapes}
        Ptc = {n: self.critics.view(self.critics.target, n) for n in self.critics.shapes}
        Pc = self.critic_leaves
        last = C - 1
        if self.recurrent:
            # MADDPG.py:95-132. critic_values, target_critic_values and the actions are overwritten at every chunk
            # step and read only after the loop, so before the last step only the four GRU recurrences reach the
            # loss: each runs as one whole-chunk gru_seq, and the heads run once, on the last step's hidden states
            # (identical results, C x less head work). hidden[done_mask[:, i]] = 0 is the keep mask (:117-132).
            keep = (D == 0).permute(1, 2, 0)                                # [C, N, B]
            with torch.no_grad():
                y_ta = actor_seq(Pta, AS2, keep)[:, last]
                y_tc = critic_seq(Ptc, S2, keep)[0][:, last]
                y_a = actor_seq(Pa, AS, keep)[:, last]
            G = self._direct_grads(Pc)
            hs_c, fx = critic_seq(Pc, S, keep, G)
            y_c = hs_c[:, last]                                             # the heads see the pre-reset state
            h_c = torch.where(keep[last].unsqueeze(-1), y_c, 0.0)
            with torch.no_grad():
                cta = actor_head(Pta, y_ta).transpose(0, 1).reshape(B, 2 * N)   # torch.cat(..., dim=1)
                tq = critic_head(Ptc, F.relu(blinear(y_tc, Ptc["fc1.weight"], Ptc["fc1.bias"])), cta)
                cpa = actor_head(Pa, y_a).transpose(0, 1).reshape(B, 2 * N)
            # the actor-loss critic call (:137) steps the GRU once more from the reset hidden state; its head and
            # the critic-loss head share one pass over a 2B batch
            h_aq = critic_gru(Pc, fx[:, last], h_c)
            y = F.relu(blinear(torch.cat([y_c, h_aq], 1), Pc["fc1.weight"], Pc["fc1.bias"]))
            qq = critic_head(Pc, y, torch.cat([act[last], cpa], 0), G)
            q, aq = qq[:, :B], qq[:, B:]
        else:  # maddpg_official/MADDPG.py:67-108 (C == 1)
            G = self._direct_grads(Pc, ("fc2.weight_a", "fc2.bias"))
            zero = torch.zeros((N, B, HR), device=self.device)
            with torch.no_grad():
                ta, _ = actor_forward(Pta, AS2[:, 0], zero, False)
                tq, _ = critic_forward(Ptc, S2[0], ta.transpose(0, 1).reshape(B, 2 * N), zero, False)
                pa, _ = actor_forward(Pa, AS[:, 0], zero, False)
                cpa = pa.transpose(0, 1).reshape(B, 2 * N)
            y = F.relu(shared_linear(S[0], Pc["fc1.weight"], Pc["fc1.bias"]))
            qq = critic_head(Pc, torch.cat([y, y], 1), torch.cat([act[0], cpa], 0), G)
            q, aq = qq[:, :B], qq[:, B:]
        r = R[:, last].t().unsqueeze(-1)
        d = D[:, last].t().unsqueeze(-1)
        target = r + self.gamma * tq * (1 - d)                                  # MADDPG.py:135
        critic_loss = ((target - q) ** 2).mean(dim=(1, 2))                      # F.mse_loss per agent (:136)
        actor_loss = -aq.mean(dim=(1, 2))
        self.critics.grads_into(critic_loss.sum() + actor_loss.sum(), Pc, direct=G)
        with torch.no_grad():
            self.losses[0].copy_(critic_loss.detach().mean())
            self.losses[1].copy_(actor_loss.detach().mean())

    # ---------------------------------------------------------------- agent-sharded update (agent_shard=True)
    def _local_batch(self):
        """This rank's sampled rows, in the layouts the update reads (the reference action layout per rank)."""
        N, B, C, k = self.N, self.B, self.C, self.k
        idx = self.static_idx
        tidx = idx.t().contiguous()
        act = self.replay.gather("action", tidx)                                # [C, B, N, 2]
        return {"S": self.replay.gather("state", tidx).reshape(C, B, N * k),
                "S2": self.replay.gather("next_state", tidx).reshape(C, B, N * k),
                "AS": self.replay.gather("actor_state", idx).permute(2, 1, 0, 3),   # [N, C, B, k]
                "AS2": self.replay.gather("actor_next_state", idx).permute(2, 1, 0, 3),
                "act": act.contiguous(),                                         # [C, B, N, 2], raw
                "R": self.replay.gather("reward", idx), "D": self.replay.gather("done", idx)}  # [B, C, N]

    # batch dimension of each field: the union batch is every rank's rows, rank after rank
    _BATCH_DIM = {"S": 1, "S2": 1, "AS": 2, "AS2": 2, "act": 1, "R": 0, "D": 0}

    def _gather_cat(self, t, dim):
        parts = [torch.empty_like(t) for _ in range(torch.distributed.get_world_size(self.group))]
        torch.distributed.all_gather(parts, t.contiguous(), group=self.group)
        return torch.cat(parts, dim)

    def _train_shard(self):
        """One train() of this rank's agents on the union batch (MADDPG.py:78-150 per agent)."""
        lo, hi = self.a0, self.a0 + self.na
        U = {n: self._gather_cat(v, self._BATCH_DIM[n]) for n, v in self._local_batch().items()}
        C = self.C
        Bu = U["S"].shape[1]
        # the action layout is applied to the UNION batch, as one process sampling all Bu rows would
        if self.reference_action_layout:  # actors_action [N,Bu,C,2].reshape(Bu,C,2N) (MADDPG.py:86)
            U["act"] = U["act"].permute(2, 1, 0, 3).contiguous().reshape(Bu, C, 2 * self.N).transpose(0, 1)
        else:
            U["act"] = U["act"].reshape(C, Bu, 2 * self.N)
        last = C - 1
        sl = lambda fp, buf: {n: fp.view(buf, n)[lo:hi] for n in fp.shapes}  # noqa: E731
        Pa, Pta = sl(self.actors, self.actors.data), sl(self.actors, self.actors.target)
        Ptc = {n: self.critics.view(self.critics.target, n) for n in self.critics.shapes}
        Pc = self.critic_leaves
        keep = (U["D"] == 0).permute(1, 2, 0)[:, lo:hi]                      # [C, na, Bu]
        with torch.no_grad():
            y_ta = actor_seq(Pta, U["AS2"][lo:hi], keep)[:, last]
            y_a = actor_seq(Pa, U["AS"][lo:hi], keep)[:, last]
            heads = torch.stack([actor_head(Pta, y_ta), actor_head(Pa, y_a)])  # [2, na, Bu, 2]
            heads = self._gather_cat(heads, 1)                                 # every agent's actions
            cta = heads[0].transpose(0, 1).reshape(Bu, 2 * self.N)
            cpa = heads[1].transpose(0, 1).reshape(Bu, 2 * self.N)
            y_tc = critic_seq(Ptc, U["S2"], keep)[0][:, last]
            tq = critic_head(Ptc, F.relu(blinear(y_tc, Ptc["fc1.weight"], Ptc["fc1.bias"])), cta)
        G = self._direct_grads(Pc)
        hs_c, fx = critic_seq(Pc, U["S"], keep, G)
        y_c = hs_c[:, last]
        h_c = torch.where(keep[last].unsqueeze(-1), y_c, 0.0)
        h_aq = critic_gru(Pc, fx[:, last], h_c)
        y = F.relu(blinear(torch.cat([y_c, h_aq], 1), Pc["fc1.weight"], Pc["fc1.bias"]))
        qq = critic_head(Pc, y, torch.cat([U["act"][last], cpa], 0), G)
        q, aq = qq[:, :Bu], qq[:, Bu:]
        r = U["R"][:, last, lo:hi].t().unsqueeze(-1)
        d = U["D"][:, last, lo:hi].t().unsqueeze(-1)
        target = r + self.gamma * tq * (1 - d)                                  # MADDPG.py:135
        critic_loss = ((target - q) ** 2).mean(dim=(1, 2))
        actor_loss = -aq.mean(dim=(1, 2))
        self.critics.grads_into(critic_loss.sum() + actor_loss.sum(), Pc, direct=G)
        self.critics.adam_step_dev(self.critic_lr, tau=self.tau, target_mode=0)
        for n in self.actors.shapes:  # the target actors of this rank's agents (mode 0, as _step)
            t, p_ = self.actors.view(self.actors.target, n)[lo:hi], self.actors.view(self.actors.data, n)[lo:hi]
            _ops().soft_update(t, p_, float(self.tau), 0)
        with torch.no_grad():
            sums = torch.stack([critic_loss.detach().sum(), actor_loss.detach().sum()])
            torch.distributed.all_reduce(sums, group=self.group)
            self.losses.copy_(sums / self.N)

    def _step(self):
        # critic_optimizer.step() + update_target_networks() (:148-150): one launch for all agents
        self.critics.adam_step_dev(self.critic_lr, tau=self.tau, target_mode=0)
        self.actors.soft_update(self.tau, mode=0)                               # target actor (actor unchanged)

    def train(self, starts=None):
        """SuperAgent.train(): one update of every agent. starts: optional [B] physical chunk starts (parity)."""
        self.sync()  # after a train_overlapped(): its update must land first (same stream order as serial trains)
        self.check_shared_obs()
        if not self.check_buffer_size():
            return None
        rng = min(self.replay.counter, self.replay.capacity)
        hi = rng - self.C if self.recurrent else rng
        if starts is None:  # np.random.choice(hi, B, replace=False)
            starts = torch.randperm(hi, device=self.device, generator=self.gen)[:self.B]
        starts = torch.as_tensor(starts, device=self.device)
        self.static_idx.copy_(starts[:, None] + torch.arange(self.C, device=self.device)[None])
        if self.shard:  # collectives between the phases: eager
            self._train_shard()
            return self.losses
        fn = self._fwd_bwd if self.distributed else self._update
        if self.use_graph:
            if self.graph is None:
                self.graph = capture_graph(fn, self.device, self.critics.state_tensors()
                                           + self.actors.state_tensors() + [self.losses])
            self.graph.replay()
        else:
            fn()
        if self.distributed:  # critic-only all-reduce (the actors get no gradient, Q6), one bucket
            dist.allreduce_mean_(self.critics.grad, self.group)
            self._step()
        return self.losses

    def train_overlapped(self, starts=None):
        """train() beside the env steps that follow (core.OverlappedTrain): the B x C sampled rows are copied out of
        the ring on the current stream, the update runs on a stream of its own; bitwise train() on the same draws.
        Single-process graph path only (the data-parallel and agent-sharded updates call collectives: train())."""
        if self.distributed or self.shard or not self.use_graph:
            return self.train(starts)
        self.check_shared_obs()
        if not self.check_buffer_size():
            return None
        ov = self.__dict__.get("_ov")
        if ov is None:
            ov = self._ov = OverlappedTrain(self.replay, self.B * self.C, writes=(self.critics, self.actors))
            ov.idx = torch.arange(self.B * self.C, device=self.device).view(self.B, self.C)
        rng = min(self.replay.counter, self.replay.capacity)
        hi = rng - self.C if self.recurrent else rng
        if starts is None:  # the same draws as train()
            starts = torch.randperm(hi, device=self.device, generator=self.gen)[:self.B]
        starts = torch.as_tensor(starts, device=self.device)
        ov.snapshot(starts[:, None] + torch.arange(self.C, device=self.device)[None])
        if ov.graph is None:  # _update over the snapshot rows: the same code, its own graph
            saved = self.replay, self.static_idx
            self.replay, self.static_idx = ov.snap, ov.idx
            try:
                ov.graph = capture_graph(self._update, self.device, self.critics.state_tensors()
                                         + self.actors.state_tensors() + [self.losses])
            finally:
                self.replay, self.static_idx = saved
        ov.launch(ov.graph.replay)
        return self.losses

    def sync(self):
        """The current stream waits for an overlapped train() (before anything reads the networks)."""
        ov = self.__dict__.get("_ov")
        if ov is not None:
            ov.sync()

    # ---------------------------------------------------------------- state dicts (reference names)
    def load_reference_state(self, sds):
        """sds: {"actor{i}"|"critic{i}"|"target_actor{i}"|"target_critic{i}": state_dict}."""
        for key, sd in sds.items():
            net = "actor" if "actor" in key else "critic"
            i = int(key[len(key.rstrip("0123456789")):])
            fp = self.actors if net == "actor" else self.critics
            tgt = key.startswith("target")
            if not self.owns(net, i, tgt):  # agent_shard: another rank's critic or target actor
                continue
            if net == "critic" and self.shard:
                i -= self.a0
            for n, v in sd.items():
                if n in CRITIC_JOINED and net == "critic":
                    v = torch.as_tensor(v)
                    lo = 0
                    for part in CRITIC_JOINED[n]:
                        w = fp.shapes[part][1]
                        fp.load(part, v[:, lo:lo + w], agent=i, target=tgt)
                        lo += w
                else:
                    fp.load(n, v, agent=i, target=tgt)

    def owns(self, net, i, target=False):
        """Whether this rank holds agent i's network. agent_shard: the critics, critic targets and target actors of
        agents [a0, a0 + na) only (the others' target actors are never soft-updated here); the frozen actors are
        whole on every rank."""
        if not self.shard or (net == "actor" and not target):
            return True
        return self.a0 <= i < self.a0 + self.na

    def writes(self, net, i, target=False):
        """Whether this rank writes agent i's checkpoint file (one writer per file into a shared save_dir): the owner
        of a sharded network; for networks held whole on every rank (the frozen actors under agent_shard, everything
        of data-parallel replicas) rank i % world, or rank 0 for replicas."""
        if not self.distributed:
            return True
        W, r = torch.distributed.get_world_size(self.group), torch.distributed.get_rank(self.group)
        if self.shard and not (net == "actor" and not target):
            return self.owns(net, i, target)
        return r == (i % W if self.shard else 0)

    def rank_suffix(self):
        """'' on one process; '_rank<r>' for rank-local state (each rank's replay ring holds its own envs)."""
        return f"_rank{torch.distributed.get_rank(self.group)}" if self.distributed else ""

    def state_dict(self, net, i, target=False):
        """Reference state_dict of agent i's actor / critic (agent_shard: only the networks this rank owns)."""
        fp = self.actors if net == "actor" else self.critics
        if not self.owns(net, i, target):
            what = ("target " if target else "") + net
            raise KeyError(f"{what} {i} lives on another rank (this rank holds {self.a0}..{self.a0 + self.na - 1})")
        if net == "critic" and self.shard:
            i -= self.a0
        out = {}
        for n in reference_names(fp):
            if n in CRITIC_JOINED and n not in fp.shapes:
                out[n] = torch.cat([fp.export(p, i, target=target) for p in CRITIC_JOINED[n]], -1).cpu()
            else:
                out[n] = fp.export(n, i, target=target).cpu()
        return out
