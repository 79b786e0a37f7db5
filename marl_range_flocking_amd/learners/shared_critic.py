"""Shared-critic DDPG learner (reference: learners/maddpg_shared_critic/), batched over agents on MI355X.

Reference behaviour kept (learners/maddpg_shared_critic/{agent_simple_shared_critic,ddpg_network,utils}.py):
  * one CriticNetwork shared by every agent and used as its own target (Q11, :63,76); per-agent actors with target
    copies; LayerNorm MLPs fc1 -> LN -> ReLU -> fc2 -> LN (+ ReLU(action_value(a))) -> ReLU -> q (ddpg_network.py:58-70),
    actor fc1 -> LN -> ReLU -> fc2 -> LN -> ReLU -> mu -> tanh (:132-141); reference initialisations (:35-53, :106-127);
  * learn(i) == Agent.learn() of agent i (:115-155): sample B rows with replacement, y = r + gamma Q(s', mu'_i(s')) *
    notdone, critic MSE + Adam(beta), actor loss -mean Q(s, mu_i(s)) + Adam(alpha), every update_rate-th call of that
    agent the soft update (critic with itself tau*c + (1-tau)*c, target actor tau*a + (1-tau)*t, :158-185);
  * ReplayBuffer (utils.py:28-76) semantics: rows in insertion order, terminal stored as 1 - done.
What changes: all actors live in one agent-major flat buffer (per-agent Adam = one launch over the agent's slice),
the replay ring is device-resident (HIP scatter/gather rows, no CPU round trip), choose_action runs every agent's
actor in one batched GEMM chain, and the OU noise is a per-(env, agent) device process.

learn() has two implementations with the same semantics:
  * fused (default): flock_sc_critic_update + flock_sc_actor_update (csrc/flock_sc.hip), five HIP launches each,
    reading the replay rows, the agent's actor slice and the critic in place, Adam in the last launch. The bench
    loop's native pipeline (pipeline_learn) runs the critic phase of learn t and the actor phase of learn t-1 as one
    round of five launches (flock_sc_round); data-parallel replicas (dp_learn) run the round as gradients, ONE
    all-reduce of the [critic | actor] bucket and one Adam launch (flock_sc_round_adam);
  * autograd (fused=False): the same update written with torch ops and the batched helpers of core.py.
"""
import math

import torch
import torch.nn.functional as F

from .. import dist
from .core import FlatParams, ReplayRing, _ops, blayer_norm, blinear, capture_graph


def critic_shapes(input_dim, fc1=400, fc2=300, n_actions=2):
    return {"fc1.weight": (fc1, input_dim), "fc1.bias": (fc1,), "bn1.weight": (fc1,), "bn1.bias": (fc1,),
            "fc2.weight": (fc2, fc1), "fc2.bias": (fc2,), "bn2.weight": (fc2,), "bn2.bias": (fc2,),
            "action_value.weight": (fc2, n_actions), "action_value.bias": (fc2,),
            "q.weight": (1, fc2), "q.bias": (1,)}


def actor_shapes(input_dim, fc1=400, fc2=300, n_actions=2):
    return {"fc1.weight": (fc1, input_dim), "fc1.bias": (fc1,), "bn1.weight": (fc1,), "bn1.bias": (fc1,),
            "fc2.weight": (fc2, fc1), "fc2.bias": (fc2,), "bn2.weight": (fc2,), "bn2.bias": (fc2,),
            "mu.weight": (n_actions, fc2), "mu.bias": (n_actions,)}


def critic_forward(P, state, action):
    """ddpg_network.py:58-70. P: name -> [A, ...]; state [A,B,in] or [B,in]; action [A,B,n] or [B,n]."""
    sv = blinear(state, P["fc1.weight"], P["fc1.bias"])
    sv = F.relu(blayer_norm(sv, P["bn1.weight"], P["bn1.bias"]))
    sv = blinear(sv, P["fc2.weight"], P["fc2.bias"])
    sv = blayer_norm(sv, P["bn2.weight"], P["bn2.bias"])
    av = F.relu(blinear(action, P["action_value.weight"], P["action_value.bias"]))
    return blinear(F.relu(sv + av), P["q.weight"], P["q.bias"])


def actor_forward(P, state):
    """ddpg_network.py:132-141."""
    x = blinear(state, P["fc1.weight"], P["fc1.bias"])
    x = F.relu(blayer_norm(x, P["bn1.weight"], P["bn1.bias"]))
    x = blinear(x, P["fc2.weight"], P["fc2.bias"])
    x = F.relu(blayer_norm(x, P["bn2.weight"], P["bn2.bias"]))
    return torch.tanh(blinear(x, P["mu.weight"], P["mu.bias"]))


def _init_mlp(fp, names_uniform, generator):
    """Reference init: fc1/fc2 U(+-1/sqrt(out_features)) (note: size()[0]), heads U(+-0.003), LayerNorm (1, 0),
    action_value nn.Linear default U(+-1/sqrt(in_features))."""
    with torch.no_grad():
        for name, shp in fp.shapes.items():
            v = fp.view(fp.data, name)
            if name.startswith("bn"):
                v.fill_(1.0 if name.endswith("weight") else 0.0)
                continue
            layer = name.split(".")[0]
            if layer in ("fc1", "fc2"):
                bound = 1.0 / math.sqrt(fp.shapes[layer + ".weight"][0])
            elif layer in ("q", "mu"):
                bound = 0.003
            else:
                bound = 1.0 / math.sqrt(fp.shapes[layer + ".weight"][1])
            v.uniform_(-bound, bound, generator=generator)


class SharedCriticLearner:
    def __init__(self, n_agents, input_dim, n_actions=2, fc1=400, fc2=300, alpha=3e-4, beta=3e-4, gamma=0.99,
                 tau=0.001, batch_size=256, update_rate=3, buffer_size=1_000_000, device="cuda", seed=0,
                 ou_sigma=0.15, ou_theta=0.2, ou_dt=1e-2, use_graph=True, dist_group=None, fused=True,
                 snapshot=False, replay=None, n_slots=2, handoff="gate", dp_split=False, dp=None, dp_rccl=True,
                 learner_priority="high"):
        self.device = torch.device(device)
        self.n_agents, self.input_dim, self.n_actions = n_agents, input_dim, n_actions
        self.alpha, self.beta, self.gamma, self.tau = alpha, beta, gamma, tau
        self.batch_size, self.update_rate = batch_size, update_rate
        self.gen = torch.Generator(device=self.device).manual_seed(seed)
        self.seed = int(seed)
        self._learn_calls = 0
        self.critic = FlatParams(critic_shapes(input_dim, fc1, fc2, n_actions), self.device, agents=1)
        self.actors = FlatParams(actor_shapes(input_dim, fc1, fc2, n_actions), self.device, agents=n_agents,
                                 agent_major=True, target=True, agent_pad=64)
        _init_mlp(self.critic, None, self.gen)
        _init_mlp(self.actors, None, self.gen)
        self.actors.hard_update_target()  # update_network_parameters(tau=1) (:81)
        self.count = [0] * n_agents
        # replay: an existing ring from make_replay (the drop-in ReplayBuffer allocates it before the learner)
        self.replay = replay if replay is not None else self.make_replay(buffer_size, input_dim, n_actions,
                                                                           self.device)
        self.ou = dict(sigma=ou_sigma, theta=ou_theta, dt=ou_dt)
        self.ou_state = None
        # the update runs on static tensors so it can be replayed as one HIP graph: agent i's actor is copied into
        # a scratch slot (params, target, Adam moments, step) and back around the replay
        self.scratch = FlatParams(actor_shapes(input_dim, fc1, fc2, n_actions), self.device, agents=1, target=True,
                                  agent_pad=64)
        self.actor_steps = torch.zeros(n_agents, dtype=torch.int64, device=self.device)
        self.static_idx = torch.zeros(batch_size, dtype=torch.int64, device=self.device)
        self.losses = torch.zeros(2, dtype=torch.float32, device=self.device)
        self.use_graph = use_graph
        self.graph = None
        self.critic_leaves = self.critic.new_leaves(squeeze=True)
        self.scratch_leaves = self.scratch.new_leaves(squeeze=True)
        self.group = dist_group
        # dp: None = data-parallel when the group has more than one rank; True = the data-parallel path even on one
        # rank (its collectives then run over a one-rank communicator: the RCCL path tested on a one-GPU box)
        self.distributed = dist.active(dist_group) if dp is None else bool(
            dp and torch.distributed.is_available() and torch.distributed.is_initialized())
        # fused data-parallel path: gradients are all-reduced as sums and the Adam kernels scale them by 1 / world
        # (bitwise the mean for power-of-two worlds)
        self.inv_world = (torch.full((1,), 1.0 / torch.distributed.get_world_size(dist_group), device=device)
                          if self.distributed else None)
        self.graphs = None
        if self.distributed:
            dist.sync_params(self.critic, group=dist_group)
            dist.sync_params(self.actors, group=dist_group)
        self.fused = fused
        self.fc1, self.fc2 = fc1, fc2
        # snapshot (fused only): learn() first copies its B sampled rows out of the ring (flock_sc_prep_snapshot)
        # into one of two staging slots and the update reads that copy, so the ring may be rewritten while the
        # update runs (snapshot_into / update_slot: the copy on the env stream, the update on another one)
        self.snapshot = bool(snapshot and fused)
        self.n_slots = max(2, int(n_slots))
        # the native pipeline's snapshot hand-off (pipeline()): "gate" the device-side gate polled by the critic row
        # blocks, "event" a cross-queue event wait
        if handoff not in ("gate", "event"):
            raise ValueError("handoff is 'gate' or 'event'")
        self.handoff = handoff
        # the native pipeline's learner stream: one per (device, priority) for the whole process, created in C++
        # (ScPipeline.stream), not taken from torch's stream pool, whose streams share hardware queues with the env
        # stream once a process holds more streams than GPU_MAX_HW_QUEUES (the same loop then serialises: 0.084 vs
        # 0.125 ms per step, profiles/r05/rccl_host/host_cost_q4.txt). "high": the device's greatest priority, whose
        # streams HIP keeps on hardware queues of their own, apart from every normal-priority stream
        if learner_priority not in ("high", "normal"):
            raise ValueError("learner_priority is 'high' or 'normal'")
        self.learner_priority = learner_priority
        self._learner_stream = None
        # data-parallel pipelines: the actor half of each round all-reduced and stepped off the learner chain, over a
        # second process group of the same ranks (flock_sc_pipeline_set_dp_actor); created here, collectively
        self.dp_split = bool(dp_split and self.distributed and self.snapshot)
        # the native pipeline's collectives as direct RCCL calls when the group's backend is RCCL ("nccl"): c10d
        # ProcessGroup calls from the C++ loop cost tens of microseconds of host time each. One rank over RCCL on one
        # GPU (tools/rccl_host_cost.py, profiles/r05/rccl_host/): single GPU 0.084 ms per step; unsplit rounds 0.112
        # (c10d) / 0.091 (direct RCCL); split rounds (dp_split) 0.205 / 0.150: the split's extra chain work (a
        # second critic all-reduce, a cross-stream wait, the separate Adam launches) costs more than the actor
        # all-reduce it takes off the chain, so the unsplit round is the default
        self.dp_rccl = bool(dp_rccl)
        self.actor_group = None
        if self.dp_split:
            ranks = torch.distributed.get_process_group_ranks(dist_group) if dist_group is not None else None
            self.actor_group = torch.distributed.new_group(ranks=ranks)
        if fused:
            self._init_fused()

    # ------------------------------------------------------------------ fused HIP update (csrc/flock_sc.hip)
    def _init_fused(self):
        dev = self.device
        B, n_in, na = self.batch_size, self.input_dim, self.n_actions
        self.static_agent = torch.zeros(1, dtype=torch.int64, device=dev)
        n_ws = _ops().sc_workspace_floats(B, n_in, na, self.fc1, self.fc2)
        self.sc_workspace = torch.zeros(int(n_ws), dtype=torch.float32, device=dev)
        self.sc_counters = torch.zeros(2, dtype=torch.int32, device=dev)
        # critic views (FlockScUpdate.critic_view): the critic phase writes the post-Adam critic into a view and the
        # self soft update into critic.data; the actor phase reads the view. One view and one workspace per staging
        # slot let the critic phase of learn t+1 run beside the actor phase of learn t (pipeline(), flock_sc_round).
        ns = self.n_slots if self.snapshot else 2
        self.critic_views = [torch.zeros_like(self.critic.data) for _ in range(ns)]
        self.sc_workspaces = [self.sc_workspace] + [torch.zeros_like(self.sc_workspace) for _ in range(ns - 1)]
        rb = self.replay.bufs
        C, A = self.critic, self.actors
        # the update as torch.ops.flock.sc_round arguments (csrc/flock_torch_learn.cpp): the learner state, one job per
        # phase ([idx, agent, 5 replay-row fields, workspace, critic_view(, actor_grad_out)]), sizes, rates
        rows = lambda d: [d["state"], d["new_state"], d["action"], d["reward"], d["terminal"]]  # noqa: E731
        self._sc_learner = [C.data, C.grad, C.exp_avg, C.exp_avg_sq, C.step_dev, A.data, A.grad, A.exp_avg,
                            A.exp_avg_sq, A.target, self.actor_steps, self.losses, self.sc_counters]
        self._sc_dims = [B, n_in, na, self.fc1, self.fc2, self.update_rate, 1]
        self._sc_dims_grads = [B, n_in, na, self.fc1, self.fc2, 0, 0]
        self._sc_hyper = [self.alpha, self.beta, self.gamma, 0.9, 0.999, 1e-8, self.tau]
        self._sc_job = [self.static_idx, self.static_agent, *rows(rb), self.sc_workspace, self.critic_views[0]]
        # data-parallel gradient phases read the critic itself (no critic view: Adam runs between the phases)
        self._no_view = torch.empty(0, device=dev)
        self._sc_job_grads = self._sc_job[:8] + [self._no_view]
        self._ring_rows = rows(rb)
        self._slots = []
        self._pipe = None
        if self.snapshot:
            self.identity_idx = torch.arange(B, dtype=torch.int64, device=dev)
            if self.distributed:
                # data-parallel rounds: the critic gradient and the round's actor gradient in ONE contiguous bucket
                # (FlockScUpdate.critic_grad / actor_grad_out), all-reduced as one collective per env step
                ct = C.numel
                self.dp_actor_off = -(-ct // 64) * 64
                self.dp_bucket = torch.zeros(self.dp_actor_off + A.per_agent, device=dev)
            for i in range(self.n_slots):
                stg = {"state": torch.zeros(B, n_in, device=dev), "new_state": torch.zeros(B, n_in, device=dev),
                       "action": torch.zeros(B, na, device=dev), "reward": torch.zeros(B, device=dev),
                       "terminal": torch.zeros(B, device=dev)}
                agent_t = torch.zeros(1, dtype=torch.int64, device=dev)
                self._slots.append(dict(staging=stg, agent=agent_t, graph=None, graph_c=None, graph_a=None,
                                        job=[self.identity_idx, agent_t, *rows(stg), self.sc_workspaces[i],
                                             self.critic_views[i]],
                                        job_grads=[self.identity_idx, agent_t, *rows(stg), self.sc_workspaces[i],
                                                   self._no_view]))
                if self.distributed:
                    self._slots[-1]["dp_job"] = self._slots[-1]["job"] + [self.dp_bucket[self.dp_actor_off:]]
            if self.distributed:  # the learner state with the critic gradient in the bucket
                self._sc_learner_dp = list(self._sc_learner)
                self._sc_learner_dp[1] = self.dp_bucket[:C.numel]
            self._dp_pending = None
            self.staging = self._slots[0]["staging"]

    def _fused_update(self, job=None, dims=None):
        """One learn() as two torch.ops.flock.sc_round launches sets: its critic phase, then its actor phase."""
        T = _ops()
        job = self._sc_job if job is None else job
        dims = self._sc_dims if dims is None else dims
        T.sc_round(self._sc_learner, job, [], dims, self._sc_hyper)
        T.sc_round(self._sc_learner, [], job, dims, self._sc_hyper)

    def _fused_state(self):
        """Everything one fused update writes (graph-capture warm-ups are undone on these): the actor targets too,
        which the in-kernel soft update moves."""
        A = self.actors
        return self.critic.state_tensors() + [A.data, A.target, A.exp_avg, A.exp_avg_sq, self.actor_steps,
                                              self.losses] + self.critic_views

    def _run_fused(self, agent, slot=None):
        S = self._slots[slot] if slot is not None else None
        job = S["job"] if S is not None else self._sc_job
        if self.distributed:
            job = S["job_grads"] if S is not None else self._sc_job_grads
        if not self.distributed:
            if not self.use_graph:
                return self._fused_update(job)
            g = S["graph"] if S is not None else self.graph
            if g is None:
                g = capture_graph(lambda: self._fused_update(job), self.device, self._fused_state())
                if S is not None:
                    S["graph"] = g
                else:
                    self.graph = g
            return g.replay()
        # data-parallel: gradient-only kernels, RCCL all-reduce (sum) of each network's gradient, then the Adam
        # steps with grad_scale = 1 / world; the actor's target soft update (:180-185) rides in its Adam launch
        T = _ops()
        T.sc_round(self._sc_learner, job, [], self._sc_dims_grads, self._sc_hyper)
        dist.allreduce_sum_(self.critic.grad, self.group)
        self.critic.adam_step_dev(self.beta, grad_scale=self.inv_world)
        T.sc_round(self._sc_learner, [], job, self._sc_dims_grads, self._sc_hyper)
        A = self.actors
        lo, hi = A.agent_range(agent)
        dist.allreduce_sum_(A.grad[lo:hi], self.group)
        self.actor_steps[agent:agent + 1].add_(1)
        soft = self.count[agent] % self.update_rate == 0
        T.adam_step(A.data[lo:hi], A.grad[lo:hi], A.exp_avg[lo:hi], A.exp_avg_sq[lo:hi],
                    self.actor_steps[agent:agent + 1], self.inv_world, A.target[lo:hi] if soft else None,
                    float(self.alpha), 0.9, 0.999, 1e-8, float(self.tau) if soft else 0.0, 1 if soft else 0)

    # ------------------------------------------------------------------ acting
    def _stacked(self, fp, target=False):
        return {n: fp.view(fp.target if target else fp.data, n) for n in fp.shapes}

    def fused_act_ok(self):
        """The widths flock_sc_act handles (the reference's 400 / 300 / 2 among them)."""
        return (self.n_actions == 2 and 1 <= self.input_dim <= 16 and self.fc1 % 8 == 0 and self.fc1 >= 8
                and 1 <= self.fc2 <= 320)

    @torch.no_grad()
    def choose_action(self, obs, noise=True, fused=None):
        """All agents at once: obs [..., n_agents, input_dim] -> actions [..., n_agents, n_actions] (mu + OU noise,
        agent_simple_shared_critic.py:92-107; OUActionNoiseGPU utils.py:6-26 with one process per (env, agent)).
        fused (default: when the widths allow): ONE flock_sc_act launch computes every agent's actor on every row
        and the OU step (csrc/flock_act.hip); else the batched torch GEMM chain below."""
        lead = obs.shape[:-2]
        if fused is None:
            fused = self.fused_act_ok()
        if fused:
            x = obs.reshape(-1, self.n_agents, self.input_dim)
            x = x if x.dtype == torch.float32 and x.is_contiguous() else x.float().contiguous()
            act = torch.empty((x.shape[0], self.n_agents, 2), dtype=torch.float32, device=self.device)
            ou = z = None
            if noise:
                shape = (*lead, self.n_agents, 2)
                if self.ou_state is None or tuple(self.ou_state.shape) != shape:
                    self.ou_state = torch.zeros(shape, dtype=torch.float32, device=self.device)
                z = torch.randn(shape, device=self.device, generator=self.gen).view(x.shape[0], self.n_agents, 2)
                ou = self.ou_state.view(x.shape[0], self.n_agents, 2)
            o = self.ou
            _ops().sc_act(x, self.actors.data, act, ou, z, self.fc1, self.fc2, float(o["theta"]), float(o["dt"]),
                          float(o["sigma"] * math.sqrt(o["dt"])))
            return act.view(*lead, self.n_agents, 2)
        x = obs.reshape(-1, self.n_agents, self.input_dim).transpose(0, 1)  # [A, rows, in]
        mu = actor_forward(self._stacked(self.actors), x).transpose(0, 1).reshape(*lead, self.n_agents,
                                                                                  self.n_actions)
        if not noise:
            return mu
        if self.ou_state is None or self.ou_state.shape != mu.shape:
            self.ou_state = torch.zeros_like(mu)
        o = self.ou
        z = torch.randn(mu.shape, device=self.device, generator=self.gen)
        self.ou_state = self.ou_state + o["theta"] * (0.0 - self.ou_state) * o["dt"] + o["sigma"] * math.sqrt(
            o["dt"]) * z
        return mu + self.ou_state

    def reset_noise(self):
        self.ou_state = None

    # ------------------------------------------------------------------ replay
    @staticmethod
    def make_replay(capacity, input_dim, n_actions, device):
        """The ReplayBuffer arrays (utils.py:29-45) as one device ring."""
        return ReplayRing(capacity, {"state": (input_dim,), "new_state": (input_dim,), "action": (n_actions,),
                                     "reward": (1,), "terminal": ()}, device)

    @staticmethod
    def store_rows(ring, state, action, reward, new_state, done):
        """ReplayBuffer.store_transitions (utils.py:47-54): rows [n, ...]; terminal stored as 1 - done."""
        n = state.shape[0]
        ring.store({"state": state.reshape(n, -1), "new_state": new_state.reshape(n, -1),
                    "action": action.reshape(n, -1), "reward": reward.reshape(n, 1),
                    "terminal": done.reshape(n)}, one_minus=("terminal",))

    def store_transitions(self, state, action, reward, new_state, done):
        self.store_rows(self.replay, state, action, reward, new_state, done)

    def replay_slots(self, n):
        """Reserve the next n replay rows for an env step that writes its transitions itself
        (VecFlockEnv.step(ring=...) -> flock_step_v2_store); same rows and counter as store_transitions (when n
        exceeds the capacity only the last `capacity` transitions are kept, as ReplayRing.store does)."""
        return self.replay.step_slots(n, "state", "action", "reward", "new_state", "terminal")

    @property
    def mem_cntr(self):
        return self.replay.counter

    def sample_indices(self):
        return torch.randint(0, len(self.replay), (self.batch_size,), device=self.device, generator=self.gen)

    # ------------------------------------------------------------------ learning
    def _update(self):
        self._critic_phase()
        self._critic_step()
        self._actor_phase()
        self._actor_step()

    def _critic_phase(self):
        """Sample, targets and critic backward (agent_simple_shared_critic.py:118-140); capturable."""
        B = self.batch_size
        idx = self.static_idx
        self._state = state = self.replay.gather("state", idx)
        action = self.replay.gather("action", idx)
        reward = self.replay.gather("reward", idx)
        new_state = self.replay.gather("new_state", idx)
        terminal = self.replay.gather("terminal", idx)
        C = self.critic_leaves
        tgt = {n: self.scratch.view(self.scratch.target, n)[0] for n in self.scratch.shapes}
        with torch.no_grad():
            target_actions = actor_forward(tgt, new_state)                    # :126
            q_next = critic_forward(C, new_state, target_actions)             # :127 (target critic == critic)
            target = reward.view(B, 1) + self.gamma * q_next * terminal.reshape(-1, 1)  # :130
        q = critic_forward(C, state, action)                                  # :128
        critic_loss = F.mse_loss(target, q)                                   # :139
        self.critic.grads_into(critic_loss, C)                                # zero_grad + backward (:138-140)
        with torch.no_grad():
            self.losses[1].copy_(critic_loss.detach())

    def _critic_step(self):
        self.critic.adam_step_dev(self.beta)                                  # :141

    def _actor_phase(self):
        """Actor loss through the UPDATED critic and its backward (:144-149); capturable."""
        C, S = self.critic_leaves, self.scratch_leaves
        mu = actor_forward(S, self._state)                                    # :145
        actor_loss = torch.mean(-critic_forward(C, self._state, mu))          # :147-148
        self.scratch.grads_into(actor_loss, S)                                # zero_grad + backward (:144-149)
        with torch.no_grad():
            self.losses[0].copy_(actor_loss.detach())

    def _actor_step(self):
        self.scratch.adam_step_dev(self.alpha)                                # :150

    def _run_update(self):
        S = self.scratch
        state = self.critic.state_tensors() + S.state_tensors() + [self.losses]
        if not self.distributed:
            if not self.use_graph:
                return self._update()
            if self.graph is None:
                self.graph = capture_graph(self._update, self.device, state)
            return self.graph.replay()
        # data-parallel: graph-captured backward phases, RCCL all-reduce of each gradient bucket, identical steps
        if self.use_graph and self.graphs is None:
            self._critic_phase()  # materialise self._state before capturing the actor phase
            self.graphs = (capture_graph(self._critic_phase, self.device, state),
                           capture_graph(self._actor_phase, self.device, state))
        (self.graphs[0].replay() if self.use_graph else self._critic_phase())
        dist.allreduce_mean_(self.critic.grad, self.group)
        self._critic_step()
        (self.graphs[1].replay() if self.use_graph else self._actor_phase())
        dist.allreduce_mean_(S.grad, self.group)
        self._actor_step()

    def learn(self, agent, idx=None):
        """Agent.learn() of agent ``agent`` (agent_simple_shared_critic.py:115-155). Returns (actor_loss,
        critic_loss, True) as device tensors (no host sync), or (0, 0, False) before the buffer holds a batch."""
        B = self.batch_size
        self.replay.bufs  # noqa: B018 (a loop with direct learns may have left the newest rows in a ring copy)
        if self.replay.counter < B:
            return 0, 0, False
        self._learn_calls += 1
        if self.fused:
            # one launch: agent index + (unless given) B rows uniform with replacement (utils.py:65-76)
            if idx is not None:
                self.static_idx.copy_(torch.as_tensor(idx).to(self.device))
            if self.snapshot:  # slot 0, one stream
                if idx is not None:  # injected rows: copy them out of the ring by index
                    S = self._slots[0]
                    for n, v in S["staging"].items():
                        v.copy_(self.replay.bufs[n][self.static_idx].reshape(v.shape))
                    S["agent"].fill_(int(agent))
                else:
                    self._learn_calls -= 1
                    self.snapshot_into(0, agent)
                return self.update_slot(0, agent)
            else:
                _ops().sc_prep(self.static_agent, None if idx is not None else self.static_idx, len(self.replay),
                               self.seed, self._learn_calls, int(agent))
            self._run_fused(agent)
            return self._finish_learn(agent, soft_in_kernel=not self.distributed, actor_soft_done=self.distributed)
        if idx is None:                                                       # utils.py:65-76 (with replacement)
            torch.randint(0, len(self.replay), (B,), device=self.device, generator=self.gen, out=self.static_idx)
        else:
            self.static_idx.copy_(torch.as_tensor(idx).to(self.device))
        lo, hi = self.actors.agent_range(agent)
        A, S = self.actors, self.scratch
        with torch.no_grad():
            for src, dst in ((A.data, S.data), (A.target, S.target), (A.exp_avg, S.exp_avg),
                             (A.exp_avg_sq, S.exp_avg_sq)):
                dst.copy_(src[lo:hi])
            S.step_dev.copy_(self.actor_steps[agent:agent + 1])
        self._run_update()
        with torch.no_grad():
            for src, dst in ((S.data, A.data), (S.exp_avg, A.exp_avg), (S.exp_avg_sq, A.exp_avg_sq)):
                dst[lo:hi].copy_(src)
            self.actor_steps[agent:agent + 1].copy_(S.step_dev)
        return self._finish_learn(agent)

    def snapshot_into(self, slot, agent):
        """learn() prologue of ``agent`` into staging slot 0 or 1, enqueued on the current stream: sample the B rows
        (utils.py:65-76) and copy them out of the ring. Returns False (nothing enqueued) before the buffer holds a
        batch. The ring may be rewritten once this has run; update_slot(slot) must follow before the slot is reused."""
        B = self.batch_size
        if not self.snapshot:
            raise RuntimeError("snapshot_into needs SharedCriticLearner(snapshot=True)")
        self.replay.bufs  # noqa: B018 (see learn)
        if self.replay.counter < B:
            return False
        self._learn_calls += 1
        S = self._slots[slot]
        stg = S["staging"]
        _ops().sc_prep_snapshot(self._ring_rows, [stg["state"], stg["new_state"], stg["action"], stg["reward"],
                                                  stg["terminal"]], S["agent"], self.static_idx, len(self.replay),
                                self.seed, self._learn_calls, int(agent))
        return True

    def _phase(self, slot, phase):
        """Enqueue the critic ("c": flock_sc_critic_update) or actor ("a": flock_sc_actor_update) phase of the
        update on staging slot ``slot`` on the current stream (one HIP graph replay per phase)."""
        S = self._slots[slot]
        T = _ops()
        job = S["job"]

        def run():
            if phase == "c":
                T.sc_round(self._sc_learner, job, [], self._sc_dims, self._sc_hyper)
            else:
                T.sc_round(self._sc_learner, [], job, self._sc_dims, self._sc_hyper)

        if not self.use_graph:
            return run()
        key = "graph_" + phase
        if S[key] is None:
            S[key] = capture_graph(run, self.device, self._fused_state())
        S[key].replay()

    def update_slot_pipelined(self, slot, agent, critic_stream, actor_stream, after_actor=None, critic_done=None):
        """update_slot as two phases on two streams (single GPU): the critic phase on critic_stream, the actor
        phase on actor_stream behind it. The critic phase of the NEXT learn() may then run beside this actor phase:
        it reads critic.data (post-soft) while this actor phase reads critic_views[slot] (post-Adam), and each slot
        has its own workspace. Ordering the caller must provide: the critic phase of a learn whose agent equals the
        previous learn's waits for that actor phase (it reads the target actor that actor phase soft-updates), and
        a slot is reused only after its previous actor phase (``after_actor``: an event recorded behind it).
        Results are bitwise those of update_slot."""
        if self.distributed:
            raise RuntimeError("update_slot_pipelined is the single-GPU path")
        done_c = critic_done if critic_done is not None else torch.cuda.Event()
        with torch.cuda.stream(critic_stream):
            self._phase(slot, "c")
            done_c.record(critic_stream)
        with torch.cuda.stream(actor_stream):
            actor_stream.wait_event(done_c)
            self._phase(slot, "a")
            if after_actor is not None:
                after_actor.record(actor_stream)
        return self._finish_learn(agent, soft_in_kernel=True)

    @property
    def learner_stream(self):
        """The stream the native pipeline's rounds run on (torch.cuda.ExternalStream over ScPipeline.stream)."""
        if self._learner_stream is None:
            from .. import torch_ops

            torch_ops.load()
            h = torch.classes.flock.ScPipeline.stream(self.device.index or 0, self.learner_priority == "high")
            self._learner_stream = torch.cuda.ExternalStream(h, device=self.device)
        return self._learner_stream

    def pipeline(self):
        """The native learn() pipeline (torch.classes.flock.ScPipeline over flock_sc_pipeline_*, include/flock_learn.h)
        over the n_slots staging slots: per learn() the minibatch snapshot on the env stream and ONE round (this
        learn's critic phase with the previous learn's actor phase, flock_sc_round) on the learner stream, enqueued by
        one call. ONE object per learner: the per-step path (pipeline_learn) and the C++ training loop
        (ScTrainLoop) share its slots and its pending actor phase. The round waits for its snapshot on the device-side
        gate (handoff="gate", single-GPU and data-parallel pipelines alike, for a learn whose env step was marked:
        pipeline_mark; not when ranks share a GPU) or on a cross-queue event. Data-parallel learners (dist_group) run every
        round as gradients, one RCCL all-reduce of the critic gradient over the group and the critic Adam launch on
        the learner stream; with dp_split (opt-in) the round's actor gradient is all-reduced over a second group and
        stepped on the pipeline's actor stream, off the learner chain (set_dp_actor); without, one all-reduce of the
        [critic | actor] bucket (set_dp; dp_learn's rounds, enqueued from C++)."""
        if self._pipe is None:
            if not (self.snapshot and self.fused):
                raise RuntimeError("the native pipeline needs a fused learner with snapshot=True")
            from .. import torch_ops

            torch_ops.load()
            slots = [t for S in self._slots for t in S["job"]]
            p = torch.classes.flock.ScPipeline(self._sc_learner, slots, self._ring_rows, self._sc_dims,
                                               self._sc_hyper)
            if self.distributed:
                group = self.group if self.group is not None else torch.distributed.group.WORLD
                # the c10d ProcessGroup as the TorchScript object the C++ class takes (ProcessGroup.boxed())
                p.set_dp(group.boxed(), self.dp_bucket, self.critic.numel, self.dp_actor_off, self.inv_world)
                if self.dp_split:  # one actor gradient buffer per slot, all-reduced over actor_group off the chain
                    self.dp_actor_grads = [torch.zeros(self.actors.per_agent, device=self.device)
                                           for _ in range(self.n_slots)]
                    p.set_dp_actor(self.actor_group.boxed(), self.dp_actor_grads)
                if self.dp_rccl and torch.distributed.get_backend(group) == "nccl":
                    # the collectives as direct RCCL calls on the pipeline's streams (ScPipeline.set_rccl): unique ids
                    # made on the group's first rank, sent to the others over the group itself
                    ids = torch.zeros(3, 128, dtype=torch.uint8, device=self.device)
                    ranks = torch.distributed.get_process_group_ranks(group)
                    if torch.distributed.get_rank() == ranks[0]:
                        for i in range(3):
                            ids[i].copy_(torch.classes.flock.ScPipeline.rccl_unique_id())
                    torch.distributed.broadcast(ids, src=ranks[0], group=group)
                    ids = ids.cpu()
                    p.set_rccl([ids[i].contiguous() for i in range(3)], ranks.index(torch.distributed.get_rank()),
                               len(ranks), self.learner_stream.cuda_stream)
            # ranks sharing one GPU (gloo rehearsals and tests: more ranks than devices) take the event hand-off: a
            # device-side wait needs its producer's queue to be scheduled, and with many processes' queues on one GPU
            # the hardware scheduler time-slices them, so a round could spin (high priority) while its snapshot's
            # queue waits for a slice
            shared = self.distributed and torch.distributed.get_world_size(self.group) > torch.cuda.device_count()
            p.set_gate(self.handoff == "gate" and not shared)
            self._pipe = p
        return self._pipe

    def pipeline_mark(self, env_stream, wait=True):
        """The device gate's guard (ScPipeline.mark) for the NEXT pipeline_learn: call it before enqueueing that
        learn's env step on env_stream (raw handle). wait=True: the learn's round first waits on the learner stream
        for an event behind everything env_stream holds now, so the gate spins only over the env step that follows;
        wait=False: the caller guarantees that nothing but its own env step is enqueued on env_stream between the
        previous learn and the next one. A pipeline_learn without a mark takes the cross-queue event hand-off (it never
        spins behind work of unknown length). No-op before the ring holds a batch (that learn enqueues nothing)."""
        if self.replay.counter >= self.batch_size:
            self.pipeline().mark(int(env_stream), bool(wait))

    def pipeline_learn(self, agent, env_stream, learner_stream):
        """Enqueue learn(agent) through the native pipeline (raw stream handles): the snapshot on env_stream, the
        round on learner_stream. The actor phase stays pending until the next call or pipeline_flush. Returns False
        (nothing enqueued) before the buffer holds a batch, like snapshot_into. The snapshot hand-off is the device
        gate when pipeline_mark was called since the previous learn (and handoff="gate"), else an event wait."""
        if self.replay.counter < self.batch_size:
            return False
        self._learn_calls += 1
        self.pipeline().learn(len(self.replay), self.seed, self._learn_calls, int(agent), int(env_stream),
                              int(learner_stream))
        self._finish_learn(agent, soft_in_kernel=True)
        return True

    def pipeline_flush(self, learner_stream):
        """Enqueue the pending actor phase of the last pipeline_learn (no-op when none)."""
        if self._pipe is not None:
            self._pipe.flush(int(learner_stream))

    def pipeline_check(self):
        """Raise if a round gave up waiting for its minibatch snapshot (the device-side gate's bounded wait,
        flock_sc_pipeline_check): its update is invalid. Synchronous; call after synchronising."""
        if self._pipe is not None:
            self._pipe.verify()

    # ------------------------------------------------------------------ data-parallel rounds (bench, N > 1)
    def _dp_round(self, c, a):
        """One data-parallel round on the current stream: critic phase of slot c and / or actor phase of slot a
        (None: absent) as gradients (flock_sc_round, do_adam = 0), ONE all-reduce (sum) of the bucket part they
        wrote, then flock_sc_round_adam with grad_scale = 1 / world."""
        T = _ops()
        S = self._slots
        job = lambda i: S[i]["dp_job"] if i is not None else []  # noqa: E731
        L = self._sc_learner_dp
        T.sc_round(L, job(c), job(a), self._sc_dims_grads, self._sc_hyper)
        lo = 0 if c is not None else self.dp_actor_off
        hi = self.dp_bucket.numel() if a is not None else self.critic.numel
        dist.allreduce_sum_(self.dp_bucket[lo:hi], self.group)
        T.sc_round_adam(L, job(c), job(a), self._sc_dims, self._sc_hyper, self.inv_world)

    def dp_learn(self, slot, agent, slot_free):
        """learn() of ``agent`` on the rows snapshot_into(slot, agent) copied, data-parallel, enqueued on the current
        (learner) stream: its critic phase in one round with the previous learn's pending actor phase (the same
        agent twice: one after the other). slot_free[i] is recorded once slot i's actor phase is enqueued."""
        q = self._dp_pending
        if q is not None and q[1] != agent:
            self._dp_round(slot, q[0])
            slot_free[q[0]].record()
        else:
            if q is not None:
                self._dp_round(None, q[0])
                slot_free[q[0]].record()
            self._dp_round(slot, None)
        self._dp_pending = (slot, agent)
        return self._finish_learn(agent, soft_in_kernel=True)

    def dp_flush(self, slot_free):
        """Enqueue the pending actor phase of the last dp_learn (no-op when none)."""
        q = self._dp_pending
        if q is not None:
            self._dp_round(None, q[0])
            slot_free[q[0]].record()
            self._dp_pending = None

    def update_slot(self, slot, agent):
        """The rest of learn() on the rows snapshot_into(slot, agent) copied, enqueued on the current stream."""
        self._run_fused(agent, slot)
        return self._finish_learn(agent, soft_in_kernel=not self.distributed, actor_soft_done=self.distributed)

    def _finish_learn(self, agent, soft_in_kernel=False, actor_soft_done=False):
        if self.count[agent] % self.update_rate == 0 and not soft_in_kernel:                         # :152-154
            self.critic.soft_update(self.tau, mode=1, self_update=True)       # :172-178 (critic is its own target)
            if not actor_soft_done:
                self.actors.soft_update(self.tau, mode=1, agent=agent)        # :180-185
        self.count[agent] += 1
        return self.losses[0], self.losses[1], True

    # ------------------------------------------------------------------ state dicts (reference key names)
    def load_reference_state(self, critic_sd, actor_sds, target_actor_sds=None):
        """actor_sds / target_actor_sds: a list over agents, or {agent index: state_dict} for a subset."""
        for n, v in critic_sd.items():
            self.critic.load(n, v, agent=0)
        for sds, target in ((actor_sds, False), (target_actor_sds, True)):
            for i, sd in (sds.items() if isinstance(sds, dict) else enumerate(sds or ())):
                for n, v in sd.items():
                    self.actors.load(n, v, agent=i, target=target)

    def critic_state_dict(self):
        return {n: self.critic.export(n, 0).cpu() for n in self.critic.shapes}

    def actor_state_dict(self, i, target=False):
        return {n: self.actors.export(n, i, target=target).cpu() for n in self.actors.shapes}


class SharedCriticBench:
    """bench.py hook for BASELINE config 3: after each vectorized env step, insert every agent's transition into the
    replay ring and run ONE learn() (agent round-robin, B=256)."""

    def __init__(self, env, device, seed=0, fused=True, overlap=True, n_slots=None, buffer_size=1_000_000,
                 handoff="gate", dp_split=False, dp=None, dp_rccl=True, pipelined=True, high_priority=None,
                 learner_priority="high"):
        self.env = env
        group = torch.distributed.group.WORLD if dist.active() else None  # replicas synced over RCCL
        # overlap: learn(s) runs on its own stream once its minibatch snapshot is taken, concurrently with env step
        # s+1 (which rewrites the ring); in this loop the actions do not come from the actor (random-action
        # exploration), so step s+1 does not depend on learn(s) and every kernel still sees the same data
        # (with data-parallel replicas the update's two all-reduces run on the learner stream too)
        self.overlap = bool(overlap and fused)
        if n_slots is None:  # staging slots (3: the env stream runs at most two learns ahead of the learner)
            n_slots = 3
        self.learner = SharedCriticLearner(env.N, env.k, device=device, seed=seed, batch_size=256,
                                           buffer_size=buffer_size, dist_group=group, fused=fused,
                                           snapshot=self.overlap, n_slots=n_slots, handoff=handoff, dp_split=dp_split,
                                           dp=dp, dp_rccl=dp_rccl, learner_priority=learner_priority)
        if self.overlap:
            # single GPU: learn() runs as two phases, the actor phase of learn s beside the critic phase of learn s+1:
            # with graphs, the native pipeline (one merged six-launch round per step on self.stream,
            # SharedCriticLearner.pipeline_learn); without, two streams (update_slot_pipelined).
            # pipelined=False keeps one serial learn() per step on self.stream (data-parallel: the Python dp_learn
            # rounds). Data-parallel learners run the same native pipeline, every round as gradients + one RCCL
            # all-reduce + the Adam launch (SharedCriticLearner.pipeline, set_dp).
            self.pipelined = bool(pipelined)
            if self.pipelined and self.learner.use_graph:
                # the native pipeline: its rounds on the learner's own stream (SharedCriticLearner.learner_stream)
                self.stream = self.learner.learner_stream
                self.actor_stream = None
            else:
                # stream priority (high_priority; default: high only for the non-pipelined one-stream learner): with
                # the two pipelined streams high priority made steps 2-3x slower in fresh processes
                # (tools/cu_mask_probe.py)
                hi = (not self.pipelined) if high_priority is None else bool(high_priority)
                prio = torch.cuda.Stream.priority_range()[1] if hi else 0
                self.stream = torch.cuda.Stream(device=device, priority=prio)
                self.actor_stream = torch.cuda.Stream(device=device, priority=prio) if self.pipelined else None
            self.critic_done = [torch.cuda.Event(), torch.cuda.Event()]
            self._handles = None
            ns = self.learner.n_slots
            self.snap_done = [torch.cuda.Event() for _ in range(ns)]
            self.learn_done = [torch.cuda.Event(), torch.cuda.Event()]
            self.slot_free = [torch.cuda.Event() for _ in range(ns)]
            self._used = [False] * ns
            self._dp_slot = 0
            self._prev_agent = None
        self.prev_obs = env.dnn.clone()
        self.prev_act = None
        self._loop = None
        self._looped = False

    # ---------------------------------------------------------------- K steps per call (torch.classes.flock)
    def loop(self):
        """torch.classes.flock.ScTrainLoop over this bench's env, replay ring and the learner's pipeline
        (csrc/flock_torch_loop.cpp): K steps of [env step with the fused replay insert, learn()] enqueued by one C++
        call, bitwise the per-step path of before() / env.step(ring=...) / after(). Overlapped native pipeline only;
        data-parallel learners included (the pipeline's rounds then carry the RCCL all-reduce)."""
        if self._loop is None:
            env, L = self.env, self.learner
            if not self.can_loop():
                raise RuntimeError("ScTrainLoop is the overlapped config-3 loop (v2, native learn() pipeline)")
            from .. import torch_ops

            torch_ops.load()
            c = env.cfg
            b0, b1 = env._bufs
            none = torch.empty(0, device=env.device)
            opt = lambda t: none if t is None else t  # noqa: E731
            e = [env.positions, env.headings, env.velocities, b0["dnn"], b1["dnn"], opt(b0["idx"]), opt(b1["idx"]),
                 env.reward, env.done, env.any_done, opt(env.seeds)]
            ef = [env.box, c.sensor_range, c.collision_distance, c.dt, c.v_min, c.max_linear_velocity]
            ei = [env.k, int(bool(c.periodic)), int(bool(c.rigid_boundary)), int(c.step_launches), env._cur]
            rb = L.replay.bufs
            ring = [rb["state"], rb["action"], rb["reward"], rb["new_state"], rb["terminal"]]
            self._loop = torch.classes.flock.ScTrainLoop(e, ef, ei, ring, L.replay.counter, L.pipeline(), L.seed,
                                                         L._learn_calls)
        return self._loop

    def can_loop(self):
        return (self.overlap and self.pipelined and self.learner.use_graph and self.env.cfg.variant == "v2")

    def run_steps(self, first, K, actions, events=(), ev_every=1):
        """Steps first .. first + K - 1 (actions[s % len(actions)] at step s) through the loop, then the Python
        mirrors (env parity and step count, ring counter, learn counters) brought up to date. The loop first takes
        the Python objects' current values (set_state): per-step steps (step(), env.step(ring=before(s))) may have
        run since its last call."""
        lp = self.loop()
        env, L = self.env, self.learner
        handles = []
        for ev in events:
            if not int(ev.cuda_event):  # torch creates the HIP event at its first record
                ev.record()
            handles.append(int(ev.cuda_event))
        lp.set_state(env._cur, L.replay.counter, L._learn_calls)
        lp.run(int(first), int(K), list(actions), torch.cuda.current_stream(env.device).cuda_stream,
               self.stream.cuda_stream, handles, int(ev_every))
        parity, counter, calls = lp.state()
        learns = calls - L._learn_calls
        for s in range(first + K - learns, first + K):
            L.count[s % L.n_agents] += 1
        L._learn_calls, L.replay.counter = calls, counter
        env._cur = parity
        env.steps += K
        from .. import vec_env

        vec_env._DEVICE_WRITES[0] += K
        self._looped = True

    def describe(self):
        return (f"maddpg_shared_critic learn() x1 per vectorized step ("
                f"{'fused HIP update' if self.learner.fused else 'autograd update'}, B={self.learner.batch_size}, "
                f"agent = step mod "
                f"{self.learner.n_agents}; all {self.env.E * self.env.N} transitions inserted into a 1e6-row "
                f"device replay ring per step by the env kernel itself"
                + (")" if not self.learner.distributed else
                   "; critic gradient all-reduce on the learner chain, the actor's on a second group and stream)"
                   if getattr(self.learner, "dp_split", False) else
                   "; one [critic | actor] gradient all-reduce over RCCL per learn)"))

    # bench.py hook interface: before(s) -> ring for the fused env step; after(s, a) -> learn(); prime()
    def before(self, s):
        slots = self.learner.replay_slots(self.env.E * self.env.N)
        if self.overlap and self.pipelined and self.learner.use_graph:
            # the device gate's guard of this step's learn (after the slots: it marks only a step that will learn),
            # before the env step is enqueued on the current (env) stream
            self.learner.pipeline_mark(torch.cuda.current_stream(self.learner.device).cuda_stream)
        return slots

    def after(self, s, action):
        L = self.learner
        agent = s % L.n_agents
        if not self.overlap:
            L.learn(agent)
            return
        # the snapshot goes on the env stream right behind the env step (the next env step follows it in order);
        # the update runs on the learner stream; staging slots alternate, and a slot is refilled only after the
        # update that read it two steps ago has finished
        if self.pipelined and L.use_graph:
            # the native pipeline (the same ScPipeline object the C++ loop drives): snapshot on the env stream, then
            # one round (this critic phase + the previous learn's actor phase; data-parallel: as gradients, one RCCL
            # all-reduce and the Adam launch) on self.stream (stream handles cached at the first call: the env stream
            # is the stream current then)
            if self._handles is None:
                self._handles = (torch.cuda.current_stream(L.device).cuda_stream, self.stream.cuda_stream)
            L.pipeline_learn(agent, *self._handles)
            return
        main = torch.cuda.current_stream(L.device)
        if L.distributed:
            # data-parallel: snapshot on the env stream, then one round of gradients, ONE all-reduce of the
            # [critic | actor] bucket and the Adam launch on the learner stream (SharedCriticLearner.dp_learn)
            slot = self._dp_slot
            if self._used[slot]:
                main.wait_event(self.slot_free[slot])
            if not L.snapshot_into(slot, agent):
                return
            self.snap_done[slot].record(main)
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(self.snap_done[slot])
                L.dp_learn(slot, agent, self.slot_free)
            self._used[slot] = True
            self._dp_slot = (slot + 1) % L.n_slots
            return
        slot = s & 1
        if self._used[slot]:
            main.wait_event(self.learn_done[slot])
        if not L.snapshot_into(slot, agent):
            return
        self.snap_done[slot].record(main)
        if self.pipelined:
            # critic phase on self.stream, actor phase on self.actor_stream; learn_done[slot] = its actor phase.
            # Slot reuse waits above (snapshot behind learn_done[slot]) cover the view and workspace of the slot.
            self.stream.wait_event(self.snap_done[slot])
            if agent == self._prev_agent:  # same agent: its target actor is soft-updated by the previous actor phase
                self.stream.wait_event(self.learn_done[slot ^ 1])
            L.update_slot_pipelined(slot, agent, self.stream, self.actor_stream, after_actor=self.learn_done[slot],
                                    critic_done=self.critic_done[slot])
            self._prev_agent = agent
        else:
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(self.snap_done[slot])
                L.update_slot(slot, agent)
                self.learn_done[slot].record(self.stream)
        self._used[slot] = True

    def finish(self):
        """Enqueue the pending actor phase (native pipeline) and join the learner stream(s) into the current one
        (end of a timed region)."""
        if self.overlap:
            if self._looped or self._handles is not None:  # one pipeline object: the loop's and the per-step path's
                self.learner.pipeline_flush(self.stream.cuda_stream)
            if self.learner.distributed and self.learner.__dict__.get("_dp_pending") is not None:
                with torch.cuda.stream(self.stream):
                    self.learner.dp_flush(self.slot_free)
            cur = torch.cuda.current_stream(self.learner.device)
            cur.wait_stream(self.stream)
            if self.actor_stream is not None:
                cur.wait_stream(self.actor_stream)

    def prime(self):
        self.finish()

    def step(self, s, action):
        """One bench step with the replay insert fused into the env kernel (flock_step_v2_store), then learn()."""
        self.env.step(action, ring=self.before(s))
        self.after(s, action)

    def after_env_step(self, s, action):
        env = self.env
        n = env.E * env.N
        self.learner.store_transitions(self.prev_obs.reshape(n, -1), action.reshape(n, -1), env.reward.reshape(n, 1),
                                       env.dnn.reshape(n, -1), env.done.reshape(n))
        self.prev_obs = env.dnn
        self.learner.learn(s % self.learner.n_agents)
