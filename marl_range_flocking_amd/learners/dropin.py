"""Reference-API adapters over the batched learners, so the reference's own drivers (main.py,
learners/*/train_flock.py) run unchanged. The thin modules under learners/compat/ re-export these under the
reference's module paths (MADDPG, vdn.net / vdn.utils / vdn.train_flock,
maddpg.agents.ddpg.agent_simple_shared_critic, maddpg.models.DDPG.DDPG_network / .utils).

Checkpoints use the reference's file names and state_dict keys (net.py:84-94 ``{save_dir}/agent_number_{i}_
{actor,critic,target_actor,target_critic}_ddpg.pt``; replay ``.npy`` + ``dict_info.json``, memory_rnn.py:104-124;
VDN QNet keys ``agent_feature_{i}.0.weight`` ...), written and read with torch.save / torch.load(weights_only=True).
"""
import json
import os
import random
import time

import numpy as np
import torch

from ..vec_env import device_writes
from .maddpg import MADDPGLearner
from .shared_critic import SharedCriticLearner
from .vdn import BatchedQNet, VDNLearner


def _device(env=None):
    d = getattr(env, "device", None)
    if d is not None:
        return torch.device(d)
    if not torch.cuda.is_available():
        raise RuntimeError("the batched learners need a HIP device (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


# ----------------------------------------------------------------------------------------------------- MADDPG
class ReplayBufferMaddpg:
    """memory_rnn.py:8-139 / memory.py:8-125 surface over the learner's device ring."""

    def __init__(self, learner):
        self.L = learner
        self.batch_size, self.chunk_size = learner.B, learner.C
        self.min_size_buffer = learner.min_size_buffer
        self.buffer_capacity = learner.replay.capacity
        self.n_agents = learner.N
        self.n_games = 0

    @property
    def buffer_counter(self):
        return self.L.replay.counter

    def __len__(self):
        return self.buffer_counter

    def check_buffer_size(self):
        return self.L.check_buffer_size()

    def update_n_games(self):
        self.n_games += 1

    def add_record(self, actor_states, actor_next_states, actions, state, next_state, reward, done):
        self.L.add_record(actor_states, actor_next_states, actions, state, next_state, reward, done)

    def save(self, folder_path):
        os.makedirs(folder_path, exist_ok=True)
        b = {k: v.cpu().numpy() for k, v in self.L.replay.bufs.items()}
        np.save(folder_path + "/states.npy", b["state"])
        np.save(folder_path + "/rewards.npy", b["reward"][..., None])
        np.save(folder_path + "/next_states.npy", b["next_state"])
        np.save(folder_path + "/dones.npy", b["done"][..., None])
        for i in range(self.n_agents):
            np.save(folder_path + f"/states_actor_{i}.npy", b["actor_state"][:, i])
            np.save(folder_path + f"/next_states_actor_{i}.npy", b["actor_next_state"][:, i])
            np.save(folder_path + f"/actions_actor_{i}.npy", b["action"][:, i])
        with open(folder_path + "/dict_info.json", "w") as f:
            json.dump({"buffer_counter": self.buffer_counter, "n_games": self.n_games}, f)

    def load(self, folder_path):
        ld = lambda n: torch.from_numpy(np.load(folder_path + n, allow_pickle=False))  # noqa: E731
        bufs = self.L.replay.bufs
        bufs["state"].copy_(ld("/states.npy"))
        bufs["next_state"].copy_(ld("/next_states.npy"))
        bufs["reward"].copy_(ld("/rewards.npy")[..., 0])
        bufs["done"].copy_(ld("/dones.npy")[..., 0])
        for i in range(self.n_agents):
            bufs["actor_state"][:, i].copy_(ld(f"/states_actor_{i}.npy"))
            bufs["actor_next_state"][:, i].copy_(ld(f"/next_states_actor_{i}.npy"))
            bufs["action"][:, i].copy_(ld(f"/actions_actor_{i}.npy"))
        with open(folder_path + "/dict_info.json") as f:
            info = json.load(f)
        self.L.replay.counter = info["buffer_counter"]
        self.n_games = info["n_games"]


class SuperAgent:
    """MADDPG.SuperAgent (maddpg_official_rnn/MADDPG.py:13-150, recurrent=True; maddpg_official/MADDPG.py, False)."""

    recurrent = True

    def __init__(self, args, env, path_save="/tmp", path_load="/tmp"):
        self.path_save, self.path_load = path_save, path_load
        self.n_agents = env.num_particles
        k = env.observation_space[1][0].shape[0]
        rnn = self.recurrent
        self.learner = MADDPGLearner(
            self.n_agents, k, recurrent=rnn, n_actions=env.action_space[0].shape[0],
            hidden1=getattr(args, "hidden1", 400), hidden2=getattr(args, "hidden2", 300),
            batch_size=getattr(args, "batch_size", 128), chunk_size=10,
            buffer_capacity=getattr(args, "buffer_size", 1_000_000) if rnn else 1_000_000,
            min_size_buffer=getattr(args, "min_size_buffer", 8_000) if rnn else 8_000,
            ou_theta=args.ou_theta, ou_mu=args.ou_mu, ou_sigma=args.ou_sigma,
            ou_sigma_min=getattr(args, "ou_sigma_min", None), device=_device(env))
        self.save_dir = getattr(args, "save_dir", "tmp")
        self.replay_buffer = ReplayBufferMaddpg(self.learner)
        self.random_process = self.learner.random_process

    def init_hidden(self):
        return self.learner.init_hidden(1)

    def get_actions(self, actor_states, hidden_states=None, test=False):
        a, h = self.learner.get_actions(torch.as_tensor(actor_states).to(self.learner.device), hidden_states, test)
        return (a, h) if self.recurrent else a

    def reset_random_process(self):
        self.learner.reset_random_process()

    def update_random_process(self):
        self.learner.update_random_process()

    def train(self, *a, **k):
        self.learner.train()

    def _ckpt(self, i, net):
        return os.path.join(self.save_dir, f"agent_number_{i}_{net}_ddpg.pt")

    def save(self):
        os.makedirs(self.save_dir, exist_ok=True)
        for i in range(self.n_agents):  # one writer per file: the owner of a sharded network, one rank otherwise
            for net in ("actor", "critic"):
                for target in (False, True):
                    if self.learner.writes(net, i, target):
                        torch.save(self.learner.state_dict(net, i, target=target),
                                   self._ckpt(i, ("target_" if target else "") + net))
        # the replay ring is rank-local (each rank's envs): one file per rank
        self.replay_buffer.save(f"{self.path_save}/save_agent_{time.strftime('%Y%m%d%H%M')}{self.learner.rank_suffix()}")

    def load(self):
        sds = {}
        for i in range(self.n_agents):
            for net in ("actor", "critic", "target_actor", "target_critic"):
                if self.learner.owns(net.replace("target_", ""), i, net.startswith("target")):
                    sds[f"{net}{i}"] = torch.load(self._ckpt(i, net), weights_only=True)
        self.learner.load_reference_state(sds)

    def load_replay_buffer(self):
        """MADDPG.py:56-58: the replay saved by save() under path_load."""
        self.replay_buffer.load(self.path_load)

    def load_single_checkpoint(self, path):
        sd = torch.load(path, weights_only=True)
        self.learner.load_reference_state({f"actor{i}": sd for i in range(self.n_agents)})

    def load_scaled_checkpoint(self, ch_path, total=5):
        """MADDPG.py:67-76: every agent takes the actor of a random saved agent (randint is inclusive)."""
        self.learner.load_reference_state({
            f"actor{i}": torch.load(os.path.join(ch_path, f"agent_number_{random.randint(0, total)}_actor_ddpg.pt"),
                                    weights_only=True) for i in range(self.n_agents)})


class SuperAgentFF(SuperAgent):
    recurrent = False


# ------------------------------------------------------------------------------------------------------- VDN
class QNet:
    """vdn/net.py:11-61 surface over BatchedQNet (stacked per-agent networks)."""

    def __init__(self, observation_space, action_space, recurrent=False, device=None):
        self.num_agents = len(observation_space)
        self.recurrent = recurrent
        self.hx_size = 32
        self.impl = BatchedQNet(self.num_agents, observation_space[0].shape[0], action_space[0].n, recurrent,
                                device or _device())
        self.engine = None

    def cuda(self, *a, **k):
        return self

    def parameters(self):
        return self.impl.P.parameters()

    def __call__(self, obs, hidden):
        return self.impl(obs, hidden)

    forward = __call__

    def init_hidden(self, batch_size=1):
        return self.impl.init_hidden(batch_size)

    def sample_action(self, obs, hidden, epsilon):
        return self.impl.sample_action(torch.as_tensor(obs).to(self.impl.device), hidden, epsilon)

    def state_dict(self):
        return self.impl.state_dict()

    def load_state_dict(self, sd):
        self.impl.load_reference_state_dict(sd)

    def load_params(self, checkpoint, agent_i=0):
        params = torch.load(checkpoint, weights_only=True)
        keys = [k for k in params if f"_{agent_i}." in k]
        self.load_state_dict({k.replace(f"_{agent_i}.", f"_{a}."): params[k] for a in range(self.num_agents)
                              for k in keys})


class ReplayBufferVDN:
    """vdn/utils.py:7-69 surface: a device ring of whole-swarm transitions (deque semantics)."""

    def __init__(self, buffer_limit, chunk_size, n_agents, input_shape, batch_size=32, device=None):
        from .core import ReplayRing

        self.chunk_size, self.batch_size, self.n_agents = chunk_size, batch_size, n_agents
        self.ring = ReplayRing(buffer_limit, {"s": (n_agents, *input_shape), "a": (n_agents,), "r": (n_agents,),
                                              "s_prime": (n_agents, *input_shape), "done": ()}, device or _device())

    def put(self, transition):
        s, a, r, s_prime, done = transition
        f = lambda t: torch.as_tensor(t).to(self.ring.device).float()  # noqa: E731
        self.ring.store({"s": f(s)[None], "a": f(a).reshape(1, -1), "r": f(r).reshape(1, -1),
                         "s_prime": f(s_prime)[None], "done": f(done).reshape(1)})

    def size(self):
        return len(self.ring)


def vdn_train(q, q_target, memory, optimizer, gamma, batch_size, update_iter=10, chunk_size=10, grad_clip_norm=5):
    """vdn/train_flock.py:16-43: update_iter iterations on all agents at once (one graph each). The torch optimizer
    the driver built is only read for its learning rate; the Adam state lives in the learner."""
    eng = q.engine
    if eng is None:
        lr = optimizer.param_groups[0]["lr"]
        eng = VDNLearner.__new__(VDNLearner)
        VDNLearner.attach(eng, q.impl, q_target.impl, memory.ring, lr=lr, gamma=gamma, batch_size=batch_size,
                          chunk_size=chunk_size, update_iter=update_iter, grad_clip_norm=grad_clip_norm)
        q.engine = eng
    eng.train()


# ---------------------------------------------------------------------------------------------- shared critic
class OUActionNoiseGPU:
    """utils.py:6-26: x = x + theta (mu - x) dt + sigma sqrt(dt) N(0,1), shared by the agents that call it."""

    def __init__(self, mu, sigma=0.15, theta=0.2, dt=1e-2, x0=None):
        self.mu = torch.as_tensor(mu).to(_device()).float()
        self.sigma, self.theta, self.dt, self.x0 = sigma, theta, dt, x0
        self.reset()

    def __call__(self):
        x = self.x_prev + self.theta * (self.mu - self.x_prev) * self.dt + self.sigma * np.sqrt(self.dt) * \
            torch.randn(self.mu.shape, device=self.mu.device)
        self.x_prev = x
        return x

    def reset(self):
        self.x_prev = self.x0 if self.x0 is not None else torch.zeros_like(self.mu)


class ReplayBuffer:
    """maddpg_shared_critic/utils.py:28-76 surface. The device ring is allocated here (max_size rows, as the reference
    allocates its arrays in the constructor, utils.py:29-45) and adopted by the shared-critic learner, so rows stored
    before the first choose_action land in HBM at once and mem_cntr is a plain counter."""

    def __init__(self, max_size, input_shape, n_actions, n_agents):
        self.mem_size, self.input_shape, self.n_actions, self.n_agents = int(max_size), input_shape, n_actions, \
            n_agents
        self.ring = SharedCriticLearner.make_replay(self.mem_size, input_shape[0], n_actions, _device())

    @property
    def mem_cntr(self):
        return self.ring.counter

    def store_transitions(self, state, action, reward, state_, done):
        SharedCriticLearner.store_rows(self.ring, state, action, reward, state_, done)

    store_single_transition = store_transitions


class CriticNetwork:
    """ddpg_network.py:11-70 surface: the shared critic; the Agents built on it form ONE batched learner. Checkpoint
    files as the reference names them (ddpg_network.py:29-34): ``{chkpt_dir}/{name}_ddpg.pt`` and
    ``{chkpt_best_dir}/{name}_ddpg.pt``, both directories created here."""

    def __init__(self, beta, input_dims, fc1_dims, fc2_dims, n_actions, name, chkpt_dir=r"tmp\ddpg",
                 chkpt_best_dir=r"tmp\ddpg_best"):
        self.beta, self.input_dims, self.fc1_dims, self.fc2_dims = beta, input_dims, fc1_dims, fc2_dims
        self.n_actions, self.name, self.chkpt_dir, self.chkpt_best_dir = n_actions, name, chkpt_dir, chkpt_best_dir
        for d in (chkpt_dir, chkpt_best_dir):
            os.makedirs(d, exist_ok=True)
        self.checkpoint_file = os.path.join(chkpt_dir, name + "_ddpg.pt")
        self.checkpoint_best_file = os.path.join(chkpt_best_dir, name + "_ddpg.pt")
        self.agents = []
        self.backend = None
        self._act_cache = None  # (observation tensor, key, all agents' mu) of the last choose_action

    def _build(self):
        if self.backend is None:
            a0 = self.agents[0]
            rb = a0.memory
            self.backend = SharedCriticLearner(
                len(self.agents), self.input_dims[0], n_actions=self.n_actions, fc1=self.fc1_dims, fc2=self.fc2_dims,
                alpha=a0.alpha, beta=self.beta, gamma=a0.gamma, tau=a0.tau, batch_size=a0.batch_size,
                update_rate=a0.update_rate, buffer_size=rb.mem_size, device=_device(), replay=rb.ring)
        return self.backend

    def actions(self, observation):
        """Every agent's mu for one observation [N, in], computed once per observation: the reference driver calls
        choose_action agent after agent with the same tensor (train_flock.py:114-115), so agents 1..N-1 slice the
        batched result. The cache holds the observation tensor itself (its address cannot be reused while cached)
        and keys on its storage, shape, strides and version counter (bumped by any in-place write) and on the count of
        VecFlockEnv steps / resets (kernel writes into an env's observation buffers bump no version counter);
        learn() and load_models() drop it."""
        t = observation if torch.is_tensor(observation) else None
        key = None if t is None else (t.data_ptr(), tuple(t.shape), t.stride(), t.dtype, t.device, t._version,
                                      device_writes())
        c = self._act_cache
        if key is not None and c is not None and c[1] == key:
            return c[2]
        L = self._build()
        obs = torch.as_tensor(observation).to(L.device).float()
        mu = L.choose_action(obs.reshape(L.n_agents, -1)[None], noise=False)[0]
        self._act_cache = (t, key, mu) if key is not None else None
        return mu

    def drop_action_cache(self):
        self._act_cache = None


class Agent:
    """agent_simple_shared_critic.py:14-220 surface: agent ``index`` of the batched shared-critic learner."""

    def __init__(self, shared_critic, alpha, beta, input_dims, tau, checkpoint_dir, checkpoint_best, index,
                 replay_buffer, noise, recurrent=False, gamma=0.99, n_actions=2, layer1_size=32, layer2_size=32,
                 batch_size=64, update_rate=3):
        if recurrent:
            raise NotImplementedError("the recurrent shared-critic variant imports modules absent from the reference")
        os.makedirs(checkpoint_dir, exist_ok=True)  # agent_simple_shared_critic.py:46-47
        self.critic = self.target_critic = shared_critic
        self.alpha, self.gamma, self.tau, self.batch_size, self.update_rate = alpha, gamma, tau, batch_size, update_rate
        self.index, self.memory, self.noise = index, replay_buffer, noise
        self.checkpoint_dir, self.checkpoint_best = checkpoint_dir, checkpoint_best
        shared_critic.agents.append(self)

    def choose_action(self, observation):
        """agent_simple_shared_critic.py:92-107: mu_i(obs[i]) + noise (the batched mu is shared by all agents)."""
        return self.critic.actions(observation)[self.index] + self.noise()

    def remember(self, state, action, reward, new_state, done):
        self.memory.store_transitions(state, action, reward, new_state, done)

    def learn(self):
        self.critic.drop_action_cache()
        return self.critic._build().learn(self.index)

    def _files(self, best):
        """Actor / TargetActor in this agent's checkpoint (or best) directory, the critic in the CriticNetwork's own
        directories (ddpg_network.py:33-34, :103-104; train_flock.py:47-48, :65-66)."""
        d = self.checkpoint_best if best else self.checkpoint_dir
        crit = self.critic.checkpoint_best_file if best else self.critic.checkpoint_file
        return [os.path.join(d, f"{n}_ddpg.pt") for n in ("Actor", "TargetActor")] + [crit]

    def save_models(self, best=False):
        """train_flock.py:143 (every 300 s) / :151 (save_models_best); agent_simple.py:200-210 file naming."""
        L = self.critic._build()
        files = self._files(best)
        for f in files:
            os.makedirs(os.path.dirname(f) or ".", exist_ok=True)
        for f, sd in zip(files, (L.actor_state_dict(self.index), L.actor_state_dict(self.index, target=True),
                                 L.critic_state_dict())):
            torch.save(sd, f)

    def save_models_best(self):
        self.save_models(best=True)

    def load_models(self, silent=False, best=False):
        """agent_simple.py:212-216: this agent's actor + target actor, and the shared critic."""
        L = self.critic._build()
        actor, target, critic = (torch.load(f, weights_only=True) for f in self._files(best))
        L.load_reference_state(critic, {self.index: actor}, {self.index: target})
        self.critic.drop_action_cache()
