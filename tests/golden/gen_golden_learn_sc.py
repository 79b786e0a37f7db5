"""Golden vectors for the shared-critic learner: the REFERENCE Agent.learn()
(learners/maddpg_shared_critic/agent_simple_shared_critic.py:115-155) run on CPU with injected replay contents and
sampled indices (np.random.choice patched, utils.py:65-76). Small layer sizes (fc1=32, fc2=24) keep the fixture
small; the code path is the reference's own. Writes tests/golden/learn_shared_critic.npz.

``--prod``: the reference's production shape (train_flock.py:15-27, :64: fc1 400, fc2 300, B 256) with 8 agents,
written compactly (tests/golden/compact.py: seeded initial parameters, sampled final parameters, well-conditioned
bit masks instead of gradients) to tests/golden/learn_shared_critic_prod.npz.

Recorded: initial state_dicts (critic, actors, target actors), the replay rows, the sampled indices, per-learn()
losses and the gradients each optimizer step consumed, and the final state_dicts.
"""
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refshim  # noqa: E402

import compact  # noqa: E402

PROD = "--prod" in sys.argv
if PROD:
    N_AGENTS, K, FC1, FC2, B, CAP, T = 8, 4, 400, 300, 256, 4096, 64
    CALLS = [0, 1, 2, 3, 0, 1]  # counts 0,0,0,0,1,1 → soft updates on the first four
else:
    N_AGENTS, K, FC1, FC2, B, CAP, T = 3, 4, 32, 24, 16, 64, 20
    CALLS = [0, 1, 2, 0, 1]  # learn() order over agents: counts 0,0,0,1,1 → soft updates on the first three


def main():
    if not refshim.available():
        print("reference not present")
        return
    import torch

    refshim.install()
    torch.nn.Module.to = lambda self, *a, **k: self  # ddpg_network.py:274-276 picks "cuda:1" without a GPU
    pkg = {}
    for name in ("maddpg", "maddpg.models", "maddpg.models.DDPG", "maddpg.agents", "maddpg.agents.ddpg"):
        pkg[name] = types.ModuleType(name)
        sys.modules[name] = pkg[name]
    utils = refshim.load("learners/maddpg_shared_critic/utils.py", "maddpg.models.DDPG.utils")
    net = refshim.load("learners/maddpg_shared_critic/ddpg_network.py", "maddpg.models.DDPG.DDPG_network")
    agent_mod = refshim.load("learners/maddpg_shared_critic/agent_simple_shared_critic.py",
                             "maddpg.agents.ddpg.agent_simple_shared_critic")
    torch.manual_seed(0)
    rng = np.random.default_rng(0)
    buf = utils.ReplayBuffer(max_size=CAP, input_shape=[K], n_actions=2, n_agents=N_AGENTS)
    noise = utils.OUActionNoiseGPU(mu=torch.zeros(2))
    critic = net.CriticNetwork(3e-4, [K], FC1, FC2, n_actions=2, name="Critic", chkpt_dir="c", chkpt_best_dir="b")
    agents = [agent_mod.Agent(shared_critic=critic, alpha=3e-4, beta=3e-4, input_dims=[K], tau=0.001,
                              checkpoint_dir=f"a{i}", checkpoint_best="b", index=i, replay_buffer=buf, noise=noise,
                              layer1_size=FC1, layer2_size=FC2, batch_size=B) for i in range(N_AGENTS)]
    sd = lambda m: {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}  # noqa: E731
    nets = {"critic": critic}
    for i, a in enumerate(agents):
        nets[f"actor{i}"], nets[f"target_actor{i}"] = a.actor, a.target_actor
    specs = []
    if PROD:  # seeded initial parameters (compact.init_value), written into the reference's own modules
        with torch.no_grad():
            for tag, m in nets.items():
                for k, v in m.state_dict().items():
                    v.copy_(torch.from_numpy(compact.init_value(tag, k, v.shape)))
                    specs.append([tag, k, list(v.shape)])
    init = {"critic": sd(critic)}
    for i, a in enumerate(agents):
        init[f"actor{i}"] = sd(a.actor)
        init[f"target_actor{i}"] = sd(a.target_actor)
    # replay contents: T store_transitions calls of N_AGENTS rows (utils.py:47-54)
    st = rng.uniform(0, 14, (T, N_AGENTS, K)).astype(np.float32)
    st2 = rng.uniform(0, 14, (T, N_AGENTS, K)).astype(np.float32)
    act = rng.uniform(-1, 1, (T, N_AGENTS, 2)).astype(np.float32)
    rew = rng.choice([-5.0, 0.01], size=(T, N_AGENTS, 1)).astype(np.float32)
    done = rng.integers(0, 2, (T, N_AGENTS)).astype(np.int64)
    for t in range(T):
        buf.store_transitions(torch.tensor(st[t]), torch.tensor(act[t]), torch.tensor(rew[t]), torch.tensor(st2[t]),
                              torch.tensor(done[t]))
    idx = rng.integers(0, T * N_AGENTS, (len(CALLS), B)).astype(np.int64)
    calls = {"i": 0}
    orig_choice = np.random.choice

    def fake_choice(maxm, size):
        assert maxm == T * N_AGENTS and size == B
        out = idx[calls["i"]]
        calls["i"] += 1
        return out

    grads = {}

    def snap(tag, module):
        return {f"{tag}.{k}": (p.grad.detach().numpy().copy() if p.grad is not None else np.zeros(p.shape, np.float32))
                for k, p in module.named_parameters()}

    losses = []
    np.random.choice = fake_choice
    try:
        for c, i in enumerate(CALLS):
            a = agents[i]
            copt, aopt = critic.optimizer.step, a.actor.optimizer.step

            def cstep(*x, _c=c):
                grads.update({f"call{_c}.{k}": v for k, v in snap("critic", critic).items()})
                return copt(*x)

            def astep(*x, _c=c, _a=a):
                grads.update({f"call{_c}.{k}": v for k, v in snap("actor", _a.actor).items()})
                return aopt(*x)

            critic.optimizer.step, a.actor.optimizer.step = cstep, astep
            al, cl, ok = a.learn()
            critic.optimizer.step, a.actor.optimizer.step = copt, aopt
            assert ok
            losses.append([float(al), float(cl)])
    finally:
        np.random.choice = orig_choice
    final = {"critic": sd(critic)}
    for i, a in enumerate(agents):
        final[f"actor{i}"] = sd(a.actor)
        final[f"target_actor{i}"] = sd(a.target_actor)
    if PROD:
        flat = {}
        for tag in nets:
            kind = "critic" if tag == "critic" else "actor"
            agent = None if tag == "critic" else int(tag[len(tag.rstrip("0123456789")):])
            calls = [c for c, a in enumerate(CALLS) if agent is None or a == agent]
            g = {k: [grads[f"call{c}.{kind}.{k}"] for c in calls] for k in final[tag]}
            flat.update(compact.encode(tag, final[tag], g))
        meta = dict(n_agents=N_AGENTS, k=K, fc1=FC1, fc2=FC2, batch=B, capacity=CAP, calls=CALLS, gamma=0.99,
                    tau=0.001, alpha=3e-4, beta=3e-4, update_rate=3, torch=torch.__version__, specs=specs,
                    source="learners/maddpg_shared_critic/agent_simple_shared_critic.py:115-185")
        np.savez_compressed(os.path.join(HERE, "learn_shared_critic_prod.npz"), meta=np.array(json.dumps(meta)),
                            state=st, next_state=st2, action=act, reward=rew, done=done, idx=idx,
                            losses=np.array(losses, np.float64), **flat)
        print("wrote learn_shared_critic_prod.npz", losses)
        return
    flat = {}
    for tag, d in (("init", init), ("final", final)):
        for net_name, params in d.items():
            for k, v in params.items():
                flat[f"{tag}/{net_name}/{k}"] = v
    for k, v in grads.items():
        flat[f"grad/{k}"] = v
    meta = dict(n_agents=N_AGENTS, k=K, fc1=FC1, fc2=FC2, batch=B, capacity=CAP, calls=CALLS, gamma=0.99, tau=0.001,
                alpha=3e-4, beta=3e-4, update_rate=3, torch=torch.__version__,
                source="learners/maddpg_shared_critic/agent_simple_shared_critic.py:115-185")
    np.savez_compressed(os.path.join(HERE, "learn_shared_critic.npz"), meta=np.array(json.dumps(meta)),
                        state=st, next_state=st2, action=act, reward=rew, done=done, idx=idx,
                        losses=np.array(losses, np.float64), **flat)
    print("wrote learn_shared_critic.npz", losses)


if __name__ == "__main__":
    main()
