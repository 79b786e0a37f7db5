"""Golden vectors for the MADDPG learners: the REFERENCE SuperAgent.train() run on CPU with injected replay rows and
sampled chunk starts (np.random.choice patched).
  rnn  learners/maddpg_official_rnn/MADDPG.py:78-150 (GRU actor/critic net.py:14-146, ReplayBufferMaddpg
       memory_rnn.py:8-99, k must be 4: MADDPG.py:84)
  ff   learners/maddpg_official/MADDPG.py:67-108 (net.py:14-115, memory.py:8-125, k must be 9: MADDPG.py:73)
Small hidden sizes (hidden1=32, hidden2=24) keep fixtures small; the code path is the reference's own.
Writes tests/golden/learn_maddpg_rnn.npz and learn_maddpg_ff.npz. Run each flavour in its own process
(``python gen_golden_learn_maddpg.py rnn|ff``): both directories define modules named agent/net/utils/MADDPG.

``rnn-prod``: the reference's production shape (net.py:14-146 defaults hidden 400/300; MADDPG.py:78 B 128,
chunk 10) with 16 agents, written compactly (tests/golden/compact.py) to learn_maddpg_rnn_prod.npz.
"""
import json
import os
import subprocess
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import compact  # noqa: E402
import refshim  # noqa: E402

SMALL = dict(N=3, B=8, CAP=64, T=40, H1=32, H2=24)
PROD = dict(N=16, B=128, CAP=256, T=150, H1=400, H2=300)
SAMPLES = 256  # sampled positions per tensor in the compact fixture (64 networks)


def run(flavour):
    import torch

    prod = flavour.endswith("-prod")
    flavour = flavour.replace("-prod", "")
    N, B, CAP, T, H1, H2 = (PROD if prod else SMALL).values()

    refshim.install()
    d = "learners/maddpg_official_rnn" if flavour == "rnn" else "learners/maddpg_official"
    K = 4 if flavour == "rnn" else 9
    C = 10 if flavour == "rnn" else 1
    utils = refshim.load(f"{d}/utils.py", "utils")
    net = refshim.load(f"{d}/net.py", "net")
    for cls in ("Actor", "Critic"):  # small hidden layers for the fixture (defaults hidden1=400, hidden2=300)
        f = getattr(net, cls).__init__
        f.__defaults__ = (H1, H2) + f.__defaults__[2:]
    refshim.load(f"{d}/agent.py", "agent")
    memmod = "memory_rnn" if flavour == "rnn" else "memory"
    mem = refshim.load(f"{d}/{memmod}.py", memmod)
    if flavour == "ff":  # SuperAgent builds ReplayBufferMaddpg(env) with defaults (1e6, 128, 8000): shrink them
        mem.ReplayBufferMaddpg.__init__.__defaults__ = (CAP, B, B)
    mad = refshim.load(f"{d}/MADDPG.py", f"ref_maddpg_{flavour}")
    torch.autograd.set_detect_anomaly(False)
    from gym import spaces

    env = types.SimpleNamespace(num_particles=N,
                                observation_space=[spaces.Box(0, 50, (N, K)), [spaces.Box(0, 50, (K,))] * N],
                                action_space=[spaces.Box(-1.5, 1.5, (2,))] * N)
    args = types.SimpleNamespace(buffer_size=CAP, batch_size=B, min_size_buffer=B, ou_theta=0.15, ou_mu=0.0,
                                 ou_sigma=0.2, ou_sigma_min=0.001, save_dir="ckpt", max_steps=250)
    os.makedirs("ckpt", exist_ok=True)
    torch.manual_seed(1)
    rng = np.random.default_rng(1)
    sa = mad.SuperAgent(args, env)
    sd = lambda m: {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}  # noqa: E731
    nets = ("actor", "critic", "target_actor", "target_critic")
    specs = []
    with torch.no_grad():
        if prod:  # seeded initial parameters (compact.init_value; targets differ from the online nets)
            for i, ag in enumerate(sa.agents):
                for nm in nets:
                    for k, v in getattr(ag, nm).state_dict().items():
                        v.copy_(torch.from_numpy(compact.init_value(f"{nm}{i}", k, v.shape)))
                        specs.append([f"{nm}{i}", k, list(v.shape)])
        else:  # make target nets differ from the online nets (as after training)
            for ag in sa.agents:
                for p in list(ag.target_critic.parameters()) + list(ag.target_actor.parameters()):
                    p.add_(0.01 * torch.randn_like(p))
    init = {f"{nm}{i}": sd(getattr(ag, nm)) for i, ag in enumerate(sa.agents) for nm in nets}
    obs = rng.uniform(0, 14, (T + 1, N, K)).astype(np.float32)
    act = rng.uniform(-1, 1.5, (T, N, 2)).astype(np.float32)
    rew = rng.choice([-5.0, 0.01], size=(T, N, 1)).astype(np.float32)
    done = (rng.uniform(size=(T, N)) < 0.1).astype(np.float32)
    for t in range(T):
        sa.replay_buffer.add_record(torch.tensor(obs[t]), torch.tensor(obs[t + 1]), torch.tensor(act[t]),
                                    torch.tensor(obs[t]), torch.tensor(obs[t + 1]), torch.tensor(rew[t]),
                                    torch.tensor(done[t]))
    rng_hi = T - C if flavour == "rnn" else T
    starts = rng.choice(rng_hi, B, replace=False).astype(np.int64)
    orig_choice = np.random.choice

    def fake_choice(hi, size, replace=True):
        assert hi == rng_hi and size == B and replace is False
        return starts

    grads = {}
    for i, ag in enumerate(sa.agents):
        opt = ag.critic_optimizer
        orig_step = opt.step

        def step(*a, _i=i, _ag=ag, _o=orig_step):
            for k, p in _ag.critic.named_parameters():
                grads[f"critic{_i}/{k}"] = p.grad.detach().numpy().copy()
            for k, p in _ag.actor.named_parameters():
                assert p.grad is None or float(p.grad.abs().max()) == 0.0
            return _o(*a)

        opt.step = step
    np.random.choice = fake_choice
    try:
        if flavour == "rnn":
            sa.train(batch_size=B, chunk_size=C)
        else:
            sa.train()
    finally:
        np.random.choice = orig_choice
    final = {f"{nm}{i}": sd(getattr(ag, nm)) for i, ag in enumerate(sa.agents) for nm in nets}
    # an acting batch: get_actions without noise (test=True)
    hidden = sa.init_hidden() if flavour == "rnn" else None
    with torch.no_grad():
        if flavour == "rnn":
            acts, hid = sa.get_actions(torch.tensor(obs[0]), hidden, test=True)
            hid = torch.stack([h.reshape(-1) for h in hid])
        else:
            acts = sa.get_actions(torch.tensor(obs[0]), test=True)
            hid = torch.zeros(1)
    meta = dict(flavour=flavour, n_agents=N, k=K, batch=B, chunk=C, capacity=CAP, T=T, hidden1=H1, hidden2=H2,
                hidden_rnn=32, lr=3e-3, gamma=0.99, tau=0.001, torch=torch.__version__, source=f"{d}/MADDPG.py")
    if prod:
        flat = {}
        for i in range(N):
            g = {k: [grads[f"critic{i}/{k}"]] for k in final[f"critic{i}"]}
            flat.update(compact.encode(f"critic{i}", final[f"critic{i}"], g, s=SAMPLES))
            flat.update(compact.encode(f"target_critic{i}", final[f"target_critic{i}"], g, s=SAMPLES))
            flat.update(compact.encode(f"actor{i}", final[f"actor{i}"], s=SAMPLES))  # frozen (Q6): bitwise
            flat.update(compact.encode(f"target_actor{i}", final[f"target_actor{i}"], s=SAMPLES))
        meta["specs"], meta["samples"] = specs, SAMPLES
        name = f"learn_maddpg_{flavour}_prod.npz"
        np.savez_compressed(os.path.join(HERE, name), meta=np.array(json.dumps(meta)), obs=obs, action=act,
                            reward=rew, done=done, starts=starts, act_out=acts.numpy(), act_hidden=hid.numpy(),
                            **flat)
        print("wrote", name)
        return
    flat = {}
    for tag, dd in (("init", init), ("final", final)):
        for nm, params in dd.items():
            for k, v in params.items():
                flat[f"{tag}/{nm}/{k}"] = v
    for k, v in grads.items():
        flat[f"grad/{k}"] = v
    np.savez_compressed(os.path.join(HERE, f"learn_maddpg_{flavour}.npz"), meta=np.array(json.dumps(meta)),
                        obs=obs, action=act, reward=rew, done=done, starts=starts, act_out=acts.numpy(),
                        act_hidden=hid.numpy(), **flat)
    print("wrote", f"learn_maddpg_{flavour}.npz")


if __name__ == "__main__":
    if not refshim.available():
        print("reference not present")
    elif len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        for f in ("rnn", "ff"):
            subprocess.check_call([sys.executable, os.path.abspath(__file__), f])
