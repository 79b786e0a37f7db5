"""Golden vectors for the recurrent VDN learner: the REFERENCE train(q, q_target, memory, ...)
(learners/vdn/train_flock.py:16-43, QNet learners/vdn/net.py:11-61, ReplayBufferVDN learners/vdn/utils.py:7-69)
run on CPU with injected replay contents and sampled chunk starts (np.random.randint patched). Also records QNet
forward outputs on a fixed batch. Writes tests/golden/learn_vdn.npz.

``--prod``: 64 agents at the reference driver's settings (train_flock.py:16-43, :60-80: B 32, chunk 10,
update_iter 10), written compactly (tests/golden/compact.py) to learn_vdn_prod.npz.
"""
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import compact  # noqa: E402
import refshim  # noqa: E402

PROD = "--prod" in sys.argv
if PROD:
    N_AGENTS, K, N_ACT, B, CHUNK, ITERS, T = 64, 4, 4, 32, 10, 10, 60
else:
    N_AGENTS, K, N_ACT, B, CHUNK, ITERS, T = 3, 4, 4, 6, 10, 3, 40
SAMPLES = 128  # sampled positions per tensor in the compact fixture (64 agents x 10 tensors)


def main():
    if not refshim.available():
        print("reference not present")
        return
    import torch

    refshim.install()
    # train_flock.py imports SummaryWriter and the env at module level: stub what the update does not use
    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = object
    sys.modules["torch.utils.tensorboard"] = tb
    sys.modules["vdn"] = types.ModuleType("vdn")
    net = refshim.load("learners/vdn/net.py", "vdn.net")
    utils = refshim.load("learners/vdn/utils.py", "vdn.utils")
    sys.modules["gym_flock_uw_discrete"] = types.ModuleType("gym_flock_uw_discrete")
    sys.modules["gym_flock_uw_discrete"].MultiAgentEnv = object
    trainmod = refshim.load("learners/vdn/train_flock.py", "ref_vdn_train_flock")
    from gym import spaces  # the stub

    torch.manual_seed(0)
    rng = np.random.default_rng(0)
    obs_space = [spaces.Box(0, 7, (K,)) for _ in range(N_AGENTS)]
    act_space = [spaces.Discrete(N_ACT) for _ in range(N_AGENTS)]
    q = net.QNet(obs_space, act_space, recurrent=True)
    q_target = net.QNet(obs_space, act_space, recurrent=True)
    q_target.load_state_dict(q.state_dict())
    specs = []
    with torch.no_grad():
        if PROD:  # seeded initial parameters (compact.init_value; the target differs from q)
            for tag, m in (("q", q), ("target_q", q_target)):
                for k_, v in m.state_dict().items():
                    v.copy_(torch.from_numpy(compact.init_value(tag, k_, v.shape)))
                    specs.append([tag, k_, list(v.shape)])
        else:  # perturb the target so q and q_target differ (as between target syncs)
            for p in q_target.parameters():
                p.add_(0.01 * torch.randn_like(p))
    sd = lambda m: {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}  # noqa: E731
    init_q, init_t = sd(q), sd(q_target)
    memory = utils.ReplayBufferVDN(50000, chunk_size=CHUNK, n_agents=N_AGENTS, input_shape=[K], batch_size=B)
    s = rng.uniform(0, 7, (T, N_AGENTS, K)).astype(np.float32)
    s2 = rng.uniform(0, 7, (T, N_AGENTS, K)).astype(np.float32)
    a = rng.integers(0, N_ACT, (T, N_AGENTS)).astype(np.float32)
    r = rng.choice([-8.9, 0.1, -9.0, 0.0], size=(T, N_AGENTS, 1)).astype(np.float32)
    d = (rng.uniform(size=T) < 0.15).astype(np.int64)
    for t in range(T):
        memory.put((torch.tensor(s[t]), torch.tensor(a[t]), torch.tensor(r[t]), torch.tensor(s2[t]), [int(d[t])]))
    starts = rng.integers(0, T - CHUNK, (ITERS, B)).astype(np.int64)
    calls = {"i": 0}
    orig = np.random.randint

    def fake_randint(lo, hi, size):
        assert lo == 0 and hi == T - CHUNK and size == B
        out = starts[calls["i"]]
        calls["i"] += 1
        return out

    optimizer = torch.optim.Adam(q.parameters(), lr=1e-3)
    rec = {"norms": [], "grads": []}
    orig_clip = torch.nn.utils.clip_grad_norm_

    def clip(params, max_norm, norm_type=2):
        params = list(params)
        rec["grads"].append({n: p.grad.detach().numpy().copy() for n, p in q.named_parameters()})
        n = orig_clip(params, max_norm, norm_type=norm_type)
        rec["norms"].append(float(n))
        return n

    np.random.randint = fake_randint
    torch.nn.utils.clip_grad_norm_ = clip
    try:
        trainmod.train(q, q_target, memory, optimizer, 0.99, B, update_iter=ITERS, chunk_size=CHUNK,
                       grad_clip_norm=5)
    finally:
        np.random.randint = orig
        torch.nn.utils.clip_grad_norm_ = orig_clip
    final_q = sd(q)
    # forward check batch
    xo = rng.uniform(0, 7, (5, N_AGENTS, K)).astype(np.float32)
    xh = rng.standard_normal((5, N_AGENTS, 32)).astype(np.float32)
    with torch.no_grad():
        qo, ho = q(torch.tensor(xo), torch.tensor(xh))
    if PROD:
        flat = compact.encode("q", final_q, {k_: [g[k_] for g in rec["grads"]] for k_ in final_q}, s=SAMPLES)
        meta = dict(n_agents=N_AGENTS, k=K, n_actions=N_ACT, batch=B, chunk=CHUNK, update_iter=ITERS, T=T, lr=1e-3,
                    gamma=0.99, grad_clip_norm=5, recurrent=True, torch=torch.__version__, specs=specs,
                    samples=SAMPLES, source="learners/vdn/train_flock.py:16-43")
        np.savez_compressed(os.path.join(HERE, "learn_vdn_prod.npz"), meta=np.array(json.dumps(meta)), s=s,
                            s_prime=s2, a=a, r=r, done=d, starts=starts, norms=np.array(rec["norms"]), fwd_obs=xo,
                            fwd_hidden=xh, fwd_q=qo.numpy(), fwd_h=ho.numpy(), **flat)
        print("wrote learn_vdn_prod.npz norms", rec["norms"])
        return
    flat = {}
    for tag, dct in (("init_q", init_q), ("init_target", init_t), ("final_q", final_q)):
        for k_, v in dct.items():
            flat[f"{tag}/{k_}"] = v
    for it, g in enumerate(rec["grads"]):
        for k_, v in g.items():
            flat[f"grad{it}/{k_}"] = v
    meta = dict(n_agents=N_AGENTS, k=K, n_actions=N_ACT, batch=B, chunk=CHUNK, update_iter=ITERS, T=T, lr=1e-3,
                gamma=0.99, grad_clip_norm=5, recurrent=True, torch=torch.__version__,
                source="learners/vdn/train_flock.py:16-43")
    np.savez_compressed(os.path.join(HERE, "learn_vdn.npz"), meta=np.array(json.dumps(meta)), s=s, s_prime=s2,
                        a=a, r=r, done=d, starts=starts, norms=np.array(rec["norms"]), fwd_obs=xo, fwd_hidden=xh,
                        fwd_q=qo.numpy(), fwd_h=ho.numpy(), **flat)
    print("wrote learn_vdn.npz norms", rec["norms"])


if __name__ == "__main__":
    main()
