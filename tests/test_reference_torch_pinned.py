"""Pin the plain-PyTorch restatements (tests/reference_torch.py) against the REFERENCE's own production-shape updates
(CPU; no GPU). The config-4/5-shape GPU tests (tests/test_gpu_learners_scale.py) compare the HIP learners with these
restatements at 512 / 1024 agents, too large for a reference fixture; this file closes that chain:

  HIP (config shape) == restatement (config shape),  restatement (prod shape) == reference (prod shape, here).

  VDN          learn_vdn_prod.npz: 64 agents, B 32, chunk 10, update_iter 10 (learners/vdn/train_flock.py:16-43).
               Each iteration's pre-clip gradient norm (the fixture records every one; clip_grad_norm_ at :42) within
               rtol 1e-4, then clip + torch.optim.Adam (lr 1e-3) exactly as :40-43, and after all 10 iterations the
               final QNet parameters at the fixture's sampled positions (tests/golden/compact.py: rtol 1e-4 where
               every consumed gradient is well-conditioned, the Adam step bound elsewhere).
  RNN-MADDPG   learn_maddpg_rnn_prod.npz: 16 agents, hidden 400/300, B 128, chunk 10
               (learners/maddpg_official_rnn/MADDPG.py:78-150): critics after one Adam step (lr 3e-3) and target
               critics after the soft update (net.py:74-78) at sampled positions (same rule), the frozen actors (Q6)
               and their target soft update bitwise.

The restatements take stacked [A, out, in] parameters; the reference keys (learners/vdn/net.py:19-25,
learners/maddpg_official_rnn/net.py:14-146) are mapped here, independently of the package.
"""
import json
import os

import numpy as np
import torch

import reference_torch as R
from golden import compact

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

VDN_LAYERS = {"feat1": "agent_feature_{i}.0", "feat2": "agent_feature_{i}.2", "gru": "agent_gru_{i}",
              "q": "agent_q_{i}"}
VDN_PARAMS = {"feat1": ("weight", "bias"), "feat2": ("weight", "bias"), "q": ("weight", "bias"),
              "gru": ("weight_ih", "weight_hh", "bias_ih", "bias_hh")}


def _vdn_stack(per_key, A):
    """{reference key: array} of A agents -> {"feat1.weight": [A, out, in], ...} (float32 tensors)."""
    out = {}
    for layer, kinds in VDN_PARAMS.items():
        for kind in kinds:
            out[f"{layer}.{kind}"] = torch.from_numpy(
                np.stack([per_key[f"{VDN_LAYERS[layer].format(i=i)}.{kind}"] for i in range(A)]))
    return out


def test_vdn_restatement_matches_reference_prod():
    z = np.load(os.path.join(GOLD, "learn_vdn_prod.npz"))
    m = json.loads(str(z["meta"]))
    A, C, iters, lr, gamma = m["n_agents"], m["chunk"], m["update_iter"], m["lr"], m["gamma"]
    init = compact.rebuild(m["specs"])
    P = {n: v.clone().requires_grad_(True) for n, v in _vdn_stack(init["q"], A).items()}
    T = _vdn_stack(init["target_q"], A)
    names = list(P)
    opt = torch.optim.Adam([P[n] for n in names], lr=lr, foreach=False)
    s, s2 = torch.from_numpy(z["s"]), torch.from_numpy(z["s_prime"])
    a, r = torch.from_numpy(z["a"]), torch.from_numpy(z["r"])[..., 0]                  # r: [T, A, 1] -> [T, A]
    done = torch.from_numpy(z["done"]).float()
    norms = z["norms"]
    assert len(norms) == iters
    for it in range(iters):
        idx = torch.from_numpy(z["starts"][it])[:, None] + torch.arange(C)[None]       # sample_chunk (utils.py:31-49)
        loss = R.vdn_loss(P, T, s[idx], a[idx], r[idx], s2[idx], done[idx][..., None], gamma)
        opt.zero_grad()
        loss.backward()
        norm = torch.nn.utils.clip_grad_norm_([P[n] for n in names], m["grad_clip_norm"], norm_type=2)
        np.testing.assert_allclose(float(norm), norms[it], rtol=1e-4, err_msg=f"iteration {it} gradient norm")
        opt.step()
    for layer, kinds in VDN_PARAMS.items():
        for kind in kinds:
            for i in range(A):
                key = f"{VDN_LAYERS[layer].format(i=i)}.{kind}"
                compact.check(z, "q", key, P[f"{layer}.{kind}"][i].detach().numpy(), lr, iters, s=m["samples"])


def test_maddpg_rnn_restatement_matches_reference_prod():
    z = np.load(os.path.join(GOLD, "learn_maddpg_rnn_prod.npz"))
    m = json.loads(str(z["meta"]))
    N, C, lr, gamma, tau = m["n_agents"], m["chunk"], m["lr"], m["gamma"], m["tau"]
    init = compact.rebuild(m["specs"])

    def stack(net):
        keys = list(init[f"{net}0"])
        return {k: torch.from_numpy(np.stack([init[f"{net}{i}"][k] for i in range(N)])) for k in keys}

    Pc = {n: v.clone().requires_grad_(True) for n, v in stack("critic").items()}
    Ptc, Pa, Pta = stack("target_critic"), stack("actor"), stack("target_actor")
    obs = torch.from_numpy(z["obs"])                                                   # [T+1, N, k]
    act = torch.from_numpy(z["action"])                                                # [T, N, 2]
    rew = torch.from_numpy(z["reward"])                                                # [T, N, 1]
    done = torch.from_numpy(z["done"])[..., None]                                      # [T, N, 1]
    idx = torch.from_numpy(z["starts"])[:, None] + torch.arange(C)[None]               # get_minibatch (memory_rnn.py:69-99)
    total, closs, aloss = R.maddpg_rnn_loss(
        Pc, Ptc, Pa, Pta, obs[:-1][idx], obs[1:][idx], obs[:-1][idx].permute(2, 0, 1, 3),
        obs[1:][idx].permute(2, 0, 1, 3), act[idx].permute(2, 0, 1, 3), rew[idx], done[idx], gamma)
    assert torch.isfinite(closs).all() and torch.isfinite(aloss).all()
    names = list(Pc)
    grads = torch.autograd.grad(total, [Pc[n] for n in names])
    # each agent's critic_optimizer (agent.py:32-33) is its own Adam over its own parameters; stacked, the elementwise
    # update is the same
    ps = [torch.nn.Parameter(Pc[n].detach().clone()) for n in names]
    for p, g in zip(ps, grads):
        p.grad = g
    torch.optim.Adam(ps, lr=lr, foreach=False).step()
    new = dict(zip(names, [p.detach() for p in ps]))
    for i in range(N):
        for n in names:
            compact.check(z, f"critic{i}", n, new[n][i].numpy(), lr, 1, s=m["samples"])
            tc = Ptc[n][i] * (1.0 - tau) + new[n][i] * tau                              # soft_update (net.py:74-78)
            compact.check(z, f"target_critic{i}", n, tc.numpy(), lr, 1, s=m["samples"])
        for n in Pa:  # frozen actors (Q6): unchanged; their targets soft-updated from them, bitwise
            compact.check(z, f"actor{i}", n, Pa[n][i].numpy(), lr, 1, s=m["samples"])
            compact.check(z, f"target_actor{i}", n, (Pta[n][i] * (1.0 - tau) + Pa[n][i] * tau).numpy(), lr, 1,
                          s=m["samples"])
