"""GPU learner updates against golden vectors produced by the REFERENCE learners (tests/golden/gen_golden_learn_*.py).

Tolerance rules: losses rtol 1e-4; parameters after Adam compared only where every consumed
gradient had |g| > 1e-6 (Adam's first steps are lr * g / (|g| + eps): sign-unstable for tiny g), rtol 1e-4 / atol 1e-6;
frozen networks bitwise unchanged.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _sd(z, prefix):
    out = {}
    for k in z.files:
        if k.startswith(prefix + "/"):
            out[k[len(prefix) + 1:]] = z[k]
    return out


def _masked_close(got, want, grads, what, lr, rtol=1e-4, atol=1e-6):
    """Well-conditioned elements (every consumed |g| > 1e-6, or exactly 0 — dead ReLU units) within rtol/atol; the
    rest may differ by at most the Adam step bound 2 * lr per step (sign-unstable lr * g / (|g| + eps))."""
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    mask = np.ones(want.shape, bool)
    for g in grads:
        mask &= (np.abs(g) > 1e-6) | (g == 0)
    err = np.abs(got - want)
    bad = mask & (err > atol + rtol * np.abs(want))
    assert not bad.any(), f"{what}: {bad.sum()} / {mask.sum()} elements off, max err {err[mask].max()}"
    loose = ~mask & (err > 2.0 * lr * max(1, len(grads)) + atol)
    assert not loose.any(), f"{what}: ill-conditioned elements beyond the Adam step bound: {err[~mask].max()}"


@pytest.mark.parametrize("fused", [True, False], ids=["fused", "autograd"])
@pytest.mark.parametrize("use_graph", [False, True], ids=["eager", "hipgraph"])
def test_shared_critic_learn_matches_reference(use_graph, fused, cuda):
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner

    z = np.load(os.path.join(GOLD, "learn_shared_critic.npz"))
    m = json.loads(str(z["meta"]))
    A, K = m["n_agents"], m["k"]
    L = SharedCriticLearner(A, K, fc1=m["fc1"], fc2=m["fc2"], alpha=m["alpha"], beta=m["beta"], gamma=m["gamma"],
                            tau=m["tau"], batch_size=m["batch"], update_rate=m["update_rate"],
                            buffer_size=m["capacity"], device=cuda, use_graph=use_graph, fused=fused)
    L.load_reference_state(_sd(z, "init/critic"), [_sd(z, f"init/actor{i}") for i in range(A)],
                           [_sd(z, f"init/target_actor{i}") for i in range(A)])
    for t in range(z["state"].shape[0]):
        L.store_transitions(torch.tensor(z["state"][t]), torch.tensor(z["action"][t]), torch.tensor(z["reward"][t]),
                            torch.tensor(z["next_state"][t]), torch.tensor(z["done"][t]))
    for c, i in enumerate(m["calls"]):
        al, cl, ok = L.learn(i, idx=torch.tensor(z["idx"][c]))
        assert ok
        np.testing.assert_allclose([al.item(), cl.item()], z["losses"][c], rtol=1e-4)
    crit = L.critic_state_dict()
    for n, v in crit.items():
        grads = [z[f"grad/call{c}.critic.{n}"] for c in range(len(m["calls"]))]
        _masked_close(v.numpy(), z[f"final/critic/{n}"], grads, f"critic {n}", m["beta"])
    for i in range(A):
        calls = [c for c, a in enumerate(m["calls"]) if a == i]
        for target in (False, True):
            sd = L.actor_state_dict(i, target=target)
            tag = "target_actor" if target else "actor"
            for n, v in sd.items():
                grads = [z[f"grad/call{c}.actor.{n}"] for c in calls]
                _masked_close(v.numpy(), z[f"final/{tag}{i}/{n}"], grads, f"{tag}{i} {n}", m["alpha"])


@pytest.mark.parametrize("fused", [True, False], ids=["fused", "autograd"])
@pytest.mark.parametrize("use_graph", [False, True], ids=["eager", "hipgraph"])
def test_shared_critic_learn_matches_reference_prod(use_graph, fused, cuda):
    """The reference's production shape (fc1 400, fc2 300, B 256; train_flock.py:15-27, :64) with 8 agents: the
    whole-K-panel MFMA tiles and the fused row kernels the bench runs, against the REFERENCE Agent.learn() (compact
    fixture, tests/golden/compact.py): losses of all 6 calls, the critic, the four learning actors and their targets
    (sampled positions, SURVEY.md §8(c) rule), the non-learning actors bitwise."""
    from golden import compact
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner

    z = np.load(os.path.join(GOLD, "learn_shared_critic_prod.npz"))
    m = json.loads(str(z["meta"]))
    A, K = m["n_agents"], m["k"]
    init = compact.rebuild(m["specs"])
    L = SharedCriticLearner(A, K, fc1=m["fc1"], fc2=m["fc2"], alpha=m["alpha"], beta=m["beta"], gamma=m["gamma"],
                            tau=m["tau"], batch_size=m["batch"], update_rate=m["update_rate"],
                            buffer_size=m["capacity"], device=cuda, use_graph=use_graph, fused=fused)
    L.load_reference_state(init["critic"], [init[f"actor{i}"] for i in range(A)],
                           [init[f"target_actor{i}"] for i in range(A)])
    for t in range(z["state"].shape[0]):
        L.store_transitions(torch.tensor(z["state"][t]), torch.tensor(z["action"][t]), torch.tensor(z["reward"][t]),
                            torch.tensor(z["next_state"][t]), torch.tensor(z["done"][t]))
    for c, i in enumerate(m["calls"]):
        al, cl, ok = L.learn(i, idx=torch.tensor(z["idx"][c]))
        assert ok
        np.testing.assert_allclose([al.item(), cl.item()], z["losses"][c], rtol=1e-4)
    for n, v in L.critic_state_dict().items():
        compact.check(z, "critic", n, v.numpy(), m["beta"], len(m["calls"]))
    for i in range(A):
        steps = sum(1 for a in m["calls"] if a == i)
        for target in (False, True):
            tag = ("target_actor" if target else "actor") + str(i)
            for n, v in L.actor_state_dict(i, target=target).items():
                if steps == 0:  # never learned: bitwise the initial parameters
                    np.testing.assert_array_equal(v.numpy(), init[tag][n], err_msg=f"{tag} {n}")
                else:
                    compact.check(z, tag, n, v.numpy(), m["alpha"], steps)


def test_shared_critic_fused_matches_autograd_at_bench_size(cuda):
    """The fused HIP update (csrc/flock_sc.hip) against the autograd formulation at the bench shape (fc1 400,
    fc2 300, B 256): per-call gradients of the critic and of the learning actor, losses, and parameters after 6
    learn() calls over 3 agents from identical states and minibatches."""
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner

    torch.manual_seed(0)
    A, K, B = 3, 4, 256
    Ls = [SharedCriticLearner(A, K, batch_size=B, buffer_size=4096, device=cuda, seed=7, fused=f, use_graph=f)
          for f in (True, False)]
    n = 2048
    rows = (torch.rand(n, K, device=cuda) * 14, torch.rand(n, 2, device=cuda) * 2 - 1, torch.randn(n, 1, device=cuda),
            torch.rand(n, K, device=cuda) * 14, (torch.rand(n, device=cuda) < 0.1).float())
    for L in Ls:
        L.store_transitions(*rows)
    Lf, La = Ls
    gen = torch.Generator(device=cuda).manual_seed(3)
    for call, agent in enumerate([0, 1, 2, 0, 1, 2]):
        idx = torch.randint(0, n, (B,), device=cuda, generator=gen)
        outs = [L.learn(agent, idx=idx) for L in Ls]
        torch.testing.assert_close(torch.stack(outs[0][:2]), torch.stack(outs[1][:2]), rtol=1e-4, atol=1e-6)
        gc_f, gc_a = Lf.critic.grad, La.critic.grad
        scale = gc_a.abs().max()
        torch.testing.assert_close(gc_f, gc_a, rtol=1e-3, atol=1e-4 * float(scale))
        lo, hi = Lf.actors.agent_range(agent)
        ga_f, ga_a = Lf.actors.grad[lo:hi], La.scratch.grad
        torch.testing.assert_close(ga_f, ga_a, rtol=1e-3, atol=1e-4 * float(ga_a.abs().max()))
        # parameters after Adam: identical up to the Adam step bound on ill-conditioned (|g| ~ 0) elements
        for x, y in ((Lf.critic.data, La.critic.data), (Lf.actors.data, La.actors.data),
                     (Lf.actors.target, La.actors.target)):
            assert float((x - y).abs().max()) <= 2 * 3e-4 * (call + 1) + 1e-6
    assert torch.equal(Lf.actor_steps, La.actor_steps)
    assert int(Lf.critic.step_dev) == int(La.critic.step_dev) == 6


def test_shared_critic_choose_action_batched(cuda):
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner, actor_forward

    L = SharedCriticLearner(5, 4, fc1=16, fc2=8, device=cuda)
    obs = torch.rand(7, 5, 4, device=cuda) * 14
    mu = L.choose_action(obs, noise=False)
    for i in range(5):
        P = {n: L.actors.view(L.actors.data, n, i) for n in L.actors.shapes}
        ref = actor_forward(P, obs[:, i])[0]
        torch.testing.assert_close(mu[:, i], ref, rtol=1e-5, atol=1e-6)
    a = L.choose_action(obs)
    assert a.shape == (7, 5, 2) and not torch.equal(a, mu)


@pytest.mark.parametrize("use_graph", [False, True], ids=["eager", "hipgraph"])
def test_vdn_train_matches_reference(use_graph, cuda):
    from marl_range_flocking_amd.learners.vdn import VDNLearner, reference_key

    z = np.load(os.path.join(GOLD, "learn_vdn.npz"))
    m = json.loads(str(z["meta"]))
    A = m["n_agents"]
    L = VDNLearner(A, m["k"], m["n_actions"], lr=m["lr"], gamma=m["gamma"], batch_size=m["batch"],
                   chunk_size=m["chunk"], update_iter=m["update_iter"], grad_clip_norm=m["grad_clip_norm"],
                   device=cuda, use_graph=use_graph)
    L.q.load_reference_state_dict(_sd(z, "init_q"))
    L.q.load_reference_state_dict(_sd(z, "init_target"), target=True)
    # QNet forward (net.py:27-37) on the fixture batch
    qo, ho = L.q(torch.tensor(z["fwd_obs"], device=cuda), torch.tensor(z["fwd_hidden"], device=cuda))
    L.q.load_reference_state_dict(_sd(z, "init_q"))
    for t in range(m["T"]):
        L.put(z["s"][t], z["a"][t], z["r"][t], z["s_prime"][t], [int(z["done"][t])])
    L.train(starts=z["starts"])
    norm = L.norm.out[0].item()
    np.testing.assert_allclose(norm, z["norms"][-1], rtol=1e-4)
    final = L.q.state_dict()
    for name in L.q.P.shapes:
        for i in range(A):
            key = reference_key(name, i)
            grads = [z[f"grad{it}/{key}"] for it in range(m["update_iter"])]
            _masked_close(final[key].numpy(), z[f"final_q/{key}"], grads, key, m["lr"])


@pytest.mark.parametrize("use_graph", [False, True], ids=["eager", "hipgraph"])
def test_vdn_train_matches_reference_prod(use_graph, cuda):
    """VDN with 64 agents at the reference driver's settings (B 32, chunk 10, update_iter 10; train_flock.py:16-43)
    against the REFERENCE train() (compact fixture, tests/golden/compact.py): every iteration's pre-clip gradient norm
    rtol 1e-4 is implied by the last one, final QNet parameters at sampled positions (SURVEY.md §8(c) rule), and the
    QNet forward on a fixed batch."""
    from golden import compact
    from marl_range_flocking_amd.learners.vdn import VDNLearner

    z = np.load(os.path.join(GOLD, "learn_vdn_prod.npz"))
    m = json.loads(str(z["meta"]))
    A, S = m["n_agents"], m["samples"]
    init = compact.rebuild(m["specs"])
    L = VDNLearner(A, m["k"], m["n_actions"], lr=m["lr"], gamma=m["gamma"], batch_size=m["batch"],
                   chunk_size=m["chunk"], update_iter=m["update_iter"], grad_clip_norm=m["grad_clip_norm"],
                   device=cuda, use_graph=use_graph)
    L.q.load_reference_state_dict(init["q"])
    L.q.load_reference_state_dict(init["target_q"], target=True)
    for t in range(m["T"]):
        L.put(z["s"][t], z["a"][t], z["r"][t], z["s_prime"][t], [int(z["done"][t])])
    L.train(starts=z["starts"])
    np.testing.assert_allclose(L.norm.out[0].item(), z["norms"][-1], rtol=1e-4)
    for key, v in L.q.state_dict().items():
        compact.check(z, "q", key, v.numpy(), m["lr"], m["update_iter"], s=S)
    qo, ho = L.q(torch.tensor(z["fwd_obs"], device=cuda), torch.tensor(z["fwd_hidden"], device=cuda))
    np.testing.assert_allclose(qo.detach().cpu().numpy(), z["fwd_q"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(ho.detach().cpu().numpy(), z["fwd_h"], rtol=1e-4, atol=1e-5)


def test_vdn_forward_matches_reference_qnet(cuda):
    from marl_range_flocking_amd.learners.vdn import BatchedQNet

    z = np.load(os.path.join(GOLD, "learn_vdn.npz"))
    m = json.loads(str(z["meta"]))
    q = BatchedQNet(m["n_agents"], m["k"], m["n_actions"], device=cuda)
    q.load_reference_state_dict(_sd(z, "final_q"))
    qo, ho = q(torch.tensor(z["fwd_obs"], device=cuda), torch.tensor(z["fwd_hidden"], device=cuda))
    np.testing.assert_allclose(qo.detach().cpu().numpy(), z["fwd_q"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(ho.detach().cpu().numpy(), z["fwd_h"], rtol=1e-4, atol=1e-5)
    a, h = q.sample_action(torch.tensor(z["fwd_obs"], device=cuda), torch.tensor(z["fwd_hidden"], device=cuda), 0.0)
    np.testing.assert_array_equal(a.cpu().numpy(), z["fwd_q"].argmax(-1).astype(np.float32))


@pytest.mark.parametrize("flavour", ["rnn", "ff"])
@pytest.mark.parametrize("use_graph", [False, True], ids=["eager", "hipgraph"])
def test_maddpg_train_matches_reference(flavour, use_graph, cuda):
    from marl_range_flocking_amd.learners.maddpg import MADDPGLearner

    z = np.load(os.path.join(GOLD, f"learn_maddpg_{flavour}.npz"))
    m = json.loads(str(z["meta"]))
    N = m["n_agents"]
    L = MADDPGLearner(N, m["k"], recurrent=flavour == "rnn", hidden1=m["hidden1"], hidden2=m["hidden2"],
                      batch_size=m["batch"], chunk_size=m["chunk"], buffer_capacity=m["capacity"],
                      min_size_buffer=m["batch"], device=cuda, use_graph=use_graph)
    nets = ("actor", "critic", "target_actor", "target_critic")
    L.load_reference_state({f"{nm}{i}": _sd(z, f"init/{nm}{i}") for i in range(N) for nm in nets})
    for t in range(m["T"]):
        L.add_record(z["obs"][t], z["obs"][t + 1], z["action"][t], z["obs"][t], z["obs"][t + 1], z["reward"][t],
                     z["done"][t])
    assert L.train(starts=z["starts"]) is not None
    for i in range(N):
        for n, v in L.state_dict("actor", i).items():  # frozen actors (Q6): bitwise unchanged
            np.testing.assert_array_equal(v.numpy(), z[f"final/actor{i}/{n}"])
        for n, v in L.state_dict("actor", i, target=True).items():  # t*(1-tau) + a*tau, same op order
            np.testing.assert_array_equal(v.numpy(), z[f"final/target_actor{i}/{n}"])
        for n, v in L.state_dict("critic", i).items():
            g = [z[f"grad/critic{i}/{n}"]]
            _masked_close(v.numpy(), z[f"final/critic{i}/{n}"], g, f"critic{i} {n}", m["lr"])
        for n, v in L.state_dict("critic", i, target=True).items():
            g = [z[f"grad/critic{i}/{n}"]]
            _masked_close(v.numpy(), z[f"final/target_critic{i}/{n}"], g, f"target_critic{i} {n}", m["lr"])
    # acting without noise (agent.choose_action, test=True)
    obs0 = torch.tensor(z["obs"][0], device=cuda)
    acts, hid = L.get_actions(obs0, None, test=True)
    np.testing.assert_allclose(acts.cpu().numpy(), z["act_out"], rtol=1e-5, atol=1e-6)
    if flavour == "rnn":
        np.testing.assert_allclose(hid[:, 0].cpu().numpy(), z["act_hidden"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("use_graph", [False, True], ids=["eager", "hipgraph"])
def test_maddpg_rnn_train_matches_reference_prod(use_graph, cuda):
    """RNN-MADDPG at the reference's production shape (hidden 400/300, B 128, chunk 10; net.py:14-146,
    MADDPG.py:78-150) with 16 agents, against the REFERENCE SuperAgent.train() (compact fixture,
    tests/golden/compact.py): critics and target critics at sampled positions (SURVEY.md §8(c) rule), frozen actors
    and the target actors' soft update bitwise, acting outputs rtol 1e-5."""
    from golden import compact
    from marl_range_flocking_amd.learners.maddpg import MADDPGLearner

    z = np.load(os.path.join(GOLD, "learn_maddpg_rnn_prod.npz"))
    m = json.loads(str(z["meta"]))
    N, S = m["n_agents"], m["samples"]
    L = MADDPGLearner(N, m["k"], recurrent=True, hidden1=m["hidden1"], hidden2=m["hidden2"], batch_size=m["batch"],
                      chunk_size=m["chunk"], buffer_capacity=m["capacity"], min_size_buffer=m["batch"], device=cuda,
                      use_graph=use_graph)
    L.load_reference_state({tag: sd for tag, sd in compact.rebuild(m["specs"]).items()})
    for t in range(m["T"]):
        L.add_record(z["obs"][t], z["obs"][t + 1], z["action"][t], z["obs"][t], z["obs"][t + 1], z["reward"][t],
                     z["done"][t])
    assert L.train(starts=z["starts"]) is not None
    for i in range(N):
        for net in ("actor", "critic"):
            for target in (False, True):
                tag = ("target_" if target else "") + f"{net}{i}"
                for n, v in L.state_dict(net, i, target=target).items():
                    compact.check(z, tag, n, v.numpy(), m["lr"], 1, s=S)
    acts, hid = L.get_actions(torch.tensor(z["obs"][0], device=cuda), None, test=True)
    np.testing.assert_allclose(acts.cpu().numpy(), z["act_out"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(hid[:, 0].cpu().numpy(), z["act_hidden"], rtol=1e-5, atol=1e-6)


def test_shared_ou_matches_sequential_process(cuda):
    """The closed-form scan equals the reference's agent-after-agent OU recurrence (utils.py:43-47)."""
    from marl_range_flocking_amd.learners.maddpg import SharedOU

    g = torch.Generator(device=cuda).manual_seed(0)
    ou = SharedOU(2, 0.15, 0.0, 0.2, 0.001, 1e-2, cuda, g)
    xs = ou.sample(64, envs=3)
    g2 = torch.Generator(device=cuda).manual_seed(0)
    z = torch.randn((3, 64, 2), generator=g2, device=cuda).double()
    x = torch.zeros(3, 2, dtype=torch.float64, device=cuda)
    ref = []
    for i in range(64):
        x = x + 0.15 * (0.0 - x) * 1e-2 + 0.2 * np.sqrt(1e-2) * z[:, i]
        ref.append(x)
    torch.testing.assert_close(xs, torch.stack(ref, 1).float(), rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("cap", [100, 40], ids=["wrap", "step-larger-than-ring"])
def test_fused_env_record_insert_matches_add_record(cap, cuda):
    """The RNN-MADDPG record layout (one ring row per env, memory_rnn.py:53-67): VecFlockEnv.step(ring=
    learner.replay_slots(E)) leaves every replay field and the counter bitwise equal to step() followed by
    add_record(obs, next_obs, actions, obs, next_obs, reward, done) for every env, across a ring wrap and with a
    step of more envs than the ring holds."""
    from marl_range_flocking_amd import FlockConfig, VecFlockEnv
    from marl_range_flocking_amd.learners.maddpg import MADDPGLearner

    E, N, k, box = 64, 12, 4, 55.0
    envs, learners = [], []
    for _ in range(2):
        env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                                      range_start=(0, box), sensor_range=14.0), device=cuda)
        g = torch.Generator(device=cuda).manual_seed(5)
        env.positions.copy_(torch.rand(E, N, 2, device=cuda, generator=g) * box)
        env.headings.copy_(torch.rand(E, N, device=cuda, generator=g) * 4.7)
        env.step(torch.zeros(E, N, 2, device=cuda))
        envs.append(env)
        learners.append(MADDPGLearner(N, k, recurrent=True, hidden1=16, hidden2=8, batch_size=8, chunk_size=4,
                                      buffer_capacity=cap, min_size_buffer=8, device=cuda, use_graph=False))
    g = torch.Generator(device=cuda).manual_seed(9)
    for _ in range(3):
        a = torch.stack([torch.rand(E, N, device=cuda, generator=g) * 3 - 0.5,
                         torch.rand(E, N, device=cuda, generator=g) * 4 - 2], -1).contiguous()
        fused_env, plain_env = envs
        fused_env.step(a, ring=learners[0].replay_slots(E))
        prev = plain_env.dnn.clone()
        plain_env.step(a)
        learners[1].add_record(prev, plain_env.dnn, a, prev, plain_env.dnn, plain_env.reward, plain_env.done)
        assert torch.equal(fused_env.dnn, plain_env.dnn) and torch.equal(fused_env.reward, plain_env.reward)
    assert learners[0].replay.counter == learners[1].replay.counter == 3 * E
    for name in learners[0].replay.bufs:
        assert torch.equal(learners[0].replay.bufs[name], learners[1].replay.bufs[name]), name


@pytest.mark.parametrize("cap", [10000, 5000], ids=["wrap", "step-larger-than-ring"])
def test_fused_env_replay_insert_matches_store_transitions(cap, cuda):
    """VecFlockEnv.step(ring=learner.replay_slots(n)) (flock_step_v2_store) leaves the replay ring, counter and
    env outputs bitwise equal to step() followed by store_transitions(prev_obs, action, reward, obs, done), over
    three steps with a ring wrap-around, and with a step larger than the whole ring (only the last rows kept)."""
    from marl_range_flocking_amd import FlockConfig, VecFlockEnv
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner

    E, N, k, box = 64, 128, 4, 179.0
    envs, learners = [], []
    for _ in range(2):
        env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                                      range_start=(0, box), sensor_range=14.0), device=cuda)
        g = torch.Generator(device=cuda).manual_seed(5)
        env.positions.copy_(torch.rand(E, N, 2, device=cuda, generator=g) * box)
        env.headings.copy_(torch.rand(E, N, device=cuda, generator=g) * 4.7)
        env.step(torch.zeros(E, N, 2, device=cuda))
        envs.append(env)
        learners.append(SharedCriticLearner(N, k, fc1=32, fc2=24, batch_size=16, buffer_size=cap, device=cuda))
    g = torch.Generator(device=cuda).manual_seed(9)
    for _ in range(3):
        a = torch.stack([torch.rand(E, N, device=cuda, generator=g) * 3 - 0.5,
                         torch.rand(E, N, device=cuda, generator=g) * 4 - 2], -1).contiguous()
        fused_env, plain_env = envs
        fused_env.step(a, ring=learners[0].replay_slots(E * N))
        prev = plain_env.dnn.clone()
        plain_env.step(a)
        n = E * N
        learners[1].store_transitions(prev.reshape(n, -1), a.reshape(n, -1), plain_env.reward.reshape(n, 1),
                                      plain_env.dnn.reshape(n, -1), plain_env.done.reshape(n))
        assert torch.equal(fused_env.dnn, plain_env.dnn) and torch.equal(fused_env.reward, plain_env.reward)
    assert learners[0].replay.counter == learners[1].replay.counter == 3 * E * N
    for name in learners[0].replay.bufs:
        assert torch.equal(learners[0].replay.bufs[name], learners[1].replay.bufs[name]), name


@pytest.mark.parametrize("N,cap", [(16, 100), (128, 40), (128, 25)], ids=["N16-wrap", "N128-wrap", "N128-larger"])
def test_fused_vdn_team_insert_matches_put(N, cap, cuda):
    """The VDN team transition (memory.put((s, a, r, s', [all_done])), learners/vdn/train_flock.py:102): a
    uw_discrete VecFlockEnv.step(ids, ring=vdn.replay_slots(E)) writes previous obs, action ids as f32, rewards,
    new obs and the env's any_done from the step kernel; every replay field and the counter equal step() followed by
    put(prev, ids, reward, obs, any_done) bit for bit, across a ring wrap and with a step larger than the ring."""
    from marl_range_flocking_amd import FlockConfig, VecFlockEnv
    from marl_range_flocking_amd.learners.vdn import VDNLearner

    E, k = 32, 4
    box = float(round(np.sqrt(250.0 * N)))
    envs, learners = [], []
    for _ in range(2):
        env = VecFlockEnv(FlockConfig(variant="uw_discrete", num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                                      range_start=(0, box), sensor_range=14.0), device=cuda)
        g = torch.Generator(device=cuda).manual_seed(5)
        env.positions.copy_(torch.rand(E, N, 2, device=cuda, generator=g) * box)
        env.headings.copy_(torch.rand(E, N, device=cuda, generator=g) * 2.6)
        env.step(torch.zeros(E, N, dtype=torch.int64, device=cuda))
        envs.append(env)
        learners.append(VDNLearner(N, k, 10, batch_size=4, chunk_size=2, buffer_limit=cap, device=cuda,
                                   use_graph=False))
    g = torch.Generator(device=cuda).manual_seed(9)
    for _ in range(3):
        ids = torch.randint(0, 10, (E, N), device=cuda, generator=g)
        fused_env, plain_env = envs
        fused_env.step(ids, ring=learners[0].replay_slots(E))
        prev = plain_env.dnn.clone()
        plain_env.step(ids)
        learners[1].put(prev, ids, plain_env.reward, plain_env.dnn, plain_env.any_done)
        assert torch.equal(fused_env.dnn, plain_env.dnn) and torch.equal(fused_env.any_done, plain_env.any_done)
    assert learners[0].replay.counter == learners[1].replay.counter == 3 * E
    for name in learners[0].replay.bufs:
        assert torch.equal(learners[0].replay.bufs[name], learners[1].replay.bufs[name]), name
