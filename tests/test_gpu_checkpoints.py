"""Checkpoint files in the reference's formats, written and read by the drop-ins.

* MADDPG: ``{save_dir}/agent_number_{i}_{actor,critic,target_actor,target_critic}_ddpg.pt`` holding a torch
  state_dict with the reference module's keys and shapes (net.py:84-94, agent.py:24-30); replay as ``.npy`` +
  ``dict_info.json`` (memory_rnn.py:104-124); load / load_replay_buffer / load_single_checkpoint /
  load_scaled_checkpoint (MADDPG.py:50-76).
* VDN: ``q_{ep}.pth`` = torch.save(q.state_dict()) (vdn/train_flock.py:130-132), read back by QNet.load_params
  (vdn/net.py:39-50, one agent's weights broadcast to all).
* Shared critic: Actor/TargetActor/Critic files per agent, also the ``best`` copy (train_flock.py:143-151).

Key names and shapes are checked against the golden fixtures the reference's own modules produced
(tests/golden/gen_golden_learn_*.py); every file is read with torch.load(weights_only=True).
"""
import glob
import json
import os
import random
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
NETS = ("actor", "critic", "target_actor", "target_critic")


def _sd(z, prefix):
    return {k[len(prefix) + 1:]: z[k] for k in z.files if k.startswith(prefix + "/")}


def _space(*shape):
    return types.SimpleNamespace(shape=shape)


def _super_agent(flavour, m, tmp, cuda):
    from marl_range_flocking_amd.learners.dropin import SuperAgent, SuperAgentFF

    N, k = m["n_agents"], m["k"]
    env = types.SimpleNamespace(num_particles=N, device=cuda,
                                observation_space=[_space(N, k), [_space(k)] * N], action_space=[_space(2)] * N)
    args = types.SimpleNamespace(ou_theta=0.15, ou_mu=0.0, ou_sigma=0.2, ou_sigma_min=0.001, batch_size=m["batch"],
                                 buffer_size=m["capacity"], min_size_buffer=m["batch"], hidden1=m["hidden1"],
                                 hidden2=m["hidden2"], save_dir=os.path.join(tmp, "ckpt"))
    cls = SuperAgent if flavour == "rnn" else SuperAgentFF
    agent = cls(args, env, path_save=tmp, path_load=tmp)
    agent.learner.min_size_buffer = m["batch"]  # the feed-forward SuperAgent hard-codes 8000 (memory.py)
    return agent


def _assert_same_learner(a, b, N):
    for i in range(N):
        for net in ("actor", "critic"):
            for target in (False, True):
                sa, sb = a.state_dict(net, i, target=target), b.state_dict(net, i, target=target)
                assert list(sa) == list(sb)
                for n in sa:
                    assert torch.equal(sa[n], sb[n]), (net, i, target, n)


@pytest.mark.parametrize("flavour", ["rnn", "ff"])
def test_maddpg_checkpoint_files_round_trip(flavour, tmp_path, cuda):
    z = np.load(os.path.join(GOLD, f"learn_maddpg_{flavour}.npz"))
    m = json.loads(str(z["meta"]))
    N, tmp = m["n_agents"], str(tmp_path)
    a = _super_agent(flavour, m, tmp, cuda)
    a.learner.load_reference_state({f"{nm}{i}": _sd(z, f"init/{nm}{i}") for i in range(N) for nm in NETS})
    for t in range(m["T"]):
        a.replay_buffer.add_record(z["obs"][t], z["obs"][t + 1], z["action"][t], z["obs"][t], z["obs"][t + 1],
                                   z["reward"][t], z["done"][t])
    a.replay_buffer.update_n_games()
    assert a.learner.train(starts=z["starts"]) is not None  # trained critics differ from their targets
    a.save()

    # the files: reference names, the reference modules' keys (in module order) and shapes, the learner's values
    for i in range(N):
        for nm in NETS:
            sd = torch.load(os.path.join(tmp, "ckpt", f"agent_number_{i}_{nm}_ddpg.pt"), weights_only=True)
            gold = _sd(z, f"init/{nm}{i}")
            assert list(sd) == list(gold), (nm, i)
            net, target = nm.replace("target_", ""), nm.startswith("target_")
            mine = a.learner.state_dict(net, i, target=target)
            for n, v in sd.items():
                assert v.dtype == torch.float32 and tuple(v.shape) == gold[n].shape
                assert torch.equal(v, mine[n])
    (folder,) = glob.glob(os.path.join(tmp, "save_agent_*"))
    cap, k = a.replay_buffer.buffer_capacity, m["k"]  # ff: memory.py:12 fixes 1e6 rows
    shapes = {"states": (cap, N, k), "next_states": (cap, N, k), "rewards": (cap, N, 1), "dones": (cap, N, 1)}
    for i in range(N):
        shapes.update({f"states_actor_{i}": (cap, k), f"next_states_actor_{i}": (cap, k),
                       f"actions_actor_{i}": (cap, 2)})
    for name, shape in shapes.items():
        arr = np.load(os.path.join(folder, name + ".npy"))
        assert arr.shape == shape and arr.dtype == np.float32, name
    T = m["T"]
    np.testing.assert_array_equal(np.load(os.path.join(folder, "states.npy"))[:T], z["obs"][:T].reshape(T, N, k))
    np.testing.assert_array_equal(np.load(os.path.join(folder, "actions_actor_1.npy"))[:T],
                                  z["action"][:T].reshape(T, N, 2)[:, 1])
    with open(os.path.join(folder, "dict_info.json")) as f:
        assert json.load(f) == {"buffer_counter": T, "n_games": 1}

    # a fresh agent: load() + load_replay_buffer() restore both; the next update is then bitwise the same
    b = _super_agent(flavour, m, folder, cuda)
    b.save_dir = a.save_dir
    b.load()
    b.load_replay_buffer()
    assert b.replay_buffer.buffer_counter == T and b.replay_buffer.n_games == 1
    for name, buf in a.learner.replay.bufs.items():
        assert torch.equal(buf, b.learner.replay.bufs[name]), name
    _assert_same_learner(a.learner, b.learner, N)
    # the Adam moments are not part of the reference checkpoint: copy a's, then train both once more
    for pa, pb in ((a.learner.actors, b.learner.actors), (a.learner.critics, b.learner.critics)):
        for name in ("exp_avg", "exp_avg_sq", "step_dev"):
            if getattr(pa, name) is not None:  # the frozen MADDPG actors carry no Adam state
                getattr(pb, name).copy_(getattr(pa, name))
        pb.step_count, pb.agent_steps = pa.step_count, list(pa.agent_steps)
    a.learner.train(starts=z["starts"])
    b.learner.train(starts=z["starts"])
    torch.cuda.synchronize()
    _assert_same_learner(a.learner, b.learner, N)

    # load_single_checkpoint: one actor file for every agent; load_scaled_checkpoint: a random saved actor each
    c = _super_agent(flavour, m, tmp, cuda)
    c.load_single_checkpoint(os.path.join(tmp, "ckpt", "agent_number_1_actor_ddpg.pt"))
    want = a.learner.state_dict("actor", 1)
    for i in range(N):
        for n, v in c.learner.state_dict("actor", i).items():
            assert torch.equal(v, want[n])
    random.seed(4)
    picks = [random.randint(0, N - 1) for _ in range(N)]
    random.seed(4)
    c.load_scaled_checkpoint(os.path.join(tmp, "ckpt"), total=N - 1)
    for i, p in enumerate(picks):
        want = a.learner.state_dict("actor", p)
        for n, v in c.learner.state_dict("actor", i).items():
            assert torch.equal(v, want[n])


def test_vdn_q_pth_and_load_params(tmp_path, cuda):
    from marl_range_flocking_amd.learners.dropin import QNet

    z = np.load(os.path.join(GOLD, "learn_vdn.npz"))
    m = json.loads(str(z["meta"]))
    A = m["n_agents"]
    obs_space = [_space(m["k"])] * A
    act_space = [types.SimpleNamespace(n=m["n_actions"])] * A
    q = QNet(obs_space, act_space, recurrent=True, device=cuda)
    gold = _sd(z, "final_q")
    q.load_state_dict(gold)
    path = os.path.join(str(tmp_path), "q_100.pth")  # train_flock.py:131
    torch.save(q.state_dict(), path)
    sd = torch.load(path, weights_only=True)
    assert sorted(sd) == sorted(gold)
    for n, v in sd.items():
        np.testing.assert_array_equal(v.numpy(), gold[n])
    # test_flock.py:27: q.load_params(q_dir, agent_i=best_agent) gives every agent that agent's network
    q2 = QNet(obs_space, act_space, recurrent=True, device=cuda)
    q2.load_params(path, agent_i=2)
    got = q2.state_dict()
    for n, v in got.items():
        src = n.replace(n.split(".")[0], n.split(".")[0].rsplit("_", 1)[0] + "_2", 1)
        np.testing.assert_array_equal(v.cpu().numpy(), gold[src], err_msg=n)


@pytest.mark.parametrize("best", [False, True], ids=["save_models", "save_models_best"])
def test_shared_critic_models_files(tmp_path, best, cuda):
    """The reference driver's directory layout (maddpg_shared_critic/train_flock.py:40-66): the critic in
    CHECKPOINT_DIR/critic (best: CHECKPOINT_DIR/best), each agent's Actor / TargetActor in CHECKPOINT_DIR/agent_i
    (best: CHECKPOINT_DIR/best); file names {name}_ddpg.pt (ddpg_network.py:33-34). save_models(_best) writes the
    reference's files with its state_dict keys; load_models on a fresh learner reads them back."""
    from marl_range_flocking_amd.learners import dropin

    z = np.load(os.path.join(GOLD, "learn_shared_critic.npz"))
    m = json.loads(str(z["meta"]))
    A, K = m["n_agents"], m["k"]
    ck = str(tmp_path)

    def build():
        rb = dropin.ReplayBuffer(64, [K], n_actions=2, n_agents=A)
        critic = dropin.CriticNetwork(m["beta"], [K], m["fc1"], m["fc2"], n_actions=2, name="Critic",
                                      chkpt_dir=os.path.join(ck, "critic"), chkpt_best_dir=os.path.join(ck, "best"))
        agents = [dropin.Agent(shared_critic=critic, replay_buffer=rb, noise=None, index=i, alpha=m["alpha"],
                               beta=m["beta"], input_dims=[K], layer1_size=m["fc1"], layer2_size=m["fc2"],
                               tau=m["tau"], batch_size=m["batch"], checkpoint_dir=os.path.join(ck, f"agent_{i}"),
                               checkpoint_best=os.path.join(ck, "best")) for i in range(A)]
        return critic._build(), agents

    L, agents = build()
    L.load_reference_state(_sd(z, "final/critic"), [_sd(z, f"final/actor{i}") for i in range(A)],
                           [_sd(z, f"final/target_actor{i}") for i in range(A)])
    if best:
        agents[2].save_models_best()
    else:
        agents[2].save_models()
    adir = os.path.join(ck, "best" if best else "agent_2")
    files = {"Actor": os.path.join(adir, "Actor_ddpg.pt"), "TargetActor": os.path.join(adir, "TargetActor_ddpg.pt"),
             "Critic": os.path.join(ck, "best" if best else "critic", "Critic_ddpg.pt")}
    for n, gold in (("Actor", "final/actor2"), ("TargetActor", "final/target_actor2"), ("Critic", "final/critic")):
        sd, g = torch.load(files[n], weights_only=True), _sd(z, gold)
        assert list(sd) == list(g), n
        for key, v in sd.items():
            np.testing.assert_array_equal(v.numpy(), g[key], err_msg=f"{n} {key}")
    L2, agents2 = build()
    if best:  # agent 0 takes agent 2's saved best actor; the critic is shared
        agents2[0].load_models(best=True)
        src, dst = 2, 0
    else:
        agents2[2].load_models()
        src, dst = 2, 2
    for key, v in L2.actor_state_dict(dst).items():
        np.testing.assert_array_equal(v.numpy(), z[f"final/actor{src}/{key}"])
    for key, v in L2.actor_state_dict(dst, target=True).items():
        np.testing.assert_array_equal(v.numpy(), z[f"final/target_actor{src}/{key}"])
    for key, v in L2.critic_state_dict().items():
        np.testing.assert_array_equal(v.numpy(), z[f"final/critic/{key}"])
