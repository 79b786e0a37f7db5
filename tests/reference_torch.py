"""Plain-PyTorch fp32 restatements of the reference learner updates, batched over agents (test infrastructure only).

These follow the reference's own loop structure step by step — one forward per chunk step, nn.GRUCell math written
out, the done resets as in-place masks, heads evaluated at every step — with autograd for the gradients. They share
no code with the build's learners (no gru_seq, no fused kernels, no flat buffers), so the config-scale tests
(tests/test_gpu_learners_scale.py) compare two independent formulations at shapes too large for a reference fixture.

  vdn_loss        learners/vdn/train_flock.py:18-38 (QNet learners/vdn/net.py:27-37)
  maddpg_rnn_loss learners/maddpg_official_rnn/MADDPG.py:83-139 (Actor / Critic net.py:50-72, :130-146)
"""
import torch
import torch.nn.functional as F


def lin(x, w, b):
    """Per-agent nn.Linear: x [A,B,in], w [A,out,in], b [A,out] -> [A,B,out]."""
    return torch.baddbmm(b[:, None], x, w.transpose(1, 2))


def gru_cell(x, h, wih, whh, bih, bhh):
    """nn.GRUCell (gates r, z, n), per agent."""
    gi, gh = lin(x, wih, bih), lin(h, whh, bhh)
    ir, iz, i_n = gi.chunk(3, -1)
    hr, hz, h_n = gh.chunk(3, -1)
    r = torch.sigmoid(ir + hr)
    z = torch.sigmoid(iz + hz)
    n = torch.tanh(i_n + r * h_n)
    return (1 - z) * n + z * h


# ------------------------------------------------------------------------------------------------------------ VDN
def qnet(P, obs, h):
    """QNet.forward (net.py:27-37) for all agents: obs [A,B,n_obs], h [A,B,32] -> q [A,B,n_act], h'."""
    x = F.relu(lin(obs, P["feat1.weight"], P["feat1.bias"]))
    x = F.relu(lin(x, P["feat2.weight"], P["feat2.bias"]))
    x = gru_cell(x, h, P["gru.weight_ih"], P["gru.weight_hh"], P["gru.bias_ih"], P["gru.bias_hh"])
    return lin(x, P["q.weight"], P["q.bias"]), x


def vdn_loss(P, T, s, a, r, s_prime, done, gamma):
    """One update iteration's loss (train_flock.py:18-38). s, s_prime [B,C,A,n_obs]; a, r [B,C,A]; done [B,C,1]."""
    B, C, A, _ = s.shape
    hidden = torch.zeros((A, B, 32), dtype=s.dtype, device=s.device)
    target_hidden = torch.zeros_like(hidden)
    loss = 0
    for t in range(C):
        q_out, hidden = qnet(P, s[:, t].transpose(0, 1), hidden)
        q_a = q_out.gather(2, a[:, t].t().long().unsqueeze(-1)).squeeze(-1)       # [A, B]
        sum_q = q_a.t().sum(dim=1, keepdim=True)                                    # [B, 1]
        with torch.no_grad():
            mq, target_hidden = qnet(T, s_prime[:, t].transpose(0, 1), target_hidden)
            mq = mq.max(dim=2)[0].t()                                               # [B, A]
            target_q = r[:, t].sum(dim=1, keepdim=True)
            target_q = target_q + gamma * mq.sum(dim=1, keepdim=True) * (1 - done[:, t])
        loss = loss + F.smooth_l1_loss(sum_q, target_q)
        keep = (done[:, t, 0] == 0)[None, :, None]                                  # hidden[done_mask] = 0
        hidden = torch.where(keep, hidden, 0.0)
        target_hidden = torch.where(keep, target_hidden, 0.0)
    return loss


# ---------------------------------------------------------------------------------------------------- RNN-MADDPG
def rnn_actor(P, x, h):
    """Actor.forward (net.py:50-72): x [A,B,k], h [A,B,32] -> actions [A,B,2], h'."""
    out = lin(x, P["fce.weight"], P["fce.bias"])
    h = gru_cell(out, h, P["gru.weight_ih"], P["gru.weight_hh"], P["gru.bias_ih"], P["gru.bias_hh"])
    out = F.relu(lin(h, P["fc1.weight"], P["fc1.bias"]))
    out = F.relu(lin(out, P["fc2.weight"], P["fc2.bias"]))
    speed = (torch.tanh(lin(out, P["linear_speed.weight"], P["linear_speed.bias"])) + 1) / 2
    ang = torch.tanh(lin(out, P["angular_speed.weight"], P["angular_speed.bias"])) * 1.5
    return torch.cat([speed, ang], -1), h


def rnn_critic(P, x, a, h):
    """Critic.forward (net.py:130-146) of every agent on the SAME (x [B, N*k], a [B, 2N]): h [A,B,32] ->
    q [A,B,1], h'. P["fc2.weight"] is the reference's joined [A, h2, h1 + 2N] weight."""
    A = h.shape[0]
    out = torch.einsum("bi,aoi->abo", x, P["fce.weight"]) + P["fce.bias"][:, None]
    h = gru_cell(out, h, P["gru.weight_ih"], P["gru.weight_hh"], P["gru.bias_ih"], P["gru.bias_hh"])
    out = F.relu(lin(h, P["fc1.weight"], P["fc1.bias"]))
    out = F.relu(lin(torch.cat([out, a.unsqueeze(0).expand(A, *a.shape)], -1), P["fc2.weight"], P["fc2.bias"]))
    return lin(out, P["fc3.weight"], P["fc3.bias"]), h


def maddpg_rnn_loss(Pc, Ptc, Pa, Pta, states, next_states, actors_states, actors_next_states, actors_action,
                    rewards, done, gamma):
    """SuperAgent.train() losses (MADDPG.py:83-139), summed over agents (each agent's critic owns its own terms).
    Minibatch as get_minibatch returns it (memory_rnn.py:69-99): states / next_states [B,C,N,k], actors_states
    [N,B,C,k], actors_action [N,B,C,2], rewards / done [B,C,N,1]. Returns (sum of critic + actor losses, per-agent
    critic losses [N], per-agent actor losses [N])."""
    B, C, N, k = states.shape
    states = states.reshape(B, C, N * 4)  # MADDPG.py:84-86 (k must be 4)
    next_states = next_states.reshape(B, C, N * 4)
    concat_actors_action = actors_action.reshape(B, C, N * 2)  # the raw reshape of [N,B,C,2] (row mixing)
    z = lambda: torch.zeros((N, B, 32), dtype=states.dtype, device=states.device)  # noqa: E731
    h_ta, h_tc, h_c, h_a = z(), z(), z(), z()
    for t in range(C):
        with torch.no_grad():
            ta, h_ta = rnn_actor(Pta, actors_next_states[:, :, t], h_ta)
            concat_target_actions = ta.transpose(0, 1).reshape(B, 2 * N)            # torch.cat(..., dim=1)
            target_critic_values, h_tc = rnn_critic(Ptc, next_states[:, t], concat_target_actions, h_tc)
        critic_values, h_c = rnn_critic(Pc, states[:, t], concat_actors_action[:, t], h_c)
        pa, h_a = rnn_actor(Pa, actors_states[:, :, t], h_a)
        concat_policy_actions = pa.transpose(0, 1).reshape(B, 2 * N)
        keep = (done[:, t, :, 0] == 0).t().unsqueeze(-1)                             # [N, B, 1]
        h_ta, h_tc = torch.where(keep, h_ta, 0.0), torch.where(keep, h_tc, 0.0)
        h_c, h_a = torch.where(keep, h_c, 0.0), torch.where(keep, h_a, 0.0)
    last = C - 1
    r = rewards[:, last].permute(1, 0, 2)                                            # [N, B, 1]
    d = done[:, last].permute(1, 0, 2)
    targets = r + gamma * target_critic_values * (1 - d)
    critic_losses = ((targets - critic_values) ** 2).mean(dim=(1, 2))               # F.mse_loss per agent
    aq, _ = rnn_critic(Pc, states[:, last].detach(), concat_policy_actions.detach(), h_c)
    actor_losses = -aq.mean(dim=(1, 2))
    return critic_losses.sum() + actor_losses.sum(), critic_losses.detach(), actor_losses.detach()
