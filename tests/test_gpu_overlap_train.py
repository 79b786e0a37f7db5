"""Configs 4 / 5: train() on its own stream beside the env steps that follow it (learners/core.py OverlappedTrain;
bench.py VDNBench / MADDPGBench). The overlapped update must be bitwise the in-line train() on the same draws, even
when the ring rows it sampled are overwritten right after the call (the snapshot is taken on the caller's stream
before anything later runs): RNN-MADDPG SuperAgent.train() (learners/maddpg_official_rnn/MADDPG.py:78-150) and VDN
train() (learners/vdn/train_flock.py:16-43)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _maddpg(cuda, seed=3):
    from marl_range_flocking_amd.learners.maddpg import MADDPGLearner

    return MADDPGLearner(16, 4, recurrent=True, hidden1=32, hidden2=24, batch_size=16, chunk_size=4,
                         buffer_capacity=400, min_size_buffer=16, device=cuda, seed=seed, shared_obs=True)


def _maddpg_records(L, g, E, cuda):
    N, k = L.N, L.k
    obs, nxt = torch.rand(E, N, k, device=cuda, generator=g), torch.rand(E, N, k, device=cuda, generator=g)
    act = torch.rand(E, N, 2, device=cuda, generator=g)
    rew, done = torch.rand(E, N, device=cuda, generator=g), (torch.rand(E, N, device=cuda, generator=g) < 0.1).float()
    L.add_record(obs, nxt, act, obs, nxt, rew, done)


def test_maddpg_overlapped_train_is_bitwise_train(cuda):
    out = []
    for overlapped in (False, True):
        L = _maddpg(cuda)
        g = torch.Generator(device=cuda).manual_seed(11)
        for _ in range(6):
            _maddpg_records(L, g, 50, cuda)
        for rep in range(3):
            loss = L.train_overlapped() if overlapped else L.train()
            for _ in range(3):  # the env steps that follow overwrite ring rows (the ring wraps every 8 calls)
                _maddpg_records(L, g, 50, cuda)
        if overlapped:
            assert L._ov.pending
            L.sync()
        torch.cuda.synchronize()
        out.append((L, loss.clone()))
    (a, la), (b, lb) = out
    assert torch.equal(la, lb)
    for x, y in ((a.critics.data, b.critics.data), (a.critics.target, b.critics.target),
                 (a.critics.exp_avg, b.critics.exp_avg), (a.critics.exp_avg_sq, b.critics.exp_avg_sq),
                 (a.actors.target, b.actors.target), (a.actors.data, b.actors.data)):
        assert torch.equal(x, y)
    for name in a.replay.bufs:
        assert torch.equal(a.replay.bufs[name], b.replay.bufs[name]), name


def _vdn(cuda, seed=5):
    from marl_range_flocking_amd.learners.vdn import VDNLearner

    return VDNLearner(8, 4, 5, batch_size=8, chunk_size=4, update_iter=3, buffer_limit=300, device=cuda, seed=seed)


def _vdn_put(L, g, E, cuda):
    A = L.A
    s, s2 = torch.rand(E, A, L.n_obs, device=cuda, generator=g), torch.rand(E, A, L.n_obs, device=cuda, generator=g)
    a = torch.randint(0, L.n_actions, (E, A), device=cuda, generator=g)
    r = torch.rand(E, A, device=cuda, generator=g)
    done = (torch.rand(E, device=cuda, generator=g) < 0.1).float()
    L.put(s, a, r, s2, done)


def test_vdn_overlapped_train_is_bitwise_train(cuda):
    out = []
    for overlapped in (False, True):
        L = _vdn(cuda)
        g = torch.Generator(device=cuda).manual_seed(17)
        for _ in range(5):
            _vdn_put(L, g, 60, cuda)
        for rep in range(3):
            loss = L.train_overlapped() if overlapped else L.train()
            for _ in range(3):  # ring rows overwritten right after the call (300 rows: wraps every 5 puts)
                _vdn_put(L, g, 60, cuda)
        L.sync() if overlapped else None
        torch.cuda.synchronize()
        out.append((L, loss.clone()))
    (a, la), (b, lb) = out
    assert torch.equal(la, lb)
    P, Q = a.q.P, b.q.P
    for x, y in ((P.data, Q.data), (P.target, Q.target), (P.exp_avg, Q.exp_avg), (P.exp_avg_sq, Q.exp_avg_sq)):
        assert torch.equal(x, y)


def _delay_current_stream(cuda):
    """Queue ~10 ms of work on the current stream so that a missing cross-stream wait would show as a race."""
    x = torch.rand(2048, 2048, device=cuda)
    for _ in range(8):
        x = x @ x / 2048.0
    return x


def test_maddpg_mixed_paths_are_bitwise_serial(cuda):
    """train() and get_actions() / state_dict() right after train_overlapped() wait for the overlapped update
    (FlatParams.sync_writers): the results equal serial train() calls on the same draws."""
    out = []
    for mixed in (False, True):
        L = _maddpg(cuda)
        g = torch.Generator(device=cuda).manual_seed(23)
        for _ in range(6):
            _maddpg_records(L, g, 50, cuda)
        acts = []
        for rep in range(3):
            if mixed and rep % 2 == 0:
                if "_ov" in L.__dict__:  # the overlapped update then starts ~10 ms late on its stream
                    with torch.cuda.stream(L._ov.stream):
                        _delay_current_stream(cuda)
                L.train_overlapped()
            else:
                L.train()
            x = torch.rand(4, L.N, L.k, device=cuda, generator=g)
            acts.append(L.get_actions(x, test=True)[0].clone())
            sd = L.state_dict("critic", 0)
            _maddpg_records(L, g, 50, cuda)
        loss = L.train().clone()
        torch.cuda.synchronize()
        out.append((L, loss, acts, sd))
    (a, la, aa, sa), (b, lb, ab, sb) = out
    assert torch.equal(la, lb)
    for x, y in zip(aa, ab):
        assert torch.equal(x, y)
    for n in sa:
        assert torch.equal(sa[n], sb[n]), n
    for x, y in ((a.critics.data, b.critics.data), (a.critics.exp_avg_sq, b.critics.exp_avg_sq),
                 (a.actors.target, b.actors.target)):
        assert torch.equal(x, y)


def test_vdn_mixed_paths_are_bitwise_serial(cuda):
    """VDN: train(), sync_target(), the q network's forward and state_dict() right after train_overlapped() wait for
    the overlapped update; bitwise serial train() calls on the same draws."""
    out = []
    for mixed in (False, True):
        L = _vdn(cuda)
        g = torch.Generator(device=cuda).manual_seed(29)
        for _ in range(5):
            _vdn_put(L, g, 60, cuda)
        qs = []
        for rep in range(3):
            if mixed and rep % 2 == 0:
                if "_ov" in L.__dict__:  # the overlapped update then starts ~10 ms late on its stream
                    with torch.cuda.stream(L._ov.stream):
                        _delay_current_stream(cuda)
                L.train_overlapped()
            else:
                L.train()
            obs = torch.rand(4, L.A, L.n_obs, device=cuda, generator=g)
            qs.append(L.q(obs, L.q.init_hidden(4))[0].clone())
            if rep == 1:
                L.sync_target()
            sd = L.q.state_dict()
            _vdn_put(L, g, 60, cuda)
        loss = L.train().clone()
        torch.cuda.synchronize()
        out.append((L, loss, qs, sd))
    (a, la, qa, sa), (b, lb, qb, sb) = out
    assert torch.equal(la, lb)
    for x, y in zip(qa, qb):
        assert torch.equal(x, y)
    for n in sa:
        assert torch.equal(sa[n], sb[n]), n
    P, Q = a.q.P, b.q.P
    for x, y in ((P.data, Q.data), (P.target, Q.target), (P.exp_avg_sq, Q.exp_avg_sq)):
        assert torch.equal(x, y)
