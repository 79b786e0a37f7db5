"""Overlapped env step / learner (bench.py config 3 hook): learn(s) on its own stream after its minibatch snapshot,
env step s+1 concurrently on the main stream. Every kernel must still see the same data, so after several steps
every parameter, Adam moment, replay field and loss equals the serial loop's bit for bit."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(cuda, overlap, E=64, N=16, k=4, box=63.0):
    from marl_range_flocking_amd import FlockConfig, VecFlockEnv
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

    env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                                  range_start=(0, box), sensor_range=14.0), device=cuda)
    g = torch.Generator(device=cuda).manual_seed(3)
    env.positions.copy_(torch.rand(E, N, 2, device=cuda, generator=g) * box)
    env.headings.copy_(torch.rand(E, N, device=cuda, generator=g) * 4.7)
    hook = SharedCriticBench(env, device=cuda, seed=11, overlap=overlap)
    return env, hook


def test_snapshot_prologue_copies_the_sampled_rows(cuda):
    """flock_sc_prep_snapshot samples the rows flock_sc_prep samples and copies every field of them."""
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner

    a = SharedCriticLearner(8, 4, device=cuda, seed=5, batch_size=64, buffer_size=500, snapshot=True)
    b = SharedCriticLearner(8, 4, device=cuda, seed=5, batch_size=64, buffer_size=500, snapshot=False)
    g = torch.Generator(device=cuda).manual_seed(1)
    n = 300
    rows = (torch.rand(n, 4, device=cuda, generator=g), torch.rand(n, 2, device=cuda, generator=g),
            torch.rand(n, 1, device=cuda, generator=g), torch.rand(n, 4, device=cuda, generator=g),
            torch.rand(n, device=cuda, generator=g) > 0.5)
    for L in (a, b):
        L.store_transitions(*rows)
    a.learn(3)
    b.learn(3)
    torch.cuda.synchronize()
    assert torch.equal(a.static_idx, b.static_idx)
    for name, v in a.staging.items():
        assert torch.equal(v, a.replay.bufs[name][a.static_idx].reshape(v.shape)), name
    for x, y in ((a.critic.data, b.critic.data), (a.actors.data, b.actors.data), (a.losses, b.losses)):
        assert torch.equal(x, y)


@pytest.mark.parametrize("N,steps", [(16, 8), (6, 14)], ids=["distinct-agents", "repeated-agents"])
def test_overlapped_bench_loop_equals_serial(N, steps, cuda):
    """The default overlapped hook runs learn() as a critic phase and an actor phase on two streams, the actor phase
    of learn s beside the critic phase of learn s+1 (update_slot_pipelined). With 6 agents each agent learns 2-3
    times, so soft and non-soft learns (count % 3) alternate in the pipeline."""
    runs = [_pair(cuda, overlap, N=N) for overlap in (False, True)]
    assert runs[1][1].pipelined
    g = torch.Generator(device=cuda).manual_seed(7)
    E, N = runs[0][0].E, runs[0][0].N
    for s in range(steps):
        a = torch.stack([torch.rand(E, N, device=cuda, generator=g),
                         torch.rand(E, N, device=cuda, generator=g) * 3 - 1.5], -1).contiguous()
        for env, hook in runs:
            ring = hook.before(s)
            env.step(a, ring=ring)
            hook.after(s, a)
    for _, hook in runs:
        hook.finish()
    torch.cuda.synchronize()
    (e0, h0), (e1, h1) = runs
    assert h1.overlap and not h0.overlap
    L0, L1 = h0.learner, h1.learner
    assert torch.equal(e0.positions, e1.positions) and torch.equal(e0.dnn, e1.dnn)
    for x, y in ((L0.critic.data, L1.critic.data), (L0.critic.exp_avg, L1.critic.exp_avg),
                 (L0.critic.exp_avg_sq, L1.critic.exp_avg_sq), (L0.actors.data, L1.actors.data),
                 (L0.actors.target, L1.actors.target), (L0.actor_steps, L1.actor_steps), (L0.losses, L1.losses)):
        assert torch.equal(x, y)
    for name in L0.replay.bufs:
        assert torch.equal(L0.replay.bufs[name], L1.replay.bufs[name]), name


def test_pipelined_phases_same_agent_equal_serial(cuda):
    """update_slot_pipelined with the SAME agent learning back to back (its critic phase must wait for the previous
    actor phase, which soft-updates that agent's target actor): bitwise the serial learn() sequence."""
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner

    Ls = [SharedCriticLearner(1, 4, device=cuda, seed=5, batch_size=64, buffer_size=500, snapshot=True)
          for _ in range(2)]
    g = torch.Generator(device=cuda).manual_seed(2)
    n = 300
    rows = (torch.rand(n, 4, device=cuda, generator=g), torch.rand(n, 2, device=cuda, generator=g),
            torch.rand(n, 1, device=cuda, generator=g), torch.rand(n, 4, device=cuda, generator=g),
            torch.rand(n, device=cuda, generator=g) > 0.5)
    for L in Ls:
        L.store_transitions(*rows)
    ser, pip = Ls
    sc, sa = torch.cuda.Stream(device=cuda), torch.cuda.Stream(device=cuda)
    done = [torch.cuda.Event(), torch.cuda.Event()]
    main = torch.cuda.current_stream(cuda)
    for t in range(7):
        ser.learn(0)
        slot = t & 1
        if t >= 2:
            main.wait_event(done[slot])
        assert pip.snapshot_into(slot, 0)
        ev = torch.cuda.Event()
        ev.record(main)
        sc.wait_event(ev)
        if t >= 1:
            sc.wait_event(done[slot ^ 1])  # same agent as the previous learn
        pip.update_slot_pipelined(slot, 0, sc, sa, after_actor=done[slot])
    main.wait_stream(sc)
    main.wait_stream(sa)
    torch.cuda.synchronize()
    for x, y in ((ser.critic.data, pip.critic.data), (ser.critic.exp_avg, pip.critic.exp_avg),
                 (ser.actors.data, pip.actors.data), (ser.actors.target, pip.actors.target),
                 (ser.actor_steps, pip.actor_steps), (ser.critic.step_dev, pip.critic.step_dev)):
        assert torch.equal(x, y)


@pytest.mark.parametrize("agents,n_slots", [((0, 0, 0, 1, 1, 0, 2, 1, 1, 2), 2), ((0, 1, 2, 0, 0, 1, 2, 2, 1, 0), 3),
                                            ((3, 1, 4, 1, 5, 9, 2, 6, 5, 3), 4),
                                            ((3, 1, 4, 1, 5, 9, 2, 6, 5, 3, 5, 8, 9, 7, 9, 3, 2, 3, 8, 4, 6, 6), 8)],
                         ids=["same-agent-runs-2slots", "mixed-3slots", "distinct-4slots",
                              "8slots-sparse-free-events"])
@pytest.mark.parametrize("handoff", ["gate", "event"])
def test_native_pipeline_rounds_equal_serial(agents, n_slots, handoff, cuda):
    """The native pipeline (flock_sc_pipeline_learn): one six-launch round per learn() = its critic phase merged
    with the previous learn's actor phase (flock_sc_round), or the two phases one after the other when both learns
    have the same agent; the last actor phase is enqueued by flock_sc_pipeline_flush. After a sequence with runs of
    the same agent, every parameter, moment, target, step counter and loss is bitwise the serial learn() sequence,
    with either snapshot hand-off (the device-side gate polled by the critic row blocks, or the event wait)."""
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner

    ser = SharedCriticLearner(10, 4, device=cuda, seed=5, batch_size=64, buffer_size=500, snapshot=False)
    pip = SharedCriticLearner(10, 4, device=cuda, seed=5, batch_size=64, buffer_size=500, snapshot=True,
                              n_slots=n_slots, handoff=handoff)
    g = torch.Generator(device=cuda).manual_seed(4)
    n = 300
    rows = (torch.rand(n, 4, device=cuda, generator=g), torch.rand(n, 2, device=cuda, generator=g),
            torch.rand(n, 1, device=cuda, generator=g), torch.rand(n, 4, device=cuda, generator=g),
            torch.rand(n, device=cuda, generator=g) > 0.5)
    for L in (ser, pip):
        L.store_transitions(*rows)
    ls = torch.cuda.Stream(device=cuda)
    main = torch.cuda.current_stream(cuda)
    losses = []
    for i, a in enumerate(agents):
        ser.learn(a)
        losses.append(ser.losses.clone())
        pip.pipeline_mark(main.cuda_stream, wait=i % 3 != 2)  # the gate's guard: an event, or declared bounded
        assert pip.pipeline_learn(a, main.cuda_stream, ls.cuda_stream)
    pip.pipeline_flush(ls.cuda_stream)
    pip.pipeline_flush(ls.cuda_stream)  # nothing pending: a no-op
    main.wait_stream(ls)
    torch.cuda.synchronize()
    pip.pipeline_check()  # no round gave up waiting for its snapshot (device-side gate)
    assert pip.pipeline().gated() == int(handoff == "gate")
    assert pip.pipeline().gated_learns() == (len(agents) if handoff == "gate" else 0)
    for x, y in ((ser.critic.data, pip.critic.data), (ser.critic.exp_avg, pip.critic.exp_avg),
                 (ser.critic.exp_avg_sq, pip.critic.exp_avg_sq), (ser.actors.data, pip.actors.data),
                 (ser.actors.exp_avg, pip.actors.exp_avg), (ser.actors.target, pip.actors.target),
                 (ser.actor_steps, pip.actor_steps), (ser.critic.step_dev, pip.critic.step_dev),
                 (ser.losses, pip.losses)):
        assert torch.equal(x, y)


@pytest.mark.parametrize("n_slots", [2, 3])
@pytest.mark.parametrize("free_events", [0, 1], ids=["slots-freed-on-device", "slot-free-events"])
def test_pipeline_mixed_gated_and_event_learns_equal_serial(n_slots, free_events, cuda):
    """Learns with and without a mark in one pipeline: the gated ones take the device gate, the rest the event
    hand-off, so a slot passes between the two ways of being freed (on the device: the round's sc_gemm stores the
    consumed snapshot's number and the slot's next gated snapshot polls it; by event: a free point on the learner
    stream; and, under flock_set_diag("sc_free_events", 1), every slot by event). Bitwise the serial learns."""
    from marl_range_flocking_amd import _native
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner

    lib = _native.lib()
    agents = (0, 1, 2, 0, 0, 1, 2, 2, 1, 0, 3, 4, 3)
    marks = (1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1, 1, 1)
    g = torch.Generator(device=cuda).manual_seed(6)
    n = 300
    rows = (torch.rand(n, 4, device=cuda, generator=g), torch.rand(n, 2, device=cuda, generator=g),
            torch.rand(n, 1, device=cuda, generator=g), torch.rand(n, 4, device=cuda, generator=g),
            torch.rand(n, device=cuda, generator=g) > 0.5)
    ls = torch.cuda.Stream(device=cuda)
    main = torch.cuda.current_stream(cuda)
    assert lib.flock_set_diag(b"sc_free_events", free_events) == 0
    try:
        ser = SharedCriticLearner(5, 4, device=cuda, seed=5, batch_size=64, buffer_size=500, snapshot=False)
        pip = SharedCriticLearner(5, 4, device=cuda, seed=5, batch_size=64, buffer_size=500, snapshot=True,
                                  n_slots=n_slots)
        for L in (ser, pip):
            L.store_transitions(*rows)
        for a, mk in zip(agents, marks):
            ser.learn(a)
            if mk:
                pip.pipeline_mark(main.cuda_stream)
            assert pip.pipeline_learn(a, main.cuda_stream, ls.cuda_stream)
        pip.pipeline_flush(ls.cuda_stream)
        main.wait_stream(ls)
        torch.cuda.synchronize()
    finally:
        lib.flock_set_diag(b"sc_free_events", 0)
    pip.pipeline_check()
    assert pip.pipeline().gated_learns() == sum(marks)
    for x, y in ((ser.critic.data, pip.critic.data), (ser.critic.exp_avg_sq, pip.critic.exp_avg_sq),
                 (ser.actors.data, pip.actors.data), (ser.actors.target, pip.actors.target),
                 (ser.actor_steps, pip.actor_steps), (ser.losses, pip.losses)):
        assert torch.equal(x, y)


def _sleep_s(seconds):
    """A kernel that holds the current stream for about `seconds` (s_memtime cycles at >= 2.1 GHz)."""
    torch.cuda._sleep(int(2.5e9 * seconds))


@pytest.mark.parametrize("path", ["no-mark", "mark", "loop"])
def test_learn_never_fails_behind_a_busy_env_stream(path, cuda):
    """A learn() must never fail because the env stream is busy (agent_simple_shared_critic.py:115-117: learn() is
    synchronous and never fails): a ~3-s kernel on the env stream ahead of the learns, longer than the gate's 2-s
    bound. Without a mark the learns take the event hand-off; with a mark (wait) behind the sleep, the round first
    waits for the mark on the learner stream (no CU held) and the gate spins only over the env step; the C++ loop
    marks its first learning step the same way. Every case: no error word, bitwise the serial learn() sequence."""
    from marl_range_flocking_amd import FlockConfig, VecFlockEnv
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

    E, Na, steps = 64, 16, 5
    g = torch.Generator(device=cuda).manual_seed(2)
    pool = [torch.stack([torch.rand(E, Na, device=cuda, generator=g),
                         torch.rand(E, Na, device=cuda, generator=g) * 3 - 1.5], -1).contiguous() for _ in range(3)]
    out = []
    for mode in ("serial", path):
        env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=Na, k=4, collision_distance=2.5,
                                      range_start=(0, 63.0), sensor_range=14.0), device=cuda)
        gp = torch.Generator(device=cuda).manual_seed(5)
        env.positions.copy_(torch.rand(E, Na, 2, device=cuda, generator=gp) * 63.0)
        env.headings.copy_(torch.rand(E, Na, device=cuda, generator=gp) * 4.7)
        hook = SharedCriticBench(env, device=cuda, seed=7, overlap=mode != "serial", buffer_size=2000)
        L = hook.learner
        main = torch.cuda.current_stream(cuda)
        # the ring holds a batch before the timed steps (one env step of 64 x 16 transitions)
        env.step(pool[0], ring=L.replay_slots(E * Na))
        torch.cuda.synchronize()
        if mode == "loop":
            _sleep_s(3.0)
            hook.run_steps(1, steps, pool)
        else:
            for s in range(1, 1 + steps):
                if mode == "serial":
                    hook.step(s, pool[s % 3])
                    continue
                ring = L.replay_slots(E * Na)
                if s == 2:
                    _sleep_s(3.0)  # foreign work on the env stream between two learns
                if mode == "mark":
                    L.pipeline_mark(main.cuda_stream)  # behind the sleep
                env.step(pool[s % 3], ring=ring)
                hook.after(s, pool[s % 3])
        hook.finish()
        torch.cuda.synchronize()
        if mode != "serial":
            L.pipeline_check()  # no error word
            gl = L.pipeline().gated_learns()
            assert gl == (0 if mode == "no-mark" else steps), gl
        C, A = L.critic, L.actors
        out.append([C.data.clone(), C.exp_avg_sq.clone(), A.data.clone(), A.target.clone(), L.actor_steps.clone(),
                    L.losses.clone(), env.positions.clone()])
    for i, (x, y) in enumerate(zip(*out)):
        assert torch.equal(x, y), i


def test_specialised_row_kernels_equal_generic(cuda):
    """At the reference widths (fc1 400, fc2 300, 2 actions) the rounds run row kernels with compile-time widths;
    flock_set_diag("sc_no_spec", 1) forces the generic ones. Merged rounds of both are bitwise equal."""
    from marl_range_flocking_amd import _native
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner

    lib = _native.lib()
    g = torch.Generator(device=cuda).manual_seed(9)
    n, d = 600, 20
    rows = (torch.rand(n, d, device=cuda, generator=g), torch.rand(n, 2, device=cuda, generator=g) * 2 - 1,
            torch.rand(n, 1, device=cuda, generator=g), torch.rand(n, d, device=cuda, generator=g),
            torch.rand(n, device=cuda, generator=g) > 0.8)
    ls = torch.cuda.Stream(device=cuda)
    main = torch.cuda.current_stream(cuda)
    out = []
    for no_spec in (0, 1):
        L = SharedCriticLearner(6, d, device=cuda, seed=3, batch_size=256, buffer_size=1000, snapshot=True,
                                n_slots=3)
        L.store_transitions(*rows)
        assert lib.flock_set_diag(b"sc_no_spec", no_spec) == 0
        try:
            for a in (0, 3, 3, 1, 5, 2, 0):
                assert L.pipeline_learn(a, main.cuda_stream, ls.cuda_stream)
            L.pipeline_flush(ls.cuda_stream)
            main.wait_stream(ls)
            torch.cuda.synchronize()
        finally:
            lib.flock_set_diag(b"sc_no_spec", 0)
        out.append(L)
    a, b = out
    for x, y in ((a.critic.data, b.critic.data), (a.critic.exp_avg_sq, b.critic.exp_avg_sq),
                 (a.actors.data, b.actors.data), (a.actors.target, b.actors.target), (a.losses, b.losses)):
        assert torch.equal(x, y)
    assert torch.isfinite(a.critic.data).all() and a.losses.abs().sum() > 0


@pytest.mark.parametrize("n_slots", [2, 3, 8])
def test_device_gate_is_bitwise_the_event_wait(n_slots, cuda):
    """The device-side snapshot gate (the critic row blocks poll a sequence number the `sc1` snapshot publishes, then
    read the staged rows `sc1`) against the cross-queue event wait, in the overlapped config-3 loop at the reference
    widths with env kernels co-running on the env stream (uneven load, L1-warm consumers): every learner tensor ends
    bitwise equal (the event loop runs twice: a determinism baseline), and no wait gave up."""
    from marl_range_flocking_amd import FlockConfig, VecFlockEnv
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

    E, Na, steps = 512, 256, 24
    g = torch.Generator(device=cuda).manual_seed(2)
    pool = [torch.stack([torch.rand(E, Na, device=cuda, generator=g),
                         torch.rand(E, Na, device=cuda, generator=g) * 3 - 1.5], -1).contiguous() for _ in range(3)]
    out = []
    modes = ("event", "event", "gate", "gate")
    for handoff in modes:
        env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=Na, k=4, collision_distance=2.5,
                                      range_start=(0, 253.0), sensor_range=14.0, step_launches=3), device=cuda)
        gp = torch.Generator(device=cuda).manual_seed(5)
        env.positions.copy_(torch.rand(E, Na, 2, device=cuda, generator=gp) * 253.0)
        env.headings.copy_(torch.rand(E, Na, device=cuda, generator=gp) * 4.7)
        hook = SharedCriticBench(env, device=cuda, seed=7, n_slots=n_slots, handoff=handoff)
        hook.run_steps(0, steps, pool)
        hook.finish()
        torch.cuda.synchronize()
        L = hook.learner
        L.pipeline_check()
        assert L.pipeline().gated() == int(handoff == "gate")
        C, A = L.critic, L.actors
        out.append([C.data.clone(), C.exp_avg.clone(), C.exp_avg_sq.clone(), A.data.clone(), A.target.clone(),
                    A.exp_avg.clone(), A.exp_avg_sq.clone(), L.actor_steps.clone(), L.losses.clone(),
                    C.step_dev.clone()])
    bad = {}
    for m, mode in enumerate(out[1:], 1):
        diff = [i for i, (x, y) in enumerate(zip(out[0], mode)) if not torch.equal(x, y)]
        if diff:
            bad[(m, modes[m])] = (diff, float((out[0][0] - mode[0]).abs().max()))
    assert not bad, bad  # (run, hand-off) -> (differing tensors, max |critic diff|)
