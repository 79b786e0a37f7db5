"""torch.classes.flock.ScTrainLoop (csrc/flock_torch_loop.cpp): the config-3 training loop enqueued K steps per C++ call
is bitwise the per-step Python path (VecFlockEnv.step(ring=...) through flock::step_v2_store, then
SharedCriticLearner.pipeline_learn) — env state, replay ring, critic, actors, targets, Adam moments and step counts —
including a call boundary in the middle of the run and the learner's pending actor phase across it."""
import pytest
import torch

from marl_range_flocking_amd import FlockConfig, VecFlockEnv

pytestmark = pytest.mark.gpu
E, N, K = 16, 128, 4


def _bench(cuda):
    from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

    box = float(round((250 * N) ** 0.5))
    env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=K, collision_distance=2.5,
                                  range_start=(0, box), sensor_range=14.0, seed=1, step_launches=2), device=cuda)
    g = torch.Generator(device=cuda).manual_seed(0)
    env.positions.copy_(torch.rand(E, N, 2, device=cuda, generator=g) * box)
    env.headings.copy_((1.0 - torch.rand(E, N, device=cuda, generator=g)) * 4.712389)
    return env, SharedCriticBench(env, device=cuda, seed=3)


def _pool(cuda):
    g = torch.Generator(device=cuda).manual_seed(1)
    return [torch.stack([torch.rand(E, N, device=cuda, generator=g),
                         torch.rand(E, N, device=cuda, generator=g) * 3 - 1.5], -1).contiguous() for _ in range(5)]


def _state(env, hook):
    L = hook.learner
    C, A = L.critic, L.actors
    out = {n: getattr(env, n) for n in ("positions", "headings", "velocities", "dnn", "nn_idx", "reward", "done",
                                        "any_done", "seeds")}
    out.update({f"ring_{n}": v for n, v in L.replay.bufs.items()})
    out.update(critic=C.data, critic_m=C.exp_avg, critic_v=C.exp_avg_sq, critic_step=C.step_dev, actors=A.data,
               actors_target=A.target, actors_m=A.exp_avg, actors_v=A.exp_avg_sq, actor_steps=L.actor_steps,
               losses=L.losses)
    return out


def test_train_loop_is_bitwise_the_per_step_path(cuda):
    pool = _pool(cuda)
    env_a, hook_a = _bench(cuda)
    for s in range(12):
        hook_a.step(s, pool[s % len(pool)])
    hook_a.finish()
    env_b, hook_b = _bench(cuda)
    assert hook_b.can_loop()
    hook_b.run_steps(0, 5, pool)
    hook_b.run_steps(5, 7, pool)
    hook_b.finish()
    torch.cuda.synchronize()
    sa, sb = _state(env_a, hook_a), _state(env_b, hook_b)
    for name in sa:
        assert torch.equal(sa[name], sb[name]), name
    La, Lb = hook_a.learner, hook_b.learner
    assert (La.replay.counter, La._learn_calls, La.count) == (Lb.replay.counter, Lb._learn_calls, Lb.count)
    assert (env_a._cur, env_a.steps) == (env_b._cur, env_b.steps)
    # the Python path continues from the loop's mirrors: one more step each, still equal
    hook_a.step(12, pool[0])
    hook_b.env.step(pool[0], ring=hook_b.before(12))
    torch.cuda.synchronize()
    assert torch.equal(env_a.positions, env_b.positions) and torch.equal(env_a.dnn, env_b.dnn)
    for n in La.replay.bufs:
        assert torch.equal(La.replay.bufs[n], Lb.replay.bufs[n]), n


def test_train_loop_records_timing_events(cuda):
    pool = _pool(cuda)
    env, hook = _bench(cuda)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    hook.run_steps(0, 6, pool, evs, 4)  # steps 0 and 4 are bracketed
    hook.finish()
    torch.cuda.synchronize()
    for a, b in zip(evs[::2], evs[1::2]):
        assert a.elapsed_time(b) > 0
