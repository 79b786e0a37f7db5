"""Generate golden env fixtures by running the REFERENCE environments on CPU (torch) with injected state.

Run here (build container) only:  ``python tests/golden/gen_golden_env.py``  → ``tests/golden/env_*.npz``.
The reference never travels to the GPU box; the fixtures (inputs + the reference's outputs) do.

Each fixture holds E independent reference env instances stepped T times with injected actions (and, for
``gym_flock_uw_discrete``, injected Gaussian noise: ``torch.normal`` is patched to return ``mean + noise``, which is
the reference's own arithmetic ``normal_(0, std).add_(mean)``). Outputs are recorded after every step.

Reference entry points exercised (paths relative to /root/reference):
  v2       environments/gym_flock_v2.py:71-83  (step: _updateState :317, check_boundary :271,
           _computePeriodicDistances :135, _computeCollisions :212, _computeObs :127, _computeDone :306,
           _computeReward :252)
  v2fork   learners/maddpg_official_rnn/gym_flock_v2.py:71-82 (Euclidean _computeDistances, v_min 0.5 :310)
  uw       environments/gym_flock_uw.py:69-81
  uwd      environments/gym_flock_uw_discrete.py:110-122
  flock    environments/gym_flock.py:48-60
  sense    _computePeriodicDistances / _computeDistances on injected positions (incl. lattice ties)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refshim  # noqa: E402

OUT = HERE


def _meta(**kw):
    import torch

    kw.update(torch=torch.__version__, numpy=np.__version__, generator="tests/golden/gen_golden_env.py",
              reference_pins="torch==1.13.1+cu117 (requirements.txt:5); run here on torch CPU")
    return json.dumps(kw)


def _mods():
    refshim.install()
    return {
        "v2": refshim.load("environments/gym_flock_v2.py", "ref_gym_flock_v2"),
        "v2fork": refshim.load("learners/maddpg_official_rnn/gym_flock_v2.py", "ref_gym_flock_v2_fork"),
        "uw": refshim.load("environments/gym_flock_uw.py", "ref_gym_flock_uw"),
        "uwd": refshim.load("environments/gym_flock_uw_discrete.py", "ref_gym_flock_uw_discrete"),
        "flock": refshim.load("environments/gym_flock.py", "ref_gym_flock"),
    }


def _boundary_rows(rng, pos, head, box, variant):
    """Put a few agents right at the teleport seams (gym_flock_v2.py:292-304)."""
    n = pos.shape[0]
    if n < 8:
        return
    pos[0] = [box - 1e-3, box * 0.5]
    pos[1] = [1e-3, box * 0.25]
    pos[2] = [box * 0.75, box - 5e-4]
    pos[3] = [box * 0.33, 2e-4]
    if head is not None:
        head[0] = 0.0
        head[1] = np.float32(np.pi)
        head[2] = np.float32(np.pi / 2)
        head[3] = np.float32(-np.pi / 2)


def gen_traj(mods, variant, N, k, E, T, box, cd=2.5, sr=14.0, seed=0, tag="", normalize=False):
    import torch

    rng = np.random.default_rng(seed)
    mod = mods[variant]
    pos0 = rng.uniform(0.0, box, size=(E, N, 2)).astype(np.float32)
    if variant in ("v2", "v2fork"):
        head0 = rng.uniform(0.0, 1.5 * np.pi, size=(E, N)).astype(np.float32)
    elif variant == "uw":
        head0 = rng.uniform(0.0, 2 * np.pi, size=(E, N)).astype(np.float32)
    elif variant == "uwd":
        head0 = rng.uniform(0.0, np.pi / 1.2, size=(E, N)).astype(np.float32)
    else:
        head0 = np.zeros((E, N), np.float32)
    for e in range(E):
        _boundary_rows(rng, pos0[e], head0[e], box, variant)
    prevh0 = np.zeros((E, N), np.float32)
    mem0 = np.zeros((E, N, 4, k), np.float32)
    if variant == "uw":
        mem0 = rng.uniform(0.0, sr, size=(E, N, 4, k)).astype(np.float32)
    vel0 = np.zeros((E, N, 2), np.float32)

    if variant in ("v2", "v2fork"):
        act = np.stack([rng.uniform(-0.5, 3.0, size=(T, E, N)), rng.uniform(-2.5, 2.5, size=(T, E, N))], -1)
        act = act.astype(np.float32)
        if N >= 8:
            act[:, :, 0, 0] = 2.5
            act[:, :, 0, 1] = 0.0
            act[:, :, 1, 0] = 2.5
            act[:, :, 1, 1] = 0.0
    elif variant in ("uw", "flock"):
        act = rng.uniform(-1.0, 1.0, size=(T, E, N, 2)).astype(np.float32)
        if variant == "uw" and N >= 8:
            act[:, :, 4] = 0.0  # zero action → 0/0 → nan_to_num → 0 (gym_flock_uw.py:294-298)
            act[:, :, 0] = [1.0, 0.0]
            act[:, :, 1] = [-1.0, 0.0]
    else:  # uwd: integer actions into the 10-entry dictionary (gym_flock_uw_discrete.py:59-75)
        act = rng.integers(0, 10, size=(T, E, N)).astype(np.int64)
    noise = (0.1 * rng.standard_normal(size=(T, E, N, 2))).astype(np.float32)

    rec = {k_: [] for k_ in ("pos", "head", "vel", "dnn", "nn_idx", "reward", "done", "any_done", "obs", "prevh")}
    orig_normal = torch.normal
    for e in range(E):
        env_kw = dict(agents=N, k=k, collision_distance=cd, range_start=(0, box))
        if normalize:  # _computeDistances on positions / max |p| (gym_flock_uw.py:127-133 and siblings)
            env_kw["normalize_distance"] = True
        if variant != "flock":
            env_kw["sensor_range"] = sr
        env = mod.MultiAgentEnv(**env_kw)
        env.positions = torch.tensor(pos0[e].copy())
        env.velocities = torch.tensor(vel0[e].copy())
        if variant != "flock":
            env.headings = torch.tensor(head0[e].copy())
            env.prev_headings = torch.tensor(prevh0[e].copy())
        if variant in ("uw", "flock"):
            env.observation_memory = torch.tensor(mem0[e].copy())
        per = {k_: [] for k_ in rec}
        for t in range(T):
            if variant == "uwd":
                calls = {"i": 0}
                nz = torch.tensor(noise[t, e])

                def fake_normal(mean, std, _nz=nz, _calls=calls):
                    assert abs(std - 0.1) < 1e-12
                    col = _calls["i"]
                    _calls["i"] += 1
                    return mean + _nz[:, col]

                torch.normal = fake_normal
                a = torch.tensor(act[t, e]).float()  # VDN passes float action ids (learners/vdn/train_flock.py:99)
            else:
                a = torch.tensor(act[t, e])
            try:
                obs, reward, dones, _ = env.step(a)
            finally:
                torch.normal = orig_normal
            per["pos"].append(env.positions.numpy().copy())
            per["vel"].append(env.velocities.numpy().copy())
            per["head"].append(env.headings.numpy().copy() if variant != "flock" else np.zeros(N, np.float32))
            per["dnn"].append(env.distances_to_nearest_neighbors.numpy().copy())
            nn = getattr(env, "nearest_neighbors", None)
            per["nn_idx"].append(nn.numpy().copy() if nn is not None else np.full((N, k), -1, np.int64))
            per["reward"].append(reward.reshape(-1).numpy().astype(np.float32).copy())
            per["done"].append(dones[0].numpy().copy())
            per["any_done"].append(bool(dones[1]))
            if isinstance(obs, dict):
                assert np.array_equal(obs["critic"].numpy(), obs["actors"].numpy())
                per["obs"].append(obs["actors"].numpy().copy())
            else:
                per["obs"].append(obs.numpy().copy())
            ph = getattr(env, "prev_headings", None)
            per["prevh"].append(ph.numpy().copy() if ph is not None else np.zeros(N, np.float32))
        for k_ in rec:
            rec[k_].append(np.stack([np.asarray(x) for x in per[k_]]))
    out = {k_: np.stack(v, axis=1) for k_, v in rec.items()}  # [T, E, ...]
    v_min = {"v2": 0.005, "v2fork": 0.5}.get(variant, 5e-6)
    name = f"env_{variant}_N{N}_k{k}{tag}.npz"
    np.savez_compressed(
        os.path.join(OUT, name),
        meta=np.array(_meta(variant=variant, N=N, k=k, E=E, T=T, box=box, collision_distance=cd,
                            sensor_range=sr, dt=0.1, v_min=v_min, seed=seed, normalize_distance=normalize)),
        pos0=pos0, head0=head0, prevh0=prevh0, mem0=mem0, vel0=vel0, actions=act, noise=noise,
        **out,
    )
    print("wrote", name, {k_: v.shape for k_, v in out.items()})


def gen_sense(mods, N, k, E, box, sr=14.0, seed=0, lattice=False, tag=""):
    """kNN only: reference _computePeriodicDistances (gym_flock_v2.py:135-151) and _computeDistances (:155-175)."""
    import torch

    rng = np.random.default_rng(seed)
    if lattice:
        side = int(np.ceil(np.sqrt(N)))
        g = np.stack(np.meshgrid(np.arange(side), np.arange(side), indexing="ij"), -1).reshape(-1, 2)[:N]
        pos = np.broadcast_to((g * (box / side) + 0.5).astype(np.float32), (E, N, 2)).copy()
    else:
        pos = rng.uniform(0.0, box, size=(E, N, 2)).astype(np.float32)
    res = {f"{m}_{o}": [] for m in ("per", "euc") for o in ("dnn", "idx", "D")}
    for e in range(E):
        env = mods["v2"].MultiAgentEnv(agents=N, k=k, collision_distance=2.5, range_start=(0, box), sensor_range=sr)
        env.positions = torch.tensor(pos[e].copy())
        env._computePeriodicDistances()
        res["per_dnn"].append(env.distances_to_nearest_neighbors.numpy().copy())
        res["per_idx"].append(env.nearest_neighbors.numpy().copy())
        res["per_D"].append(env.distances.numpy().copy())
        env._computeDistances()
        res["euc_dnn"].append(env.distances_to_nearest_neighbors.numpy().copy())
        res["euc_idx"].append(env.nearest_neighbors.numpy().copy())
        res["euc_D"].append(env.distances.numpy().copy())
    name = f"sense_N{N}_k{k}{tag}.npz"
    np.savez_compressed(os.path.join(OUT, name),
                        meta=np.array(_meta(kind="sense", N=N, k=k, E=E, box=box, sensor_range=sr,
                                            lattice=lattice, seed=seed)),
                        pos=pos, **{k_: np.stack(v) for k_, v in res.items() if N <= 64 or not k_.endswith("_D")})
    print("wrote", name)


def gen_errors(mods):
    """k+1 > N: the reference's topk raises RuntimeError (gym_flock_v2.py:147)."""
    import torch

    env = mods["v2"].MultiAgentEnv(agents=4, k=4, collision_distance=1.0, range_start=(0, 10), sensor_range=7)
    env.positions = torch.rand(4, 2) * 10
    try:
        env._computePeriodicDistances()
        msg = ""
    except RuntimeError as ex:
        msg = str(ex)
    with open(os.path.join(OUT, "errors.json"), "w") as f:
        json.dump({"k_plus_1_gt_N": {"N": 4, "k": 4, "raises": "RuntimeError", "message": msg}}, f, indent=1)
    print("errors:", msg)


def gen_normalized(mods):
    """normalize_distance=True (the Euclidean steps: uw, uw_discrete, gym_flock, the RNN fork of v2). Collision
    distances are in normalised units (distances are <= 2 there)."""
    gen_traj(mods, "uw", N=16, k=4, E=2, T=4, box=45, cd=0.05, seed=30, tag="_norm", normalize=True)
    gen_traj(mods, "uwd", N=16, k=4, E=2, T=4, box=45, cd=0.05, seed=31, tag="_norm", normalize=True)
    gen_traj(mods, "flock", N=16, k=4, E=2, T=4, box=45, cd=0.05, seed=32, tag="_norm", normalize=True)
    gen_traj(mods, "v2fork", N=64, k=4, E=2, T=3, box=126, cd=0.02, seed=33, tag="_norm", normalize=True)


def main():
    if not refshim.available():
        print("reference not present; nothing to do")
        return
    mods = _mods()
    if "--normalized" in sys.argv:  # only the normalize_distance fixtures
        gen_normalized(mods)
        return
    # config-1-like plumbing + long trajectories
    gen_traj(mods, "flock", N=8, k=4, E=3, T=20, box=45, seed=1)
    gen_traj(mods, "v2", N=8, k=4, E=3, T=20, box=45, seed=2)
    gen_traj(mods, "uw", N=8, k=4, E=3, T=20, box=45, seed=3)
    gen_traj(mods, "uwd", N=8, k=4, E=3, T=20, box=45, seed=4)
    # config-sized agents, short trajectories
    gen_traj(mods, "v2", N=64, k=4, E=2, T=5, box=126, seed=5)
    gen_traj(mods, "v2", N=256, k=4, E=2, T=3, box=253, seed=6)
    gen_traj(mods, "v2fork", N=64, k=4, E=2, T=5, box=126, seed=7)
    gen_traj(mods, "uw", N=64, k=4, E=2, T=5, box=126, seed=8)
    gen_traj(mods, "uwd", N=64, k=4, E=2, T=5, box=126, seed=9)
    gen_traj(mods, "uwd", N=512, k=4, E=1, T=2, box=358, seed=10)
    gen_traj(mods, "flock", N=64, k=4, E=2, T=5, box=126, seed=11)
    # edge cases: N = k+1, dense swarm (many collisions), k != 4
    gen_traj(mods, "v2", N=5, k=4, E=2, T=3, box=10, seed=12, tag="_edge")
    gen_traj(mods, "v2", N=16, k=2, E=2, T=4, box=10, cd=1.0, seed=13, tag="_dense")
    gen_traj(mods, "uw", N=16, k=9, E=1, T=3, box=20, seed=14, tag="_k9")
    # sensing only
    gen_sense(mods, N=64, k=4, E=2, box=126, seed=20)
    gen_sense(mods, N=64, k=4, E=1, box=64, seed=21, lattice=True, tag="_lattice")
    gen_sense(mods, N=256, k=4, E=1, box=253, seed=22)
    gen_errors(mods)
    gen_normalized(mods)


if __name__ == "__main__":
    main()
