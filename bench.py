"""Headline benchmark: agent-steps/sec, gym_flock_v2 (periodic) 256 agents x 4096 envs per MI355X (BASELINE config 3).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config {2,3,4,5}]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

One process per GPU. Envs are independent, so each rank steps its own 4096 envs with no data-path collective
(weak scaling); the only collectives are the barrier around the timed region and the max-over-ranks of its time.
A "step" = one vectorized env step of all the rank's envs (kinematics, boundary, sensing, kNN obs, collision,
reward, done: one HIP launch) plus the config's learner: config 3 (default) inserts every transition into the
shared-critic replay ring inside that same launch and runs one learn() (B=256); configs 4 / 5 insert every env's
transition and run VDN / RNN-MADDPG train() every 150 / 250 steps. Inputs (state, a pool of synthetic actions)
are resident in HBM before the timed region starts; the first update (graph capture) happens before it.

Rank 0 prints ONE JSON line. Extra fields:
  roofline      the env step kernel (the dominant kernel), timed with HIP events on its launch stream.
                HBM side: achieved = algorithmic bytes per agent-step (v2 93, uw 149,
                uw_discrete 69) x agent-steps per launch / kernel time, frac = achieved / 8 TB/s; the fused replay
                insert's bytes are reported beside it (insert_bytes_per_agent_step), not in frac; traffic = measured
                HBM bytes per launch (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE, profiles/pmc_*.json).
                VALU side (profiles/pmc_valu_*.json, profiles/ubench_valu.json): gfx950 co-issues the simple VALU ops
                (f32 add/sub/mul/fma, v_mov_b32, v_add_u32, v_and_b32) of two waves in one quad-cycle (2 cycles per
                wave64 instruction) and issues the rest in 4 (min/max/med3, compares, packed f32, 64-bit, 3-operand
                integer ops) or 8 cycles (transcendental); SQ_ACTIVE_INST_VALU charges every instruction its
                quad-cycles and SQ_ACTIVE_INST_VALU2 counts the co-issued pairs, so the step's VALU issue time per
                SIMD is busy = 4 x (ACT - ACT2) / 1024 SIMDs cycles (a saturating ubench stream of any class reads
                0.86-0.97 of its wall cycles on this measure). frac = busy / (kernel time x 2.4 GHz); peak = the
                lane-op rate of this instruction mix with every SIMD issuing every cycle at 2.4 GHz
                (64 x SQ_INSTS_VALU x 2.4e9 / busy); frac_full_rate = against 78.6 T lane-op/s (every instruction
                co-issued). "binding" names the larger of the HBM and VALU fractions (measured alone when the
                line has an alone measurement), or "latency" when neither reaches half of its peak.
  cpu_baseline  the reference's step on the host: v2 = environments/gym_flock_v2.py's torch-CPU op sequence
                (oracle/torch_ref.py, calibrated against the reference, tests/golden/cpu_calibration.json) stepping
                one env at a time on every host CPU this process may use (sched_getaffinity, capped by the cgroup
                CPU quota) and on 1 thread; other variants the C oracle port; a bounded sample; N=1 only.
Configs 4 and 5 are 8-GPU configs: their GLOBAL env count (8192 / 16384) is split over the ranks (strong scaling);
config 3 (the headline) keeps 4096 envs per GPU (weak scaling).
"""
import argparse
import ctypes
import json
import os
import time

import numpy as np
import torch

HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
CLOCK_HZ = 2.4e9                 # MI355X peak engine clock (MI355X_MICROARCH.md); the roofline's clock
SIMDS = 1024                     # 256 CU x 4 SIMD
MFMA_F32_PEAK = 157.3e12         # MI355X_MICROARCH.md: dense f32 matrix peak (v_mfma_f32_*)
VALU_PEAK_FULL_RATE = 64 * SIMDS * CLOCK_HZ / 2  # 78.6e12 lane-op/s: every wave64 instruction co-issued (2 cycles)
BYTES_PER_AGENT_STEP = {"v2": 93, "uw": 149, "uw_discrete": 69, "flock": 129}  # SURVEY §8(d) (flock: +vel rw)
# fused replay insert (flock_step_v2_store / the uw_discrete ring), per agent-step: + previous obs read (k=4 floats)
# + the ring fields written. shared critic: state 16 + action 8 + reward 4 + new_state 16 + terminal 4; RNN-MADDPG
# record: state, next_state 16 each (actor_state / actor_next_state alias them: MADDPGLearner(shared_obs=True)) +
# action 8 + reward 4 + done 4; VDN team transition: s 16 + a (f32 id) 4 + r 4 + s' 16 (+ one done flag per env: 4 / N)
RING_BYTES_PER_AGENT_STEP = {"shared_critic": 16 + 48, "maddpg_rnn": 16 + 48, "vdn": 16 + 40}
# the uw rollout kernel's HBM bytes per agent-step (state on chip): action 8 r + observation memory 64 w + reward 4 w +
# done 1 w (+ any_done per env, and the state once per launch)
ROLLOUT_MOVED_BYTES = 8 + 64 + 4 + 1
# steps between HIP-event-timed env launches in the timed region: each timed step adds two marker packets to the env
# stream (every 4th step: driver command 0.0855-0.0860 ms per step, every 16th 0.0838-0.0848; profiles/r06/ev/)
EV_EVERY = int(os.environ.get("FLOCK_BENCH_EV_EVERY", 16))


class DevEvent:
    """A timing event whose record is a DEVICE-scope release (hipEventReleaseToDevice). torch.cuda.Event records a
    system-scope fence (an L2 writeback + invalidation on this GPU) each time: inside the timed region that would
    perturb the very kernels it times. Same interface as torch.cuda.Event for what bench.py uses (record, elapsed_time,
    cuda_event)."""
    _hip = None

    def __init__(self):
        import ctypes

        if DevEvent._hip is None:
            DevEvent._hip = ctypes.CDLL("libamdhip64.so")
        self._ct = ctypes
        h = ctypes.c_void_p()
        assert DevEvent._hip.hipEventCreateWithFlags(ctypes.byref(h), ctypes.c_uint(0x40000000)) == 0
        self.cuda_event = h.value

    def record(self, stream=None):
        s = (stream or torch.cuda.current_stream()).cuda_stream
        assert DevEvent._hip.hipEventRecord(self._ct.c_void_p(self.cuda_event), self._ct.c_void_p(s)) == 0

    def elapsed_time(self, end):
        ms = self._ct.c_float()
        assert DevEvent._hip.hipEventElapsedTime(self._ct.byref(ms), self._ct.c_void_p(self.cuda_event),
                                                 self._ct.c_void_p(end.cuda_event)) == 0
        return ms.value


def binding(valu, hbm_frac, alone_ms, alg_bytes):
    """The roofline the env kernel is closest to (fractions of the kernel alone when measured, else in the loop);
    "latency" when neither HBM nor VALU issue reaches half of its peak."""
    h = alg_bytes / (alone_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if alone_ms else hbm_frac
    v = (valu["frac_alone"] if alone_ms and valu.get("frac_alone") is not None else valu["frac"]) if valu else 0.0
    name, f = ("valu", v) if v > h else ("hbm", h)
    return name if f >= 0.5 else "latency"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: 200; configs 4/5: 300/500, "
                                                                 "a multiple of the training cadence)")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: the config's; configs 4 / 5: "
                                                         "their global env count / world size)")
    ap.add_argument("--agents", type=int, default=None)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--variant", default=None, choices=["v2", "uw", "uw_discrete", "flock"])
    ap.add_argument("--learner", default=None, choices=["none", "shared_critic", "vdn", "maddpg_rnn"],
                    help="default: the config's learner (config 3: shared_critic)")
    ap.add_argument("--config", type=int, default=3, choices=[2, 3, 4, 5],
                    help="BASELINE.json config: 2 uw 64x1024 env only; 3 v2 256x4096 per GPU + shared critic "
                         "(default); 4 uw_discrete 512x8192 (global, split over the ranks) + VDN every 150 steps; "
                         "5 v2 1024x16384 (global) + RNN-MADDPG every 250 steps. --envs/--agents/--variant/--learner "
                         "override it")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc", default=None, help="JSON with measured HBM bytes per launch (profiles/)")
    ap.add_argument("--step-launches", type=int, default=None,
                    help="env step as this many launches over env ranges (FlockConfig.step_launches; default: 3 "
                         "with the overlapped shared-critic learner, whose rounds take the slots each launch's "
                         "tail frees; 1 otherwise)")
    ap.add_argument("--loop", type=int, default=1, choices=[0, 1],
                    help="config 3: enqueue the timed steps (env step + learn()) through torch.classes.flock."
                         "ScTrainLoop, K steps per C++ call (bitwise the per-step path); 0: one Python call per step "
                         "(flock::step_v2_store + the native learn() pipeline)")
    ap.add_argument("--policy-steps", type=int, default=20,
                    help="config 3, N=1: also time this many steps of the actor-driven loop of the reference's "
                         "driver (choose_action of every agent + OU noise -> env.step + insert -> learn(), "
                         "learners/maddpg_shared_critic/train_flock.py:114-121) after the headline, reported in the "
                         "policy_in_loop field (0: skip)")
    ap.add_argument("--diag-presleep-us", type=float, default=0.0,
                    help="diagnostics only (never a bench line): a sleep kernel of this length opens the timed region "
                         "so the host enqueues ahead of the GPU; the line then reports it in diag_presleep_ms")
    ap.add_argument("--diag-prewarm-ms", type=float, default=0.0,
                    help="diagnostics only (never a bench line): keep the GPU busy with matmuls for this long before "
                         "the warmup steps (clock / power-state probe)")
    ap.add_argument("--diag-cu-split", type=int, default=0,
                    help="diagnostics only (A/B): the learner stream on this many CUs (spread CU-mask bits) and the env "
                         "stream on the rest (hipExtStreamCreateWithCUMask, two masked streams made once)")
    ap.add_argument("--diag-knob", action="append", default=[],
                    help="diagnostics only (A/B): name=value for flock_set_diag before anything is built, e.g. "
                         "sc_event_system_scope=1 (the learner pipeline's events as system-scope fences)")
    ap.add_argument("--train-overlap", default="auto", choices=["auto", "0", "1"],
                    help="configs 4 / 5: train() on its own stream beside the following env steps (auto: on for VDN, "
                         "where it measured -3.5 %% per step; off for RNN-MADDPG, where it measured flat and its "
                         "update's HBM traffic slows the env launches it overlaps, profiles/r05/trainov/)")
    ap.add_argument("--rollout", type=int, default=None,
                    help="uw with no learner (config 2): the timed steps as VecFlockEnv.rollout calls of this many "
                         "steps each (flock_rollout_uw: all of them in ONE launch at N = 64, k = 4, the env state on "
                         "chip; the random-action regime, actions known up front). Default 50 for config 2, 0 "
                         "(one launch per step) otherwise")
    ap.add_argument("--sc-slots", type=int, default=None,
                    help="config 3: staging slots of the learn() pipeline (default 3; 5 or more also record the "
                         "slot-free events on every ((slots - 1) / 2)-th round only)")
    ap.add_argument("--overlap", type=int, default=1, choices=[0, 1],
                    help="config 3: run learn(s) on its own stream beside env step s+1 (minibatch snapshot; same "
                         "results; the env kernel time is unchanged by it); configs 4 / 5: see --train-overlap; "
                         "0: the learner runs after each step")
    args = ap.parse_args()
    c = CONFIGS[args.config]
    args.global_split = args.envs is None and "global_envs" in c
    if args.global_split:
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if c["global_envs"] % world:
            raise SystemExit(f"config {args.config}: {c['global_envs']} envs do not split over {world} ranks")
        args.envs = c["global_envs"] // world
    for key in ("envs", "agents", "variant", "learner", "steps"):
        if getattr(args, key) is None:
            setattr(args, key, c[key])
    return args


# BASELINE.json configs. 2 and 3: per GPU. 4 and 5 are 8-GPU configs: a global env count split over the ranks.
CONFIGS = {
    2: dict(variant="uw", agents=64, envs=1024, learner="none", steps=200),
    3: dict(variant="v2", agents=256, envs=4096, learner="shared_critic", steps=200),
    4: dict(variant="uw_discrete", agents=512, global_envs=8192, learner="vdn", steps=300),
    5: dict(variant="v2", agents=1024, global_envs=16384, learner="maddpg_rnn", steps=500),
}


def setup_dist(args):
    """One process per GPU over RCCL ("nccl"). FLOCK_DIST_BACKEND=gloo rehearses the N > 1 code path with several
    ranks on one GPU (device = LOCAL_RANK mod the visible GPUs); its numbers are not scaling results."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("FLOCK_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local % torch.cuda.device_count() if backend != "nccl" else local)
    torch.cuda.set_device(dev)
    if world > 1:
        kw = {"device_id": dev} if backend == "nccl" else {}
        torch.distributed.init_process_group(backend, **kw)
    return world, rank, dev


def barrier(world):
    if world > 1:
        torch.distributed.barrier()


def _cpu_run(args, box, seconds, seed, E_s=8):
    """One thread: the C oracle stepping E_s envs of the workload sequentially for `seconds` (ctypes releases the
    GIL during each C call, so several of these run in parallel)."""
    from oracle import oracle

    N, k = args.agents, args.k
    rng = np.random.default_rng(seed)
    pos = rng.uniform(0, box, (E_s, N, 2)).astype(np.float32)
    head = rng.uniform(0, 1.5 * np.pi, (E_s, N)).astype(np.float32)
    prev = np.zeros((E_s, N), np.float32)
    mem = np.zeros((E_s, N, 4, k), np.float32)
    vel = np.zeros((E_s, N, 2), np.float32)
    vel[..., 0] = 1.0
    n = 0
    t0 = time.perf_counter()
    while True:
        if args.variant == "uw_discrete":
            act = rng.integers(0, 10, (E_s, N))
            o = oracle.step_uwd(pos, head, prev, act, (0.1 * rng.standard_normal((E_s, N, 2))).astype(np.float32),
                                k=k, box=box, cd=2.5)
        else:
            act = np.stack([rng.uniform(0, 1, (E_s, N)), rng.uniform(-1.5, 1.5, (E_s, N))], -1).astype(np.float32)
            if args.variant == "v2":
                o = oracle.step_v2(pos, head, act, k=k, box=box, cd=2.5)
            elif args.variant == "uw":
                o = oracle.step_uw(pos, head, prev, act, mem, k=k, box=box, cd=2.5)
                mem = o["obs"]
            else:
                o = oracle.step_flock(pos, vel, act, mem, k=k, box=box, cd=2.5)
                mem, vel = o["obs"], o["vel"]
        pos = o["pos"]
        head = o.get("heading", head)
        prev = o.get("prev_heading", prev)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return E_s * N * n, el


def host_cpus():
    """CPUs this process may run on: the affinity mask, capped by the cgroup v2 CPU quota (a container's share of a
    large host), and the host's CPU model string."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, model


def _torch_ref_run(args, box, seconds, threads, seed):
    """The reference's v2 step as its torch-CPU op sequence (oracle/torch_ref.py), one env object stepped at a time
    as the reference steps its single env, on `threads` torch threads for `seconds`: agent-steps/s."""
    from oracle.torch_ref import V2Env

    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        N, k = args.agents, args.k
        g = torch.Generator().manual_seed(seed)
        env = V2Env(torch.rand(N, 2, generator=g) * box, (1.0 - torch.rand(N, generator=g)) * 1.5 * np.pi, k=k,
                    box=box, sensor_range=14.0, collision_distance=2.5)
        acts = [torch.stack([torch.rand(N, generator=g), torch.rand(N, generator=g) * 3 - 1.5], -1) for _ in range(8)]
        for a in acts[:2]:
            env.step(a)
        n, t0 = 0, time.perf_counter()
        while True:
            env.step(acts[n % 8])
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                return N * n / el, n
    finally:
        torch.set_num_threads(prev)


def _torch_ref_worker(a):
    """One worker process of the all-cores CPU baseline: the reference's step (torch restatement) on 1 thread."""
    agents, k, box, seconds, seed = a
    ns = argparse.Namespace(agents=agents, k=k)
    rate, n = _torch_ref_run(ns, box, seconds, 1, seed)
    return rate, n


def _torch_ref_all_cores(args, box, seconds, procs):
    """The reference's step on every usable host core: `procs` worker processes (spawned: fresh interpreters, no GPU
    state), each stepping its own env on one torch thread for `seconds`; agent-steps/s summed over the workers."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        res = pool.map(_torch_ref_worker, [(args.agents, args.k, box, seconds, 100 + i) for i in range(procs)])
    return sum(r[0] for r in res), sum(r[1] for r in res)


def cpu_baseline(args, box, seconds):
    """The reference's CPU step on the box's host cores, a bounded sample of the same workload. v2 (the headline):
    the torch-CPU restatement of environments/gym_flock_v2.py's step (oracle/torch_ref.py; pinned against the
    reference's golden vectors by tests/test_cpu_baseline.py and timed against the reference itself, ratio ~1.0, in
    tests/golden/cpu_calibration.json), one env at a time as the reference runs, on every usable host CPU and on one
    thread. Other variants: the C oracle port (oracle/flock_oracle.c) on the same cores."""
    threads, model = host_cpus()
    half = seconds / 2
    if args.variant == "v2":
        # throughput baseline: the reference's step on every usable core (one env per worker process); beside it the
        # reference's as-run speed (one env, stepped sequentially, 1 torch thread and all threads)
        va, na = _torch_ref_all_cores(args, box, half, threads)
        v1, n1 = _torch_ref_run(args, box, half / 2, 1, 0)
        vt, nt = _torch_ref_run(args, box, half / 2, threads, 1)
        calib = None
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", "cpu_calibration.json")
        if os.path.exists(path):
            with open(path) as f:
                calib = [r for r in json.load(f)["rows"] if r["N"] == args.agents] or None
        return {"value": va, "unit": "agent-steps/s", "cores": threads, "kind": "port",
                "reference_as_run_1thread": v1, "reference_as_run_all_threads": vt, "cpu_model": model,
                "host_cpus": os.cpu_count(), "calibration_vs_reference": calib,
                "sample": f"oracle/torch_ref.py: environments/gym_flock_v2.py's step as its torch-CPU op sequence "
                          f"(meshgrid distances, topk, clamp, .item() sync) on {args.agents}-agent envs. value: "
                          f"{threads} worker processes (the CPUs this process may use), each stepping its own env on "
                          f"1 torch thread for {half:.0f} s ({na} steps in all, {va:.3g} agent-steps/s). The "
                          f"reference as it runs (one env stepped sequentially): {half / 2:.1f} s on 1 thread ({n1} "
                          f"steps, {v1:.3g} agent-steps/s), {half / 2:.1f} s on {threads} threads ({nt} steps, "
                          f"{vt:.3g}); {model}"}
    s1, t1 = _cpu_run(args, box, half, 0)
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(threads) as ex:  # 32 envs per C call: the per-call Python work is negligible
        res = list(ex.map(lambda i: _cpu_run(args, box, half, 1 + i, E_s=32), range(threads)))
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {"value": steps / wall, "unit": "agent-steps/s", "cores": threads, "kind": "port",
            "value_1thread": s1 / t1, "cpu_model": model, "host_cpus": os.cpu_count(),
            "sample": f"oracle/flock_oracle.c {args.variant} step of {args.agents}-agent envs, sequential vectorized "
                      f"steps for {half:.0f} s: 1 thread x 8 envs ({s1 / t1:.3g} agent-steps/s), {threads} threads "
                      f"(the CPUs this process may use) x 32 envs ({steps / wall:.3g} agent-steps/s); {model}"}


def valu_fields(vp, busy, lane_ops, kern_s, alone_ms, tag):
    """The VALU roofline block: one step's counters (one launch, profiles/pmc_valu_<tag>.json) against the step's
    HIP-event time in the timed region (kern_s) and alone (alone_ms)."""
    peak = lane_ops * CLOCK_HZ / busy  # this instruction mix with every SIMD issuing every cycle
    out = {"insts_per_launch": vp["SQ_INSTS_VALU"], "insts_per_wave": vp.get("valu_insts_per_wave"),
           "issue_quadcycles": vp["SQ_ACTIVE_INST_VALU"], "coissue_quadcycles": vp["SQ_ACTIVE_INST_VALU2"],
           "coissued_share": 2.0 * vp["SQ_ACTIVE_INST_VALU2"] / vp["SQ_INSTS_VALU"],
           "busy_cycles_per_simd": busy, "clock_hz": CLOCK_HZ,
           "lane_ops_per_s": lane_ops / kern_s, "peak": peak, "unit": "lane-op/s",
           "frac": busy / (kern_s * CLOCK_HZ),
           "frac_alone": busy / (alone_ms * 1e-3 * CLOCK_HZ) if alone_ms else None,
           "peak_full_rate": VALU_PEAK_FULL_RATE, "frac_full_rate": lane_ops / kern_s / VALU_PEAK_FULL_RATE,
           "source": f"profiles/pmc_valu_{tag}.json", "rates": "profiles/ubench_valu.json"}
    return out


class VDNBench:
    """BASELINE config 4 learner: every env's team transition (obs, action ids, rewards, next obs, any_done) is put
    into the VDN replay ring each vectorized step (learners/vdn/train_flock.py:88-104), and VDN train() (10 updates
    of B=32 chunks of 10, clip 5, Adam) runs every 150 vectorized steps (the reference's episode length, :98)."""

    every = 150

    def __init__(self, env, dev, seed=0, overlap=True):
        from marl_range_flocking_amd.learners.vdn import VDNLearner

        self.env = env
        group = torch.distributed.group.WORLD if torch.distributed.is_initialized() else None
        self.learner = VDNLearner(env.N, env.k, 10, device=dev, seed=seed, dist_group=group)
        # train() beside the env steps that follow it (random actions: they do not read the QNet); the sampled rows
        # are copied out of the ring first (learners/core.py OverlappedTrain); data-parallel: in line
        self.overlap = overlap and not self.learner.distributed
        self.prev = None

    def _train(self):
        return self.learner.train_overlapped() if self.overlap else self.learner.train()

    def describe(self):
        return (f"VDN train() every {self.every} vectorized steps (update_iter 10, B 32, chunk 10"
                + ("; on its own stream beside the following env steps, sampled rows copied out first" if self.overlap
                   else "") + f"); all {self.env.E} team transitions per step inserted into a 50k-row device replay "
                f"ring by the env kernel itself" + ("; gradient all-reduce over RCCL" if self.learner.distributed else ""))

    def before(self, s):
        # the env kernel writes every env's team transition itself (memory.put, train_flock.py:102: previous obs,
        # action ids, rewards, new obs, any_done; FlockRing action_ids / env_done)
        return self.learner.replay_slots(self.env.E)

    def after(self, s, a):
        if (s + 1) % self.every == 0 and self.learner.size() > self.learner.chunk:
            self._train()

    def prime(self):
        self._train()
        self.finish()

    def finish(self):  # an overlapped train() still running joins the env stream (inside the timed region)
        self.learner.sync()


class MADDPGBench:
    """BASELINE config 5 learner: each env's record (actor obs, next obs, actions, critic state, next state,
    rewards, dones) goes into the RNN-MADDPG replay ring every vectorized step (main.py:24-59), and train()
    (B=128 chunks of 10, per-agent recurrent critics over all agents' obs and actions) runs every 250 steps
    (main.py:103)."""

    every = 250

    def __init__(self, env, dev, seed=0, overlap=True):
        from marl_range_flocking_amd.learners.maddpg import MADDPGLearner

        self.env = env
        group = torch.distributed.group.WORLD if torch.distributed.is_initialized() else None
        # under torchrun: agent-sharded critics (each rank owns N / world critics; the minibatches and the actor
        # heads' actions are all-gathered instead of all-reducing the 3.6-GB critic gradient)
        # shared_obs: gym_flock_v2's critic and actor observations are the same dnn rows (gym_flock_v2.py:110-125),
        # so the record's actor copies alias state / next_state in the ring (written once by the env kernel)
        self.learner = MADDPGLearner(env.N, env.k, recurrent=True, device=dev, seed=seed, dist_group=group,
                                     agent_shard=group is not None and env.N % torch.distributed.get_world_size() == 0,
                                     shared_obs=True)
        # train() beside the env steps that follow it (random actions: they do not read the networks); the sampled
        # chunks are copied out of the ring first (learners/core.py OverlappedTrain); multi-rank: in line
        self.overlap = overlap and not (self.learner.distributed or self.learner.shard)
        self.prev = None

    def _train(self):
        return self.learner.train_overlapped() if self.overlap else self.learner.train()

    def describe(self):
        L = self.learner
        return (f"RNN-MADDPG train() every {self.every} vectorized steps (B 128, chunk 10, {self.env.N} critics "
                f"400/300" + ("; on its own stream beside the following env steps, sampled chunks copied out first"
                             if self.overlap else "") + f"); all {self.env.E} env records per step inserted into a "
                f"45k-row device replay ring by the env kernel itself"
                + ("; agent-sharded critics, minibatch + action all-gathers over RCCL" if L.shard else
                   "; critic gradient all-reduce over RCCL" if L.distributed else ""))

    def before(self, s):
        # the env kernel writes every env's record itself (flock_step_v2_store, one ring row per env)
        return self.learner.replay_slots(self.env.E)

    def after(self, s, a):
        L = self.learner
        if (s + 1) % self.every == 0 and L.check_buffer_size():
            self._train()

    def prime(self):
        if self.learner.check_buffer_size():
            self._train()
        self.finish()

    def finish(self):  # an overlapped train() still running joins the env stream (inside the timed region)
        self.learner.sync()


def policy_loop(hook, env, first, steps):
    """The actor-driven training loop of learners/maddpg_shared_critic/train_flock.py:114-121 at the bench's size:
    choose_action of every agent on the current observation (mu + OU noise, agent_simple_shared_critic.py:92-107,
    batched over all agents and envs), the env step with the fused replay insert, then one learn(). Each step's
    actions come from the actors the previous learn() updated, so nothing of step s+1 overlaps learn(s) here."""
    L = hook.learner
    dev = env.device
    stream = torch.cuda.current_stream(dev)
    marks = []

    def one(s, timed):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if timed else None
        if e:
            e[0].record(stream)
        a = L.choose_action(env.dnn, noise=True)
        if e:
            e[1].record(stream)
        env.step(a, ring=hook.before(s))
        if e:
            e[2].record(stream)
        L.learn(s % L.n_agents)
        if e:
            e[3].record(stream)
            marks.append(e)

    for i in range(3):  # graph capture of the serial learn() and the OU state outside the timed steps
        one(first + i, False)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        one(first + 3 + i, True)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    part = lambda i: float(np.mean([m[i].elapsed_time(m[i + 1]) for m in marks]))  # noqa: E731
    # choose_action's algorithmic work: every actor's fc1, fc2 and mu head on every env row (f32 MFMA for fc2)
    flops = 2.0 * env.E * env.N * (L.fc1 * L.input_dim + L.fc1 * L.fc2 + L.fc2 * L.n_actions)
    act_ms = part(0)
    return {"ms_per_step": el / steps * 1e3, "value": env.E * env.N * steps / el, "unit": "agent-steps/s",
            "steps": steps, "act_ms": act_ms, "env_step_ms": part(1), "learn_ms": part(2),
            "act_path": "flock_sc_act (one fused MFMA launch + the OU draws)" if L.fused_act_ok() else "torch bmm chain",
            "act_tflops": flops / (act_ms * 1e-3) / 1e12, "act_mfma_frac": flops / (act_ms * 1e-3) / MFMA_F32_PEAK,
            "note": "choose_action (stacked actors, every env and agent, + OU noise) -> env step + replay insert -> "
                    "learn(agent s mod 256), serial: the next step's actions need this learn()'s actor update"}


def cu_split_streams(dev, keep):
    """Two CU-masked streams (diagnostics): the learner's on `keep` CUs spread over the mask bits, the env's on the
    rest."""
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    lb = [i for i in range(ncu) if (i * keep) // ncu != ((i + 1) * keep) // ncu]

    def masked(bits):
        words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
        for i in bits:
            words[i // 32] |= 1 << (i % 32)
        h = ctypes.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), words) == 0
        return torch.cuda.ExternalStream(h.value, device=dev)

    return masked(lb), masked([i for i in range(ncu) if i not in set(lb)])


def main():
    args = parse()
    world, rank, dev = setup_dist(args)
    from marl_range_flocking_amd import FlockConfig, VecFlockEnv

    if args.diag_knob:
        from marl_range_flocking_amd import _native

        for kv in args.diag_knob:
            name, val = kv.split("=")
            assert _native.lib().flock_set_diag(name.encode(), int(val)) == 0, kv

    E, N, k = args.envs, args.agents, args.k
    launches = args.step_launches or (3 if args.learner == "shared_critic" and args.overlap else 1)
    box = float(round(np.sqrt(250.0 * N)))  # main.py density: 10 agents in 50x50
    cfg = FlockConfig(variant=args.variant, num_envs=E, num_agents=N, k=k, collision_distance=2.5,
                      range_start=(0, box), sensor_range=14.0, seed=1234 + rank,
                      track_indices=args.variant == "v2",  # the reference returns neighbour indices for v2 only
                      step_launches=launches)
    env = VecFlockEnv(cfg, device=dev)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    env.positions.copy_(torch.rand(E, N, 2, device=dev, generator=g) * box)
    hmax = {"v2": 1.5 * np.pi, "uw": 2 * np.pi, "uw_discrete": np.pi / 1.2, "flock": 0.0}[args.variant]
    env.headings.copy_((1.0 - torch.rand(E, N, device=dev, generator=g)) * hmax)
    if args.variant == "flock":
        env.velocities[..., 0] = 1.0
    pool = []
    for _ in range(8):
        if args.variant == "uw_discrete":
            pool.append(torch.randint(0, 10, (E, N), device=dev, generator=g))
        elif args.variant == "v2":
            pool.append(torch.stack([torch.rand(E, N, device=dev, generator=g),
                                     torch.rand(E, N, device=dev, generator=g) * 3 - 1.5], -1).contiguous())
        else:
            pool.append((torch.rand(E, N, 2, device=dev, generator=g) * 2 - 1).contiguous())

    hook = None
    if args.learner == "shared_critic":
        from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench

        hook = SharedCriticBench(env, device=dev, seed=1234 + rank, overlap=bool(args.overlap), n_slots=args.sc_slots)
        if args.diag_cu_split > 0:  # A/B diagnostics: the GPU partitioned between the learner and the env stream
            ls_m, es_m = cu_split_streams(dev, args.diag_cu_split)
            torch.cuda.synchronize(dev)
            torch.cuda.set_stream(es_m)
            hook.stream = ls_m
    elif args.learner == "vdn":
        hook = VDNBench(env, dev, seed=1234 + rank,
                        overlap=bool(args.overlap) and args.train_overlap in ("auto", "1"))
    elif args.learner == "maddpg_rnn":
        hook = MADDPGBench(env, dev, seed=1234 + rank, overlap=bool(args.overlap) and args.train_overlap == "1")

    R = args.rollout if args.rollout is not None else (50 if args.config == 2 else 0)
    use_rollout = R > 0 and hook is None and args.variant == "uw"
    if use_rollout:  # the action stack of a rollout call: the pool's actions, resident before timing
        acts = torch.stack([pool[i % len(pool)] for i in range(R)]).contiguous()
        r_out = env.rollout(acts[:1])
        r_out = tuple(torch.empty((R,) + tuple(o.shape[1:]), dtype=o.dtype, device=dev) for o in r_out)

    def rollout_steps(s0, n, evs_r=None):
        for s in range(s0, s0 + n, R):
            r = min(R, s0 + n - s)
            e = evs_r.get(s - s0) if evs_r is not None else None
            if e is not None:
                e[0].record(stream)
            env.rollout(acts[:r], out=tuple(o[:r] for o in r_out))
            if e is not None:
                e[1].record(stream)

    def one_step(s, ev=None):
        a = pool[s % len(pool)]
        ring = hook.before(s) if hook is not None else None
        if ev is not None:
            ev[0].record(stream)
        env.step(a, ring=ring) if ring is not None else env.step(a)
        if ev is not None:
            ev[1].record(stream)
        if hook is not None:
            hook.after(s, a)

    stream = torch.cuda.current_stream(dev)
    if args.diag_prewarm_ms > 0:
        xw = torch.rand(4096, 4096, device=dev)
        torch.cuda.synchronize(dev)
        tw = time.perf_counter()
        while time.perf_counter() - tw < args.diag_prewarm_ms * 1e-3:
            for _ in range(4):
                xw = torch.tanh(xw @ xw * 1e-3)
            torch.cuda.synchronize(dev)
        del xw
    use_loop = bool(args.loop) and hook is not None and getattr(hook, "can_loop", lambda: False)()
    if use_loop:
        hook.run_steps(0, args.warmup, pool)
    elif use_rollout:
        rollout_steps(0, args.warmup)
    else:
        for s in range(args.warmup):
            one_step(s)
    if hook is not None:
        hook.prime()  # graph capture / first update outside the timed region
    torch.cuda.synchronize(dev)
    # the env kernel's HIP-event timing: every EV_EVERY-th step of the timed region (two timing markers per step
    # would add host and queue work of their own to a ~13-us launch-bound step)
    ev = {s: (DevEvent(), DevEvent()) for s in range(0, args.steps, R if use_rollout else EV_EVERY)}
    evs = [e for s in sorted(ev) for e in ev[s]]
    for e in evs:  # create the HIP events outside the timed region
        e.record(stream)

    span = (DevEvent(), DevEvent())
    for e in span:
        e.record(stream)
    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    span[0].record(stream)  # the GPU-side span of the timed region (its first to its last enqueued command)
    if args.diag_presleep_us > 0:
        torch.cuda._sleep(int(args.diag_presleep_us * 1e-6 * 2.1e9))  # ~2.1 GHz shader clock under load
    if use_loop:
        hook.run_steps(args.warmup, args.steps, pool, evs, EV_EVERY)
    elif use_rollout:
        rollout_steps(args.warmup, args.steps, ev)
    else:
        for s in range(args.steps):
            one_step(args.warmup + s, ev.get(s))
    if hook is not None and hasattr(hook, "finish"):
        hook.finish()  # the learner work still pending (the last learn's actor phase) runs inside the timed region
    span[1].record(stream)
    host_el = time.perf_counter() - t0  # host enqueue time of the timed steps (no synchronisation inside)
    torch.cuda.synchronize(dev)
    barrier(world)
    el = time.perf_counter() - t0
    handoff = None
    if hook is not None and hasattr(hook, "learner") and hasattr(hook.learner, "pipeline_check"):
        hook.learner.pipeline_check()  # raises if a round gave up waiting for its snapshot (device-side gate)
        if hook.learner.__dict__.get("_pipe") is not None:
            handoff = {0: "cross-queue event wait", 1: "device gate polled by the critic row blocks"}[
                hook.learner.pipeline().gated()]
            if getattr(hook.learner, "distributed", False):
                handoff += ("; data-parallel actor all-reduce + Adam on a second group and stream"
                            if getattr(hook.learner, "dp_split", False) else "; data-parallel rounds, one all-reduce")
                handoff += (", direct RCCL calls" if getattr(hook.learner, "dp_rccl", False)
                            and torch.distributed.get_backend() == "nccl" else ", c10d ProcessGroup calls")
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    if use_rollout:  # per step: each timed rollout call over the steps it ran
        kern_ms = float(np.mean([a.elapsed_time(b) / min(R, args.steps - s) for s, (a, b) in ev.items()]))
    else:
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev.values()]))
    # the env step alone (after the timed region, no learner beside it, as ONE launch): what the kernel does when it
    # has the GPU to itself
    alone_ms = None
    if hook is not None:
        env.set_param("step_launches", 1)
        ev_alone = [(DevEvent(), DevEvent()) for _ in range(10)]
        for i, (a0, a1) in enumerate(ev_alone):
            a = pool[i % len(pool)]
            ring = hook.before(args.warmup + args.steps + i)
            a0.record(stream)
            env.step(a, ring=ring) if ring is not None else env.step(a)
            a1.record(stream)
        torch.cuda.synchronize(dev)
        alone_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_alone[2:]]))

    # the host cost of enqueueing a step, apart from the GPU: the GPU is held by a ~50 ms sleep kernel on the env
    # stream while 32 steps are enqueued, so no full hardware queue throttles the enqueue (in the timed region the
    # host runs ahead until the queue is full, and host_ms_per_step then follows the GPU)
    host_us = None
    if use_loop:
        hook.finish()
        torch.cuda.synchronize(dev)
        torch.cuda._sleep(int(2.4e9 * 0.05))
        t_h = time.perf_counter()
        hook.run_steps(args.warmup + args.steps + 50, 32, pool)
        host_us = (time.perf_counter() - t_h) / 32 * 1e6
        hook.finish()
        torch.cuda.synchronize(dev)

    total_agent_steps = world * E * N * args.steps
    value = total_agent_steps / el
    fused_ring = args.learner in RING_BYTES_PER_AGENT_STEP
    bpa = BYTES_PER_AGENT_STEP[args.variant]
    ins = RING_BYTES_PER_AGENT_STEP.get(args.learner, 0)
    kern_s = kern_ms * 1e-3
    achieved = bpa * E * N / kern_s / 1e9
    tag = f"{args.variant}{'_ring' if fused_ring else ''}{'_rollout' if use_rollout else ''}_N{N}_E{E}"
    prof = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")

    def pmc(name):
        path = os.path.join(prof, name)
        if not os.path.exists(path):
            return None
        with open(path) as f:
            return json.load(f)

    pt = pmc(os.path.basename(args.pmc)) if args.pmc else pmc(f"pmc_{tag}.json")
    traffic = pt.get("hbm_bytes_per_launch") if pt else None
    if traffic is not None and use_rollout:  # per step, like achieved: the PMC pass's launches ran R steps each
        traffic = traffic / pt.get("steps_per_launch", R)
    vp = pmc(f"pmc_valu_{tag}.json")
    valu = None
    if vp and "SQ_ACTIVE_INST_VALU2" in vp:
        busy = 4.0 * (vp["SQ_ACTIVE_INST_VALU"] - vp["SQ_ACTIVE_INST_VALU2"]) / SIMDS  # VALU issue cycles per SIMD
        lane_ops = 64.0 * vp["SQ_INSTS_VALU"]
        valu = valu_fields(vp, busy, lane_ops, kern_s, alone_ms, tag)
    hbm_frac = achieved / HBM_PEAK_GBS
    periodic = cfg.resolved().periodic
    c = CONFIGS[args.config]
    is_config = (args.variant, N, args.learner) == (c["variant"], c["agents"], c["learner"]) and (
        E == c.get("envs") or (args.global_split and E * world == c["global_envs"]))
    workload = f"gym_flock_{args.variant} step, {N} agents x {E} envs per GPU"
    if args.global_split:
        workload += f" ({E * world} envs split over {world} GPU{'s' if world > 1 else ''})"
    if is_config:
        workload += f" (BASELINE config {args.config})"
    line = {
        "metric": "agent-steps/sec at 256 agents x 4096 envs; 1/2/4/8 MI355X",
        "value": value,
        "unit": "agent-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "host_ms_per_step": host_el / args.steps * 1e3,
        # HIP events at the start and the end of the timed region on the launch stream: the GPU-side span, i.e.
        # ms_per_step without the launch latency of the first command and the final synchronisation
        "gpu_span_ms_per_step": span[0].elapsed_time(span[1]) / args.steps,
        **({"diag_presleep_us": args.diag_presleep_us} if args.diag_presleep_us > 0 else {}),
        **({"diag_prewarm_ms": args.diag_prewarm_ms} if args.diag_prewarm_ms > 0 else {}),
        **({"diag_knobs": args.diag_knob} if args.diag_knob else {}),
        **({"diag_cu_split": args.diag_cu_split} if args.diag_cu_split else {}),
        "host_enqueue_us_per_step": host_us,
        "host_path": ("torch.classes.flock.ScTrainLoop: all timed steps in one C++ call" if use_loop else
                      f"VecFlockEnv.rollout: {R} steps per call (torch.ops.flock.rollout_uw)" if use_rollout else
                      "one Python step per vectorized step (torch.ops.flock)"),
        "snapshot_handoff": handoff,
        "higher_is_better": True,
        "scaling": "strong" if args.global_split else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (uniform random positions/headings at main.py density, random actions; no checkpoints)",
        "config": {
            "workload": workload,
            "agents": N, "envs_per_gpu": E, "k": k, "box": box, "periodic": periodic,
            "learner": ("none: env step only" if hook is None else hook.describe()),
            "parallelism": f"env-shard x{world}",
        },
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": hbm_frac, "traffic": traffic,
                     "kernel": (f"rollout_uw_kernel ({R} steps per launch, env state on chip)" if use_rollout
                                and N == 64 and k == 4 else
                                f"step_kernel<{k + 2},{'periodic' if periodic else 'euclidean'}"
                                f"{',cells' if N >= 128 else ''}>" + (" + fused replay insert" if fused_ring else "")),
                     "kernel_ms": kern_ms, "bytes_per_agent_step": bpa,
                     **({"rollout_steps_per_launch": R,
                         "moved_bytes_per_agent_step": ROLLOUT_MOVED_BYTES} if use_rollout else {}),
                     "insert_bytes_per_agent_step": ins,
                     "achieved_incl_insert": (bpa + ins) * E * N / kern_s / 1e9,
                     "valu": valu,
                     "binding": binding(valu, hbm_frac, alone_ms, bpa * E * N),
                     "step_launches": launches,
                     # compare with rocprofv3's per-dispatch average
                     "kernel_ms_per_launch": kern_ms * R if use_rollout else kern_ms / launches,
                     "kernel_alone_ms": alone_ms,
                     "frac_alone": (bpa * E * N / (alone_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if alone_ms else None,
                     "valu_frac_alone": valu["frac_alone"] if valu else None,
                     "note": ("kernel_ms / frac: HIP events around every rollout launch of the timed region, per "
                              "step; frac on SURVEY 8(d)'s 149-B accounting (a single step reads and rewrites the "
                              "state and the memory); the rollout moves the action read and the observation / "
                              "reward / done writes (moved_bytes_per_agent_step)" if use_rollout else
                              f"kernel_ms / frac / valu: HIP events around every {EV_EVERY}th env step of the timed "
                              "region (the "
                              "step's launches, with the learner's kernels beside them); *_alone: the same step as one "
                              "launch with no learner, after the timed region")},
    }
    if (hook is not None and args.learner == "shared_critic" and world == 1 and args.policy_steps > 0
            and args.variant == "v2"):
        hook.finish()
        line["policy_in_loop"] = policy_loop(hook, env, args.warmup + args.steps + 100, args.policy_steps)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args, box, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
