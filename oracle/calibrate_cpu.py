"""Time the CPU baseline (oracle/torch_ref.py) against the reference's own gym_flock_v2 step, here in the build
container (TEST INFRASTRUCTURE; needs /root/reference, which never reaches the GPU box). Writes
tests/golden/cpu_calibration.json: ms per step of each at N = 64 / 256 / 1024 with 1 and 8 torch threads, and the
ratio restatement / reference, which bench.py's cpu_baseline carries next to its own measurement.

    python oracle/calibrate_cpu.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:] = [p for p in sys.path if os.path.abspath(p or ".") != HERE]  # "oracle" is the package, not oracle.py
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import refshim  # noqa: E402

from oracle.torch_ref import V2Env  # noqa: E402


def timed(step, n):
    for _ in range(3):
        step()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    if not refshim.available():
        raise SystemExit("the reference is not present here")
    refshim.install()
    ref = refshim.load("environments/gym_flock_v2.py", "ref_gym_flock_v2")
    rows = []
    for N in (64, 256, 1024):
        box = float(round(np.sqrt(250.0 * N)))
        rng = np.random.default_rng(N)
        pos = rng.uniform(0, box, (N, 2)).astype(np.float32)
        head = rng.uniform(0, 1.5 * np.pi, N).astype(np.float32)
        acts = [torch.from_numpy(np.stack([rng.uniform(0, 1, N), rng.uniform(-1.5, 1.5, N)], -1).astype(np.float32))
                for _ in range(8)]
        for threads in (1, 8):
            torch.set_num_threads(threads)
            env = ref.MultiAgentEnv(agents=N, k=4, collision_distance=2.5, range_start=(0, box), sensor_range=14.0)
            env.positions = torch.from_numpy(pos.copy())
            env.headings = torch.from_numpy(head.copy())
            env.prev_headings = torch.zeros(N)
            mine = V2Env(pos, head, k=4, box=box, sensor_range=14.0, collision_distance=2.5)
            i = {"r": 0, "m": 0}

            def ref_step():
                env.step(acts[i["r"] % 8])
                i["r"] += 1

            def my_step():
                mine.step(acts[i["m"] % 8])
                i["m"] += 1

            n = max(20, int(4000 / N))
            # interleaved rounds, median of each side (the container's CPU clock and neighbours drift)
            tr, tm = [], []
            for _ in range(7):
                tr.append(timed(ref_step, n))
                tm.append(timed(my_step, n))
            t_ref, t_mine = float(np.median(tr)), float(np.median(tm))
            rows.append({"N": N, "threads": threads, "reference_ms_per_step": round(t_ref, 4),
                         "restatement_ms_per_step": round(t_mine, 4),
                         "ratio_restatement_over_reference": round(t_mine / t_ref, 3)})
            print(rows[-1])
    out = {"what": "environments/gym_flock_v2.py MultiAgentEnv.step (the reference, imported here through "
                   "tests/golden/refshim.py) vs oracle/torch_ref.py V2Env.step, one env, torch CPU, same inputs",
           "host": os.uname().nodename, "cpus": os.cpu_count(), "torch": torch.__version__, "rows": rows}
    with open(os.path.join(ROOT, "tests", "golden", "cpu_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
