"""HBM rate of the fused Adam + target soft update (torch.ops.flock.adam_step) at config 5's critic size
(diagnostics): 1024 RNN-MADDPG critics, 906M parameters; 36 B of algorithmic traffic per parameter with the target
(p, g, m, v, t read; p, m, v, t written), 32 B without.   python tools/adam_bw.py [n_millions=906]"""
import os
import sys

import torch

sys.path.insert(0, os.environ.get("FLOCK_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from marl_range_flocking_amd.learners.core import _ops

    n = int(float(sys.argv[1]) * 1e6) if len(sys.argv) > 1 else 906_000_000
    dev = torch.device("cuda", 0)
    p, g, m, v, t = (torch.rand(n, device=dev) for _ in range(5))
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    for tgt, bpp in ((t, 36), (None, 32)):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for i in range(12):
            if i == 2:
                ev[0].record()
            step.add_(1)
            _ops().adam_step(p, g, m, v, step, None, tgt, 1e-3, 0.9, 0.999, 1e-8, 0.001, 0)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / 10
        print(f"n {n}: target {tgt is not None}: {ms:.3f} ms per call, {n * bpp / ms / 1e6:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
