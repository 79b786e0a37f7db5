"""VDN train() at the config-4 shape (512 agents, obs 4, 10 actions, B 32, chunk 10, update_iter 10), eager (no
graph) under torch.profiler: the GPU time per train() and the kernels / ops it is made of (diagnostics)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from marl_range_flocking_amd.learners.vdn import VDNLearner

dev = torch.device("cuda", 0)
A, n_obs, n_act = 512, 4, 10
for use_graph in (True, False):
    L = VDNLearner(A, n_obs, n_act, device=dev, seed=3, use_graph=use_graph)
    g = torch.Generator(device=dev).manual_seed(1)
    n = 2000
    L.put(torch.rand(n, A, n_obs, device=dev, generator=g), torch.randint(0, n_act, (n, A), device=dev, generator=g),
          torch.rand(n, A, device=dev, generator=g), torch.rand(n, A, n_obs, device=dev, generator=g),
          torch.zeros(n, device=dev, dtype=torch.uint8))
    for _ in range(3):
        L.train()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        L.train()
    torch.cuda.synchronize()
    print(f"use_graph={use_graph}: {1e3 * (time.perf_counter() - t0) / 10:.2f} ms per train()", flush=True)
from torch.profiler import ProfilerActivity, profile

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    L.train()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40, max_name_column_width=60))
