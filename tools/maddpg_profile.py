"""RNN-MADDPG train() at the config-5 shape (1024 agents, k 4, hidden 400/300, B 128, chunk 10; learners/
maddpg_official_rnn/MADDPG.py:78-150) under torch.profiler: ms per train() with the HIP graph and eager, and the
kernels / ops one eager train() is made of (diagnostics)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from marl_range_flocking_amd.learners.maddpg import MADDPGLearner

dev = torch.device("cuda", 0)
N, K, T = int(os.environ.get("AGENTS", 1024)), 4, 200
L = None
for use_graph in (True, False):
    del L
    torch.cuda.empty_cache()
    L = MADDPGLearner(N, K, recurrent=True, hidden1=400, hidden2=300, batch_size=128, chunk_size=10,
                      buffer_capacity=T + 10, min_size_buffer=128, device=dev, use_graph=use_graph, seed=3)
    g = torch.Generator(device=dev).manual_seed(1)
    obs = torch.rand(T + 1, N, K, device=dev, generator=g) * 14
    act = torch.rand(T, N, 2, device=dev, generator=g) * 2.5 - 1
    rew = torch.where(torch.rand(T, N, device=dev, generator=g) < 0.05, -5.0, 0.01)
    done = (torch.rand(T, N, device=dev, generator=g) < 0.02).float()
    L.add_record(obs[:-1], obs[1:], act, obs[:-1], obs[1:], rew, done)
    for _ in range(2):
        L.train()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        L.train()
    torch.cuda.synchronize()
    print(f"use_graph={use_graph}: {1e3 * (time.perf_counter() - t0) / 5:.2f} ms per train()", flush=True)
from torch.profiler import ProfilerActivity, profile

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    L.train()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=45, max_name_column_width=60))
# the copies and GEMMs by input shape (where the time of aten::copy_ / mm / bmm goes)
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=40,
                                                         max_name_column_width=40, max_shapes_column_width=110))
# every copy-like op by input shape (the layout copies between the batched GEMMs)
rows = [e for e in prof.key_averages(group_by_input_shape=True)
        if any(k in e.key for k in ("copy", "add", "cat", "mul", "relu", "where", "sum", "Memcpy", "fill", "zero"))]
rows.sort(key=lambda e: -e.device_time_total)
print("copy-like ops by input shape (device us total, calls, shapes)")
for e in rows[:40]:
    print(f"{e.device_time_total:10.1f} {e.count:4d}  {e.key[:40]:40s} {str(e.input_shapes)[:150]}")
