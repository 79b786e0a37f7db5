"""torch.profiler of one shared-critic learn(): where does the host time go?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner  # noqa: E402

dev = torch.device("cuda", 0)
L = SharedCriticLearner(256, 4, device=dev, buffer_size=100_000)
n = 4096
L.store_transitions(torch.rand(n, 4, device=dev), torch.rand(n, 2, device=dev), torch.rand(n, 1, device=dev),
                    torch.rand(n, 4, device=dev), torch.zeros(n, device=dev))
for i in range(5):
    L.learn(i)
torch.cuda.synchronize()
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
    for i in range(10):
        L.learn(i)
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))
