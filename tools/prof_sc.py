"""rocprofv3 target: the fused shared-critic learn() at the bench shape (fc1 400, fc2 300, B 256), eager launches so
each of the 12 kernels shows up in the kernel trace (run: rocprofv3 --kernel-trace --stats -- python tools/prof_sc.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner  # noqa: E402

dev = torch.device("cuda", 0)
L = SharedCriticLearner(256, 4, device=dev, buffer_size=100_000, use_graph=os.environ.get("GRAPH", "0") == "1")
n = 8192
L.store_transitions(torch.rand(n, 4, device=dev) * 14, torch.rand(n, 2, device=dev), torch.rand(n, 1, device=dev),
                    torch.rand(n, 4, device=dev) * 14, torch.zeros(n, device=dev))
for i in range(int(os.environ.get("ITERS", "200"))):
    L.learn(i % 256)
torch.cuda.synchronize()
print("done")
