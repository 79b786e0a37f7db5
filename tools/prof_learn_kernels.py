"""Kernel-level profile target: 50 shared-critic learn() calls (graph replay) at config-3 sizes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner  # noqa: E402

dev = torch.device("cuda", 0)
L = SharedCriticLearner(256, 4, device=dev, buffer_size=1_000_000)
n = 1 << 20
L.store_transitions(torch.rand(n, 4, device=dev), torch.rand(n, 2, device=dev), torch.rand(n, 1, device=dev),
                    torch.rand(n, 4, device=dev), torch.zeros(n, device=dev))
for i in range(60):
    L.learn(i % 256)
torch.cuda.synchronize()
