"""flock_sc_act alone at the config-3 shape (4096 env rows x 256 agents, actors 4 -> 400 -> 300 -> 2): ms per launch
(HIP events) and f32 MFMA fraction. FLOCK_ACT_STAGE=0/1 picks the fc2.weight path (diagnostics)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from marl_range_flocking_amd.learners.shared_critic import SharedCriticLearner

dev = torch.device("cuda", 0)
R, A = int(os.environ.get("ROWS", 4096)), int(os.environ.get("AGENTS", 256))
L = SharedCriticLearner(A, 4, device=dev, buffer_size=64)
obs = torch.rand(R, A, 4, device=dev) * 14
for _ in range(3):
    L.choose_action(obs, noise=False)
n = 20
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(n):
    L.choose_action(obs, noise=False)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / n
fl = 2.0 * R * A * (4 * 400 + 400 * 300 + 300 * 2)
print(f"stage={os.environ.get('FLOCK_ACT_STAGE', 'default')}: {ms:.3f} ms per choose_action, "
      f"{fl / ms / 1e9:.1f} TFLOP/s = {fl / ms / 1e9 / 157.3:.3f} of f32 MFMA peak")
