"""torch-CPU restatement of the reference's gym_flock_v2 step. TEST INFRASTRUCTURE ONLY (the timed CPU baseline).

SURVEY.md §8(d): the CPU baseline beside the GPU number is "the same per-env torch-CPU op sequence, stepping E envs
sequentially as the reference does" — the reference itself cannot travel to the GPU box. This module restates
environments/gym_flock_v2.py's MultiAgentEnv.step (:71-83) as that op sequence, one env object at a time, so its
cost structure is the reference's: the O(N^2) meshgrid / abs / where / sqrt distance matrix, a full-row topk, the
elementwise kinematics and boundary, the reward's two (unused) nearest-neighbour gathers and the `.item()` of
_computeDone. It is not the checker (oracle/flock_oracle.c is); tests/test_cpu_baseline.py pins it against the
reference's golden vectors, and oracle/calibrate_cpu.py times it against the reference itself here
(tests/golden/cpu_calibration.json records the ratio). Only bench.py's cpu_baseline leg and tests/ import it.
"""
import math

import torch


class V2Env:
    """One gym_flock_v2 env (periodic sensing, the make_env defaults of main.py) on CPU tensors."""

    def __init__(self, positions, headings, k=4, box=100.0, sensor_range=7.0, collision_distance=2.5,
                 max_linear_velocity=2.5):
        self.positions = torch.as_tensor(positions, dtype=torch.float32).clone()
        self.headings = torch.as_tensor(headings, dtype=torch.float32).clone()
        self.velocities = torch.zeros_like(self.positions)
        self.prev_headings = torch.zeros_like(self.headings)
        self.k, self.boundary, self.sensor_range = int(k), float(box), float(sensor_range)
        self.collision_distance, self.max_linear_velocity = float(collision_distance), float(max_linear_velocity)

    # _updateState(action, dt, heading=True), gym_flock_v2.py:317-350
    def _update_state(self, action, dt):
        ang = torch.clamp(action[:, 1], -math.pi / 2, math.pi / 2)
        self.headings += ang * dt
        lin = torch.clamp(action[:, 0], 0.005, self.max_linear_velocity)
        self.velocities = torch.stack((lin * torch.cos(self.headings), lin * torch.sin(self.headings)), dim=1)
        self.velocities = torch.nan_to_num(self.velocities)
        self.velocities *= dt
        self.positions += self.velocities

    # check_boundary() non-rigid teleport, :292-304
    def _check_boundary(self):
        B = self.boundary
        for c in (0, 1):
            self.positions[:, c] = torch.where(self.positions[:, c] < B, self.positions[:, c], 0.001)
            self.positions[:, c] = torch.where(self.positions[:, c] > 0, self.positions[:, c], B)

    # _computePeriodicDistances(), :135-151
    def _periodic_knn(self):
        x, y = self.positions[:, 0], self.positions[:, 1]
        x1, x2 = torch.meshgrid(x, x, indexing="ij")
        y1, y2 = torch.meshgrid(y, y, indexing="ij")
        dx, dy = torch.abs(x1 - x2), torch.abs(y1 - y2)
        half = self.boundary / 2
        dx = torch.where(dx > half, self.boundary - dx, dx)
        dy = torch.where(dy > half, self.boundary - dy, dy)
        d = torch.sqrt(torch.multiply(dx, dx) + torch.multiply(dy, dy))
        vals, idx = torch.topk(-d, self.k + 1, dim=1)
        self.nearest_neighbors = idx[:, 1:]
        self.dnn = torch.clamp(-vals[:, 1:], min=0, max=self.sensor_range)

    def step(self, action, dt=0.1):
        """gym_flock_v2.MultiAgentEnv.step (:71-83): returns (obs, reward [N, 1], (dones [N], all_done), {})."""
        self._update_state(action, dt)
        self._check_boundary()
        self._periodic_knn()
        collisions = torch.where(self.dnn < self.collision_distance, 1, 0)              # :212-215
        obs = {"critic": self.dnn.clone(), "actors": self.dnn.clone()}                  # :127-133
        dones = (torch.any(collisions, 1), torch.any(collisions).item())                # :306-315 (host sync)
        # _computeReward (:252-269): the collision term, plus the two nearest-neighbour terms the reference computes
        # and then leaves out of the sum (:231-245)
        penalty = torch.where(torch.any(collisions, 1), -5, 0.01)
        com = torch.mean(self.positions[self.nearest_neighbors], dim=1)
        _ = torch.where(torch.norm(self.positions - com, dim=1).reshape(-1, 1) < self.sensor_range / 1.75, 0.01, 0)
        mean_h = torch.mean(self.headings[self.nearest_neighbors], dim=1)
        _ = torch.where(torch.abs(mean_h - self.headings) < 0.1, 0.01, 0)
        return obs, penalty.reshape(-1, 1), dones, {}
