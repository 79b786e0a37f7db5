import cProfile, pstats, sys, os, time
sys.path.insert(0, os.getcwd())
import torch
from marl_range_flocking_amd import FlockConfig, VecFlockEnv
from marl_range_flocking_amd.learners.shared_critic import SharedCriticBench
dev = torch.device("cuda", 0)
E, N = 4096, 256
env = VecFlockEnv(FlockConfig(variant="v2", num_envs=E, num_agents=N, k=4, range_start=(0, 253), sensor_range=14,
                              collision_distance=2.5, step_launches=2), device=dev)
env.positions.uniform_(0, 253)
pool = [torch.rand(E, N, 2, device=dev) for _ in range(8)]
hook = SharedCriticBench(env, dev)
def one(s):
    a = pool[s % 8]
    ring = hook.before(s)
    env.step(a, ring=ring)
    hook.after(s, a)
for s in range(30): one(s)
hook.finish(); torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for s in range(30, 430): one(s)
pr.disable()
t1 = time.perf_counter()
hook.finish(); torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host {1e6*(t1-t0)/400:.1f} us/step (profiled), GPU-bound wall {1e6*(t2-t0)/400:.1f} us/step")
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
