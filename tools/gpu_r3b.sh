# act kernel A/B (fc2.weight from global vs LDS-staged), MADDPG learner tests + config-5 train() profile
set -o pipefail
mkdir -p gpurun_out/r3b
for v in 0 1 0 1; do FLOCK_ACT_STAGE=$v timeout -k 10 120 python tools/act_bench.py || exit 1; done
FLOCK_ACT_STAGE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_act.py > gpurun_out/r3b/act_stage1.txt 2>&1 || { tail -20 gpurun_out/r3b/act_stage1.txt; exit 1; }
tail -1 gpurun_out/r3b/act_stage1.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -k "maddpg or MADDPG or checkpoint or shard" tests/test_gpu_learners.py tests/test_gpu_learners_scale.py tests/test_gpu_checkpoints.py tests/test_gpu_dist.py tests/test_gpu_dropin_drivers.py > gpurun_out/r3b/maddpg_tests.txt 2>&1 || { tail -40 gpurun_out/r3b/maddpg_tests.txt; exit 1; }
grep -c PASSED gpurun_out/r3b/maddpg_tests.txt; tail -1 gpurun_out/r3b/maddpg_tests.txt
timeout -k 10 300 python tools/maddpg_profile.py > gpurun_out/r3b/maddpg_prof.txt 2>&1 || exit 1
grep "per train" gpurun_out/r3b/maddpg_prof.txt; tail -42 gpurun_out/r3b/maddpg_prof.txt
