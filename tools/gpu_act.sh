# fused acting (flock_sc_act): GPU tests, the config-3 bench line with the policy-in-loop field, a rocprofv3 kernel
# summary of the policy loop
set -o pipefail
mkdir -p gpurun_out/act
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_act.py \
  "tests/test_gpu_learners.py::test_shared_critic_choose_action_batched" > gpurun_out/act/pytest.txt 2>&1 || { tail -30 gpurun_out/act/pytest.txt; exit 1; }
tail -3 gpurun_out/act/pytest.txt
timeout -k 10 300 python bench.py --steps 100 --policy-steps 30 --no-cpu-baseline > gpurun_out/act/bench.json 2> gpurun_out/act/bench.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/act/bench.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['policy_in_loop'])"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/act/prof -o run -- python bench.py --steps 20 --policy-steps 20 --no-cpu-baseline > gpurun_out/act/prof_bench.json 2> gpurun_out/act/prof.err || exit 1
f=$(find gpurun_out/act/prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/act/kernel_stats.csv
grep -i "sc_act\|layer_norm\|Cijk" gpurun_out/act/kernel_stats.csv | cut -c1-160 | head
