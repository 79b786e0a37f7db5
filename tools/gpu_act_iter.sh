set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_act.py "tests/test_gpu_learners.py::test_shared_critic_choose_action_batched" 2>&1 | tail -2
for v in 1 1; do timeout -k 10 120 python tools/act_bench.py || exit 1; done
bash tools/gpu_act_pmc.sh
