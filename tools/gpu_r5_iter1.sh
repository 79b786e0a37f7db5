#!/bin/bash
# Round 5 iteration 1: the learner cleanup + default device gate + split dp actor all-reduce + config-5 tests, then
# same-box A/B of configs 3 (driver command, 200 steps) and 5 against the round-4 head (and 4dcefeb for config 3)
set -o pipefail
mkdir -p gpurun_out/it1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_overlap.py \
  tests/test_gpu_train_loop.py tests/test_gpu_config5.py \
  "tests/test_gpu_dist.py::test_two_ranks_dp_train_loop_equals_python_dp_rounds" > gpurun_out/it1/pytest.log 2>&1 \
  || { tail -40 gpurun_out/it1/pytest.log; exit 1; }
tail -3 gpurun_out/it1/pytest.log
ABT_OUT=abt2 TREES="4dcefeb c2589f5 cur" tools/gpu_ab_trees.sh 3 \
  "--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0" \
  "--steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0" || exit 1
ABT_OUT=abt5 TREES="c2589f5 cur" tools/gpu_ab_trees.sh 2 "--config 5 --no-cpu-baseline" || exit 1
