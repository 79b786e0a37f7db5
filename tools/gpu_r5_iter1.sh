#!/bin/bash
# Round 5 iteration: L2-persistence / XCD-dealing probes, the learner tests, then same-box A/B of configs 3 (driver
# command, 200 steps) and 5 across trees (_ab/<tree>: 4dcefeb, c2589f5 = round-4 head, r5a = the gate default without
# the XCD-aligned round; cur = this tree)
set -o pipefail
mkdir -p gpurun_out/it1
timeout -k 10 60 tools/ubench_l2_persist > gpurun_out/it1/l2_persist.txt 2>&1 || exit 1
cat gpurun_out/it1/l2_persist.txt
timeout -k 10 60 tools/ubench_xcd_map > gpurun_out/it1/xcd_map.txt 2>&1 || exit 1
cat gpurun_out/it1/xcd_map.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_overlap.py \
  tests/test_gpu_train_loop.py tests/test_gpu_config5.py tests/test_gpu_learners.py \
  "tests/test_gpu_dist.py::test_two_ranks_dp_train_loop_equals_python_dp_rounds" > gpurun_out/it1/pytest.log 2>&1 \
  || { tail -40 gpurun_out/it1/pytest.log; exit 1; }
tail -3 gpurun_out/it1/pytest.log
ABT_OUT=abt2 TREES="${TREES3:-4dcefeb c2589f5 r5a cur}" tools/gpu_ab_trees.sh 3 \
  "--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0" \
  "--steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0" || exit 1
ABT_OUT=abt5 TREES="c2589f5 cur" tools/gpu_ab_trees.sh 2 "--config 5 --no-cpu-baseline" || exit 1
