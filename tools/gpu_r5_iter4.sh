#!/bin/bash
# Round 5 iteration 4: the minibatch snapshot carried by the next env step's first launch (block 0) in the C++ loop
# (no snapshot kernel between env steps): tests, then same-box A/B against r5c (the standalone snapshot kernel)
set -o pipefail
mkdir -p gpurun_out/it4
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train_loop.py \
  tests/test_gpu_overlap.py tests/test_gpu_cells.py tests/test_gpu_env_parity.py tests/test_gpu_torch_ops.py \
  "tests/test_gpu_dist.py::test_two_ranks_dp_train_loop_equals_python_dp_rounds" > gpurun_out/it4/pytest.log 2>&1 \
  || { tail -40 gpurun_out/it4/pytest.log; exit 1; }
tail -3 gpurun_out/it4/pytest.log
ABT_OUT=abt_it4 TREES="r5c cur" tools/gpu_ab_trees.sh 3 \
  "--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0" \
  "--steps 500 --warmup 20 --no-cpu-baseline --policy-steps 0" || exit 1
