#!/bin/bash
# Round 5 iteration 2: the env step's launches as multiples of 8 blocks with the L2 pull of the next launch's block
# (same XCD); env parity tests; same-box A/B against r5b (the XCD-aligned round without it) and a step-launches sweep
set -o pipefail
mkdir -p gpurun_out/it2
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cells.py \
  tests/test_gpu_env_parity.py tests/test_gpu_train_loop.py tests/test_gpu_config5.py > gpurun_out/it2/pytest.log 2>&1 \
  || { tail -40 gpurun_out/it2/pytest.log; exit 1; }
tail -3 gpurun_out/it2/pytest.log
ABT_OUT=abt_it2 TREES="r5b cur" tools/gpu_ab_trees.sh 3 \
  "--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0" \
  "--steps 500 --warmup 20 --no-cpu-baseline --policy-steps 0" \
  "--steps 500 --warmup 20 --no-cpu-baseline --policy-steps 0 --step-launches 2" \
  "--steps 500 --warmup 20 --no-cpu-baseline --policy-steps 0 --step-launches 4" || exit 1
