#!/bin/bash
# (1) tools/gpu_r5_rccl.sh (the data-parallel loops over RCCL on one rank + the dist tests); (2) the even-row seeded
# scan variant (_ab/v_even): env parity tests in that tree, then config-3 / config-5 A/B against this tree.
set -u
bash tools/gpu_r5_rccl.sh || exit 1
O=gpurun_out/even; mkdir -p $O
(cd _ab/v_even && timeout -k 10 600 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_cells.py tests/test_gpu_env_parity.py tests/test_gpu_train_loop.py -m gpu -q --timeout 120 --timeout-method thread) > $O/pytest_env.txt 2>&1 || { tail -30 $O/pytest_env.txt; exit 1; }
tail -2 $O/pytest_env.txt
ABT_OUT=even/ab TREES="v_even cur" bash tools/gpu_ab_trees.sh 3 "--steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0" "--config 5 --no-cpu-baseline" || exit 1
echo ALLDONE
