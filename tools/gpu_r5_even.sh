#!/bin/bash
# The even-row seeded scan (this tree) against the previous scan (_ab/v_base): env parity tests here, then the
# config-3 / config-5 A/B (gpurun_out/even/).
set -u
O=gpurun_out/even; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_cells.py tests/test_gpu_env_parity.py tests/test_gpu_train_loop.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_env.txt 2>&1 || { tail -30 $O/pytest_env.txt; exit 1; }
tail -2 $O/pytest_env.txt
ABT_OUT=even/ab TREES="v_base cur" bash tools/gpu_ab_trees.sh 3 "--steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0" "--config 5 --no-cpu-baseline" || exit 1
echo ALLDONE
