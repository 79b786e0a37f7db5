#!/bin/bash
# Config 2's candidate scan over 2 lanes per agent (this tree) against 4 (_ab/v_base): the env tests here, then the
# A/B (gpurun_out/c2spl2/).
set -u
O=gpurun_out/c2spl2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cells.py tests/test_gpu_env_parity.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_env.txt 2>&1 || { tail -30 $O/pytest_env.txt; exit 1; }
tail -2 $O/pytest_env.txt
ABT_OUT=c2spl2/ab TREES="v_base cur" bash tools/gpu_ab_trees.sh 3 "--config 2 --no-cpu-baseline" || exit 1
echo ALLDONE
