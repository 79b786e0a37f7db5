#!/bin/bash
set -o pipefail
bash tools/gpu_r6_evscope.sh || exit 1
O=gpurun_out/r6rollout; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/pytest_dist.txt 2>&1 || { tail -40 $O/pytest_dist.txt; exit 1; }
tail -2 $O/pytest_dist.txt
