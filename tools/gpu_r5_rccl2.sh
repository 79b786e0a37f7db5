#!/bin/bash
# Direct RCCL collectives in the data-parallel C++ loop: the dist tests (the one-rank RCCL test takes the direct path),
# then the host cost per variant (tools/rccl_host_cost.py). Outputs under gpurun_out/rccl2/.
set -u
O=gpurun_out/rccl2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_dist.txt 2>&1 || { tail -30 $O/pytest_dist.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest_dist.txt | tail -10
timeout -k 10 500 python -u tools/rccl_host_cost.py > $O/host_cost.txt 2>&1 || { tail -30 $O/host_cost.txt; exit 1; }
grep -E "per step" $O/host_cost.txt
echo ALLDONE
