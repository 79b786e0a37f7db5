#!/bin/bash
# The data-parallel C++ loops over RCCL on one GPU (one rank, tests/test_gpu_dist.py::test_one_rank_rccl_*), then
# the whole dist test file (gloo 2-rank tests too). Outputs under gpurun_out/rccl/.
set -u
O=gpurun_out/rccl; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_dist.txt 2>&1; rc=$?
tail -15 $O/pytest_dist.txt
exit $rc
