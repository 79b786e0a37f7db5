#!/bin/bash
# Config-5 env kernel with the round-5 pull placement and non-temporal streams: the env parity tests at its launch
# shape, then its PMC passes and bench line (tools/gpu_evidence_r5.sh, CONFIGS=5, into gpurun_out/c5final/), then the
# 2-rank rehearsal of the config-3 data-parallel loop (gloo on cuda:0; gpurun_out/rehearsal/).
set -u
O=gpurun_out/c5final; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_config5.py tests/test_gpu_cells.py tests/test_gpu_env_parity.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_env.txt 2>&1 || { tail -30 $O/pytest_env.txt; exit 1; }
tail -2 $O/pytest_env.txt
EV_OUT=$O PHASES="pmc bench" CONFIGS=5 bash tools/gpu_evidence_r5.sh || exit 1
CONFIGS=3 bash tools/gpu_dist_rehearsal.sh || exit 1
echo ALLDONE
