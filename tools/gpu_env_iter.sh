#!/bin/bash
# env-kernel iteration: parity tests, then same-box A/B of library variants (configs 3 and 2), then the phase profile.
# Usage: tools/gpu_env_iter.sh VARIANT...   (outputs under gpurun_out/iter/)
set -o pipefail
O=gpurun_out/iter; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_cells.py tests/test_gpu_env_parity.py tests/test_gpu_reset.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_swap.sh "--steps 200 --no-cpu-baseline --policy-steps 0" "$@" || exit 1
mkdir -p $O/c3 && mv gpurun_out/abs/* $O/c3/
bash tools/gpu_ab_swap.sh "--config 2 --steps 300 --no-cpu-baseline" "$@" || exit 1
mkdir -p $O/c2 && mv gpurun_out/abs/* $O/c2/
timeout -k 10 200 python tools/phase_prof.py > $O/phase.txt 2>&1; tail -22 $O/phase.txt
