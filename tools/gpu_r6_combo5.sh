#!/bin/bash
# Round 6, final tree: the GPU suite + smoke (gpurun_out/ev6b/), then config 2's rollout steps-per-launch A/B, then the long runs (stability of the device slot release)
set -o pipefail
export TMPDIR=/tmp
EV_OUT=gpurun_out/ev6b PHASES=tests bash tools/gpu_evidence_r5.sh || exit 1
bash tools/gpu_r6_rolloutk.sh
LONG_OUT=gpurun_out/long6 bash tools/gpu_r5_long.sh
