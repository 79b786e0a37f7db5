#!/bin/bash
# Round-6 final tree (after the L2 pull's removal): GPU suite + smoke, every config's bench line with rocprofv3
# kernel stats, the driver's command twice with its profile (gpurun_out/ev6c/), then the long runs
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ev6c
(while true; do date >> gpurun_out/ev6c/heartbeat.txt; sleep 30; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
EV_OUT=gpurun_out/ev6c PHASES="tests bench driver" CONFIGS="3 2 4 5" bash tools/gpu_evidence_r5.sh || exit 1
LONG_OUT=gpurun_out/long6c bash tools/gpu_r5_long.sh || exit 1
echo ALLDONE6C
