#!/bin/bash
# Round 6, last check of the final tree: GPU suite + smoke (gpurun_out/ev6d/), the driver command once, and the N > 1
# bench path rehearsed with 2 gloo ranks on the one GPU
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ev6d
(while true; do date >> gpurun_out/ev6d/heartbeat.txt; sleep 30; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
EV_OUT=gpurun_out/ev6d PHASES="tests" bash tools/gpu_evidence_r5.sh || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ev6d/driver.json 2> gpurun_out/ev6d/driver.err || { tail gpurun_out/ev6d/driver.err; exit 1; }
tail -c 300 gpurun_out/ev6d/driver.json; echo
NPROC=2 CONFIGS="3" bash tools/gpu_dist_rehearsal.sh || exit 1
echo ALLDONE6D
