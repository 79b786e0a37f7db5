#!/bin/bash
# Round 5 iteration 3: the single-GPU actor stream (each learn's actor phase off the learner chain) against merged
# rounds: pipeline tests, then an interleaved knob A/B on this tree (FLOCK_SC_ACTOR_STREAM=0 / 1)
set -o pipefail
mkdir -p gpurun_out/it3
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_overlap.py \
  tests/test_gpu_train_loop.py > gpurun_out/it3/pytest.log 2>&1 || { tail -40 gpurun_out/it3/pytest.log; exit 1; }
tail -3 gpurun_out/it3/pytest.log
TAG=s500 BENCH_ARGS="--steps 500 --warmup 20 --policy-steps 0" bash tools/gpu_knobs_tree.sh "FLOCK_SC_ACTOR_STREAM=0" "FLOCK_SC_ACTOR_STREAM=1" || exit 1
TAG=drv BENCH_ARGS="--gpus 1 --steps 20 --warmup 5 --policy-steps 0" bash tools/gpu_knobs_tree.sh "FLOCK_SC_ACTOR_STREAM=0" "FLOCK_SC_ACTOR_STREAM=1" || exit 1
