#!/bin/bash
# Round 5: gated k1 blocks pull every fc2 panel before the snapshot gate when the agent indices are host values
# (base = previous head in _ab/base). Pipeline tests in this tree, then an interleaved same-box A/B.
set -o pipefail
mkdir -p gpurun_out/pullknown
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_overlap.py tests/test_gpu_train_loop.py \
  tests/test_gpu_dist.py > gpurun_out/pullknown/tests.log 2>&1 || { tail -30 gpurun_out/pullknown/tests.log; exit 1; }
tail -2 gpurun_out/pullknown/tests.log
ABT_OUT=pullknown/ab TREES="base cur" bash tools/gpu_ab_trees.sh 4 "--steps 200 --warmup 20" "--steps 20 --warmup 5"
