#!/bin/bash
# Round 5: the two-float4 Adam: learner kernel / learner tests, then its rate at config 5's critic size.
set -o pipefail
O=gpurun_out/adam2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learn_kernels.py \
  tests/test_gpu_learners.py tests/test_gpu_learners_scale.py tests/test_gpu_torch_ops_learn.py \
  tests/test_gpu_overlap_train.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python tools/adam_bw.py > $O/adam_bw.txt 2>&1 && cat $O/adam_bw.txt
