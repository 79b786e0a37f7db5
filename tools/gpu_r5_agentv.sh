#!/bin/bash
# Host-known agent indices in the pipeline's round kernels (this tree) against the device-word reads (_ab/v_base): the
# learner / overlap / train-loop / dist GPU tests here, then the config-3 A/B (gpurun_out/agentv/).
set -u
O=gpurun_out/agentv; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_train_loop.py tests/test_gpu_learners.py tests/test_gpu_dist.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
ABT_OUT=agentv/ab TREES="v_base cur" bash tools/gpu_ab_trees.sh 3 "--steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0" "--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0" || exit 1
echo ALLDONE
