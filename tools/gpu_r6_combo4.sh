#!/bin/bash
# Round 6: data-parallel rounds with device-released slots (the agent index by value in their Adam launch): the
# multi-rank and one-rank RCCL tests and the pipeline tests, the one-rank RCCL host / step cost per variant, then the
# env-launch-count / slot-count A/B
set -o pipefail
O=gpurun_out/r6c4; mkdir -p $O; export TMPDIR=/tmp
(while true; do date >> $O/heartbeat.txt; sleep 30; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_overlap.py tests/test_gpu_train_loop.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 500 python -u tools/rccl_host_cost.py > $O/host_cost.txt 2>&1 || { tail -30 $O/host_cost.txt; exit 1; }
grep -E "per step" $O/host_cost.txt
bash tools/gpu_r6_launches.sh
