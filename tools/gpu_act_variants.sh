#!/bin/bash
# Acting kernel: GPU tests, then same-box interleaved A/B of libflock_amd.so variants on tools/act_bench.py
# (flock_sc_act alone at 4096 rows x 256 agents). Usage: tools/gpu_act_variants.sh NAME...  (outputs gpurun_out/actv/)
set -u
B=$PWD/marl_range_flocking_amd/_build; O=gpurun_out/actv; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_act.py \
  "tests/test_gpu_learners.py::test_shared_critic_choose_action_batched" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
cp $B/libflock_amd.so $B/libflock_amd_base.so
for r in 1 2 3; do
  for v in base "$@"; do
    cp $B/libflock_amd_$v.so $B/libflock_amd.so
    echo "$v r$r: $(timeout -k 10 120 python tools/act_bench.py 2>/dev/null | tail -1)" || { cp $B/libflock_amd_base.so $B/libflock_amd.so; exit 1; }
  done
done
cp $B/libflock_amd_base.so $B/libflock_amd.so
