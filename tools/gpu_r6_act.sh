#!/bin/bash
# Round 6: acting-kernel variants (tools/build_variant_act.sh builds): each variant's GPU act tests swapped in, then a
# same-box interleaved A/B on tools/act_bench.py. Usage: tools/gpu_r6_act.sh NAME...  (outputs gpurun_out/r6act/)
set -u
B=$PWD/marl_range_flocking_amd/_build; O=gpurun_out/r6act; mkdir -p $O
cp $B/libflock_amd.so $B/libflock_amd_base.so
for v in base "$@"; do
  cp $B/libflock_amd_$v.so $B/libflock_amd.so
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_act.py \
    "tests/test_gpu_learners.py::test_shared_critic_choose_action_batched" > $O/pytest_$v.txt 2>&1 || { cp $B/libflock_amd_base.so $B/libflock_amd.so; tail -30 $O/pytest_$v.txt; exit 1; }
  echo "$v tests: $(tail -1 $O/pytest_$v.txt)"
done
for r in 1 2 3; do
  for v in base "$@"; do
    cp $B/libflock_amd_$v.so $B/libflock_amd.so
    echo "$v r$r: $(timeout -k 10 120 python tools/act_bench.py 2>/dev/null | tail -1)" || { cp $B/libflock_amd_base.so $B/libflock_amd.so; exit 1; }
  done
done
cp $B/libflock_amd_base.so $B/libflock_amd.so
