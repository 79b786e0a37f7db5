#!/bin/bash
# Round 6: rows per load batch of the learner reductions (FLOCK_RED_RB 8 = default / 16 / 4) in the gap-free loop: same-box A/B, 200 steps and the driver command, three rounds; the pipeline tests on each variant first
set -o pipefail
B=$PWD/marl_range_flocking_amd/_build; O=$PWD/gpurun_out/r6rb; mkdir -p $O; export TMPDIR=/tmp
cp $B/libflock_amd.so $B/libflock_amd_base.so
for v in rb16 rb4; do
  cp $B/libflock_amd_$v.so $B/libflock_amd.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.txt 2>&1 || { cp $B/libflock_amd_base.so $B/libflock_amd.so; tail -20 $O/pytest_$v.txt; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.txt)"
done
for r in 1 2 3; do for v in base rb16 rb4; do
  cp $B/libflock_amd_$v.so $B/libflock_amd.so
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 > $O/s200_${v}_$r.json 2> $O/err.txt || { cp $B/libflock_amd_base.so $B/libflock_amd.so; tail $O/err.txt; exit 1; }
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 > $O/drv_${v}_$r.json 2> $O/err.txt || { cp $B/libflock_amd_base.so $B/libflock_amd.so; tail $O/err.txt; exit 1; }
  python -c "import json,sys; [print(f.split('/')[-1], round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5)) for f in sys.argv[1:]]" $O/s200_${v}_$r.json $O/drv_${v}_$r.json
done; done
cp $B/libflock_amd_base.so $B/libflock_amd.so
