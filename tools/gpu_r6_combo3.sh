#!/bin/bash
# Round 6: per-block round profile (alone / beside env steps) of the current tree, then a same-box A/B of the round
# kernels' wave priority (-DFLOCK_SC_PRIO=1 / 3 builds against the product build), 200 steps and the driver command
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_scprof.sh || exit 1
B=$PWD/marl_range_flocking_amd/_build; O=$PWD/gpurun_out/r6prio; mkdir -p $O
cp $B/libflock_amd.so $B/libflock_amd_base.so
for r in 1 2 3; do for v in base prio1 prio3; do
  cp $B/libflock_amd_$v.so $B/libflock_amd.so
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 > $O/s200_${v}_$r.json 2> $O/err.txt || { cp $B/libflock_amd_base.so $B/libflock_amd.so; tail $O/err.txt; exit 1; }
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 > $O/drv_${v}_$r.json 2> $O/err.txt || { cp $B/libflock_amd_base.so $B/libflock_amd.so; tail $O/err.txt; exit 1; }
  python -c "import json,sys; [print(f.split('/')[-1], round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5)) for f in sys.argv[1:]]" $O/s200_${v}_$r.json $O/drv_${v}_$r.json
done; done
cp $B/libflock_amd_base.so $B/libflock_amd.so
