#!/bin/bash
# HISTORICAL (round 6): the FLOCK_SC_NO_XCD macro was removed after this A/B measured flat (profiles/r06/noxcd/).
# Round 6: the XCD-aligned block maps of the learner round (xcd_perm, xcd_tile), now that the rounds run back to back:
# same-box A/B of the product build against -DFLOCK_SC_NO_XCD, 200 steps and the driver command, three rounds
set -o pipefail
B=$PWD/marl_range_flocking_amd/_build; O=$PWD/gpurun_out/r6noxcd; mkdir -p $O; export TMPDIR=/tmp
cp $B/libflock_amd.so $B/libflock_amd_base.so
for r in 1 2 3; do for v in base noxcd; do
  cp $B/libflock_amd_$v.so $B/libflock_amd.so
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 > $O/s200_${v}_$r.json 2> $O/err.txt || { cp $B/libflock_amd_base.so $B/libflock_amd.so; tail $O/err.txt; exit 1; }
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 > $O/drv_${v}_$r.json 2> $O/err.txt || { cp $B/libflock_amd_base.so $B/libflock_amd.so; tail $O/err.txt; exit 1; }
  python -c "import json,sys; [print(f.split('/')[-1], round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5)) for f in sys.argv[1:]]" $O/s200_${v}_$r.json $O/drv_${v}_$r.json
done; done
cp $B/libflock_amd_base.so $B/libflock_amd.so
