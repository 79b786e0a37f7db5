#!/bin/bash
# Round 6: env launches per config-3 step (1 / 2 / 3 = default / 4) and 2 vs 3 staging slots, now that the learner's
# rounds run back to back: interleaved, 200 steps and the driver command
set -o pipefail
O=gpurun_out/r6launch; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do for v in "L1 --step-launches 1" "L2 --step-launches 2" "L3 --step-launches 3" "L4 --step-launches 4" "S2 --sc-slots 2"; do
  set -- $v; n=$1; shift
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 "$@" > $O/s200_${n}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 "$@" > $O/drv_${n}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json,sys; [print(f.split('/')[-1], round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5)) for f in sys.argv[1:]]" $O/s200_${n}_$r.json $O/drv_${n}_$r.json
done; done
