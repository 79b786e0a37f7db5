#!/bin/bash
# Round 6: the GPU partitioned between the learner and the env stream (bench.py --diag-cu-split K: the learner on K
# spread CUs, the env on the rest; two masked streams per process), now that rounds follow each other with no gap:
# interleaved config-3 A/B against the unpartitioned default, 200 steps and the driver command
set -o pipefail
O=gpurun_out/r6cus; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do for K in 0 32 48 64 96; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 --diag-cu-split $K > $O/s200_${K}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 --diag-cu-split $K > $O/drv_${K}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json,sys; [print(f.split('/')[-1], round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5)) for f in sys.argv[1:]]" $O/s200_${K}_$r.json $O/drv_${K}_$r.json
done; done
