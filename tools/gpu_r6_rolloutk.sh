#!/bin/bash
# Round 6: config 2's rollout steps per launch (bench --rollout 50 = default / 100 / 200), interleaved
set -o pipefail
O=gpurun_out/r6rk; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do for K in 50 100 200; do
  timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --rollout $K > $O/c2_r${K}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['ms_per_step']*1e3, 3), 'us', '%.3e' % d['value'], round(d['roofline']['frac'], 3))" $O/c2_r${K}_$r.json
done; done
