#!/bin/bash
# Round-6 baseline on a fresh box: driver command x2, 200-step x2, round parts alone, rocprofv3 stats of the 200-step loop
set -o pipefail
O=gpurun_out/r6base; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/driver_$r.json 2> $O/driver_$r.err || { tail $O/driver_$r.err; exit 1; }
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 > $O/s200_$r.json 2> $O/s200_$r.err || { tail $O/s200_$r.err; exit 1; }
  python -c "import json,sys; [print(f, json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step']) for f in sys.argv[1:]]" $O/driver_$r.json $O/s200_$r.json
done
timeout -k 10 200 python tools/round_alone.py > $O/alone.txt 2>&1 || { tail $O/alone.txt; exit 1; }
cat $O/alone.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 > $O/bench_prof.json 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kstats.csv
python3 - $O/kstats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("sc_", "step_kernel")):
        print(f"{n[:60]:60s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:8.2f} us")
PY
