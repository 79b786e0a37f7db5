#!/bin/bash
# The learner round alone / the env step alone / both, per tree (tools/round_alone.py), interleaved, plus a rocprofv3
# kernel trace of the 200-step config-3 bench per tree (per-kernel averages in the loop). TREES="r5a cur".
set -o pipefail
O=gpurun_out/round; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
  for t in ${TREES:-r5a cur}; do
    d=$PWD/_ab/$t; [ $t = cur ] && d=$PWD
    FLOCK_TREE=$d timeout -k 10 120 python tools/round_alone.py > $O/alone_${t}_$r.txt 2>&1 || { tail $O/alone_${t}_$r.txt; exit 1; }
    echo "$t rep $r: $(grep us/call $O/alone_${t}_$r.txt | tr -s ' ' | tr '\n' ';')"
  done
done
for t in ${TREES:-r5a cur}; do
  d=_ab/$t; [ $t = cur ] && d=.
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OLDPWD/$O/prof_$t -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 > $OLDPWD/$O/bench_$t.json 2>&1) || exit 1
  f=$(find $O/prof_$t -name "*kernel_stats.csv" | head -1); cp $f $O/kstats_$t.csv
  python3 - $O/kstats_$t.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("sc_", "step_kernel")):
        print(f"{n[:60]:60s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1e3:8.2f} us")
PY
done
