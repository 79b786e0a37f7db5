#!/bin/bash
# Round 6: where the learner's ~7-us gap between rounds comes from: kernel traces with 3 slots (a slot-free event
# recorded after every round) and 8 slots (after every third), the gap after each round listed; and the bench's own
# timing markers (FLOCK_BENCH_EV_EVERY 4 = default vs 1000 = none in the timed region)
set -o pipefail
O=gpurun_out/r6gaps; mkdir -p $O; export TMPDIR=/tmp
for n in 3 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl$n -o run -- python bench.py --steps 80 --warmup 10 --policy-steps 0 --no-cpu-baseline --sc-slots $n > $O/tl$n.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python tools/trace_timeline.py $(find $O/tl$n -name "*kernel_trace.csv") > $O/timeline_$n.txt && tail -16 $O/timeline_$n.txt
  python tools/round_gaps.py $(find $O/tl$n -name "*kernel_trace.csv") > $O/gaps_$n.txt && cat $O/gaps_$n.txt
done
for r in 1 2; do for e in 4 1000; do
  FLOCK_BENCH_EV_EVERY=$e timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 > $O/s200_ev${e}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json,sys; [print(f, round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5)) for f in sys.argv[1:]]" $O/s200_ev${e}_$r.json
done; done
