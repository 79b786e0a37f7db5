#!/bin/bash
# HISTORICAL (round 6): the knob this A/B sets was removed after it measured flat / slower; flock_set_diag now rejects it, so the script fails fast against the current tree.
# Round 6: env blocks per CU capped through the launch's LDS size (flock_set_diag env_cu_blocks 0 = off / 7 / 6), so a
# learner kernel dispatched while an env launch fills the machine finds free wave slots: interleaved config-3 A/B
# (driver command + 200 steps)
set -o pipefail
O=gpurun_out/r6cub; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do for C in 0 7 6; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 --diag-knob env_cu_blocks=$C > $O/drv_${C}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 --diag-knob env_cu_blocks=$C > $O/s200_${C}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json,sys; [print(f, round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5), json.loads(open(f).read().strip().splitlines()[-1])['roofline'].get('kernel_ms')) for f in sys.argv[1:]]" $O/drv_${C}_$r.json $O/s200_${C}_$r.json
done; done
for C in 0 7; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl$C -o run -- python bench.py --steps 80 --warmup 10 --policy-steps 0 --no-cpu-baseline --diag-knob env_cu_blocks=$C > $O/tl$C.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python tools/trace_timeline.py $(find $O/tl$C -name "*kernel_trace.csv") > $O/timeline_$C.txt && tail -16 $O/timeline_$C.txt
done
