#!/bin/bash
# Round 6 A/B: the learner pipeline's events as device-scope releases (default) vs system-scope fences (HIP's
# default), interleaved, driver command + 200 steps; then a kernel-trace timeline of the default
set -o pipefail
O=gpurun_out/r6evscope; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
  for m in 0 1; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 --diag-knob sc_event_system_scope=$m > $O/drv_${m}_$r.json 2> $O/drv_${m}_$r.err || { tail $O/drv_${m}_$r.err; exit 1; }
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 --diag-knob sc_event_system_scope=$m > $O/s200_${m}_$r.json 2> $O/s200_${m}_$r.err || { tail $O/s200_${m}_$r.err; exit 1; }
    python -c "import json,sys; [print(f, round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5)) for f in sys.argv[1:]]" $O/drv_${m}_$r.json $O/s200_${m}_$r.json
  done
done
rm -rf $O/tl; mkdir -p $O/tl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- python bench.py --steps 80 --warmup 10 --policy-steps 0 --no-cpu-baseline > $O/tl/bench.json 2> $O/tl/bench.err || exit 1
f=$(find $O/tl -name "*kernel_trace.csv" | head -1)
python tools/trace_timeline.py "$f" > $O/timeline.txt
tail -16 $O/timeline.txt
