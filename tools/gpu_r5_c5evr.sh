#!/bin/bash
# Config-5 env kernel with / without the even-row layout: rocprofv3 kernel stats of the bench, both trees, twice,
# interleaved (gpurun_out/c5evr/).
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/c5evr; mkdir -p $O
for r in 1 2; do
  for t in v_base cur; do
    d=_ab/$t; [ $t = cur ] && d=.
    (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${t}_$r -o run --output-format csv -- python3 bench.py --config 5 --no-cpu-baseline --steps 100 --warmup 10 > $O/${t}_$r.json 2> $O/${t}_$r.err) || { tail -20 $O/${t}_$r.err; exit 1; }
    f=$(ls $O/${t}_$r/*kernel_stats.csv | head -1)
    echo "$t rep $r: $(grep step_kernel $f | awk -F, '{print $1, "avg_ns", $4}' | cut -c1-220)"
  done
done
echo ALLDONE
