#!/bin/bash
# Every BASELINE config's bench line + a rocprofv3 kernel-trace stats run of the same command (GPU box).
# Usage: bash tools/gpu_bench_all.sh [configs...]   (default: 3 2 4 5); outputs under gpurun_out/bench/
set -u
OUT=gpurun_out/bench; mkdir -p $OUT; export TMPDIR=/tmp
CONFIGS=${*:-3 2 4 5}
for c in $CONFIGS; do
  timeout -k 10 300 python bench.py --config $c > $OUT/bench_config$c.json 2> $OUT/bench_config$c.err
  rc=$?; echo "rc(bench $c)=$rc"; tail -c 600 $OUT/bench_config$c.json; echo
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c$c -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline > $OUT/prof_c$c.log 2>&1
  rc=$?; echo "rc(rocprof $c)=$rc"
  [ $rc -eq 0 ] || exit $rc
done
echo ALLDONE
