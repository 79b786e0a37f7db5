#!/bin/bash
# A/B of env-var knobs on the default bench (config 3) in one GPU session: each line "VAR=v VAR2=w ..." is one run.
# Usage: bash tools/gpu_knobs.sh "A=1" "A=0 B=2" ...   (outputs under gpurun_out/knobs/)
set -u
OUT=gpurun_out/knobs; mkdir -p $OUT
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/run$i.json 2> $OUT/run$i.err || { echo "FAIL $kv"; tail -5 $OUT/run$i.err; exit 1; }
  echo "$kv -> $(grep -o "\"ms_per_step\": [0-9.]*\|\"host_ms_per_step\": [0-9.]*\|\"kernel_ms\": [0-9.]*" $OUT/run$i.json | tr "\n" " ")"
done
