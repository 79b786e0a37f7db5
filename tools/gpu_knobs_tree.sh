#!/bin/bash
# A/B of env-var knobs on the bench inside a source tree exported under _ab/<tree> (see gpu_ab_trees.sh), interleaved.
# Usage: REPS=3 TREE=_ab/<sha> BENCH_ARGS="..." bash tools/gpu_knobs_tree.sh "A=1" "A=0" ...  (gpurun_out/knobs_tree/)
set -u
OUT=$PWD/gpurun_out/knobs_tree; mkdir -p $OUT
cd ${TREE:-.}
for r in $(seq 1 ${REPS:-3}); do
  i=0
  for kv in "$@"; do
    i=$((i+1))
    env $kv timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/${TAG:-run}_k${i}_r$r.json 2> $OUT/${TAG:-run}_k${i}_r$r.err || { echo "FAIL $kv"; tail -5 $OUT/${TAG:-run}_k${i}_r$r.err; exit 1; }
    echo "${TAG:-run} rep $r $kv -> $(grep -o "\"ms_per_step\": [0-9.]*\|\"snapshot_handoff\": \"[a-z -]*\|\"kernel_ms\": [0-9.]*" $OUT/${TAG:-run}_k${i}_r$r.json | tr "\n" " ")"
  done
done
