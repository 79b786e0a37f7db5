#!/bin/bash
# Round-4 evaluation on one box: GPU tests, interleaved A/B of the learner hand-off knobs (FLOCK_SC_GATE /
# FLOCK_SC_FUSE) and of library variants (VARIANTS), per-step kernel timelines of chosen modes (TIMELINES, "|"-separated
# env settings), and the driver's own bench command. Every GPU step runs under its own time limit; stops at the first
# failure. Outputs: gpurun_out/r4eval/.
set -u
OUT=gpurun_out/r4eval; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name 2>&1; local rc=$?; echo "rc($name)=$rc";
  if [ $rc -ne 0 ]; then tail -40 $OUT/$name; exit $rc; fi; }
B="--steps 200 --warmup 20 --policy-steps 0 --no-cpu-baseline"
if [ "${TESTS:-none}" != "none" ]; then
  step pytest.txt 900 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread
  grep -E "passed|failed" $OUT/pytest.txt | tail -2
fi
if [ -n "${KNOBS:-}" ]; then
  IFS='|' read -ra KS <<< "$KNOBS"
  for r in 1 2 3; do
    for kv in "${KS[@]}"; do
      tag=$(echo "$kv" | tr ' =' '__')
      step knob_${tag}_$r.json 200 env $kv python bench.py $B
      echo "$kv r$r -> $(python -c "import json,sys;d=json.loads(open('$OUT/knob_${tag}_$r.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],5), round(d['roofline']['kernel_ms'],5), d.get('snapshot_handoff'))")"
    done
  done
fi
if [ -n "${VARIANTS:-}" ]; then
  step ab.txt 900 bash tools/gpu_ab_swap.sh "$B" $VARIANTS
  cp -r gpurun_out/abs $OUT/abs 2>/dev/null; tail -12 $OUT/ab.txt
fi
if [ -n "${TIMELINES:-}" ]; then
  IFS='|' read -ra TS <<< "$TIMELINES"
  i=0
  for kv in "${TS[@]}"; do
    i=$((i+1)); d=$OUT/tl$i; mkdir -p $d
    echo "$kv" > $d/mode.txt
    step tl$i.log 300 env $kv rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 80 --warmup 10 --policy-steps 0 --no-cpu-baseline
    f=$(find $d -name "*kernel_trace.csv" | head -1)
    python3 tools/trace_timeline.py "$f" > $d/timeline.txt 2>&1; tail -12 $d/timeline.txt
  done
fi
if [ "${ACT:-0}" = "1" ]; then  # the acting kernel: 64 vs 128 env rows per block, interleaved
  for r in 1 2; do
    for tm in 64 128; do
      step act_${tm}_$r.txt 200 env FLOCK_ACT_TM=$tm python3 tools/act_bench.py
      echo "TM=$tm r$r: $(tail -1 $OUT/act_${tm}_$r.txt)"
    done
  done
fi
if [ "${DRIVER:-0}" = "1" ]; then
  step driver_1.json 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
  step driver_2.json 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
  for f in driver_1 driver_2; do python3 -c "import json;d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]);print('$f', round(d['ms_per_step'],5), '%.4g'%d['value'], d.get('snapshot_handoff'))"; done
fi
echo ALLDONE
