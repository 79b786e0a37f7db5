#!/bin/bash
# Round-4 iteration: selected GPU tests, then a same-box A/B of library variants on the config-3 bench.
#   TESTS="..." pytest targets ("none" skips); VARIANTS="name ..." libflock_amd_<name>.so variants ("" skips the A/B)
set -u
OUT=gpurun_out/r4iter; mkdir -p $OUT; export TMPDIR=/tmp
TESTS=${TESTS:-"tests -m gpu"}
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name 2>&1; local rc=$?; echo "rc($name)=$rc";
  if [ $rc -ne 0 ]; then tail -40 $OUT/$name; exit $rc; fi; }
if [ "$TESTS" != "none" ]; then
  step pytest.txt 900 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread
  grep -E "passed|failed" $OUT/pytest.txt | tail -3
fi
if [ -n "${KNOBS:-}" ]; then  # interleaved env-var A/B, 3 rounds: KNOBS="FLOCK_SC_GATE=0|FLOCK_SC_GATE=1"
  IFS='|' read -ra KS <<< "$KNOBS"
  for r in 1 2 3; do
    for kv in "${KS[@]}"; do
      tag=$(echo "$kv" | tr ' =' '__')
      env $kv timeout -k 10 200 python bench.py ${BENCH:---steps 200 --warmup 20 --policy-steps 0 --no-cpu-baseline} > $OUT/knob_${tag}_$r.json 2> $OUT/knob_${tag}_$r.err || { echo "FAIL $kv"; tail -5 $OUT/knob_${tag}_$r.err; exit 1; }
      echo "$kv r$r -> $(grep -o "\"ms_per_step\": [0-9.]*\|\"kernel_ms\": [0-9.]*\|\"snapshot_handoff\": \"[a-z ]*" $OUT/knob_${tag}_$r.json | tr "\n" " ")"
    done
  done
fi
if [ -n "${VARIANTS:-}" ]; then
  step ab.txt 900 bash tools/gpu_ab_swap.sh "${BENCH:---steps 200 --warmup 20 --policy-steps 0 --no-cpu-baseline}" $VARIANTS
  tail -20 $OUT/ab.txt
fi
echo ALLDONE
