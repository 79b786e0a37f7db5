#!/bin/bash
# One build -> measure iteration on the GPU box (run through gpurun from the repo root):
#   TESTS="tests/test_gpu_overlap.py ..."  pytest targets (default: the whole -m gpu suite; "none" skips)
#   BENCH="--config 3 ..."                  bench.py arguments (default: none = config 3; "none" skips)
#   TRACE=1                                 also a rocprofv3 kernel trace + stats of the same bench command
# Outputs under gpurun_out/iter/. Every GPU step has its own time limit; the script stops at the first failure.
set -u
OUT=gpurun_out/iter; mkdir -p $OUT; export TMPDIR=/tmp
TESTS=${TESTS:-"tests -m gpu"}
BENCH=${BENCH:-""}
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name 2>&1; local rc=$?; echo "rc($name)=$rc";
  if [ $rc -ne 0 ]; then tail -25 $OUT/$name; exit $rc; fi; }
if [ "$TESTS" != "none" ]; then
  step pytest.txt 600 python -u -m pytest $TESTS -q --timeout 120 --timeout-method thread
  tail -2 $OUT/pytest.txt
fi
if [ "$BENCH" != "none" ]; then
  step bench.json 300 python bench.py $BENCH --no-cpu-baseline
  tail -c 900 $OUT/bench.json; echo
  if [ "${TRACE:-0}" = "1" ]; then
    step trace.log 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $BENCH --no-cpu-baseline
  fi
fi
echo ALLDONE
