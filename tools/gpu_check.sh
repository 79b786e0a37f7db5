#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile. Each GPU step under its own timeout; stop at
# the first crash/timeout/abort (exit codes other than 0 = ok and 1 = test failures).
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" ; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "rc($name)=$rc"; tail -n 5 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py ${BENCH_ARGS:-}
if [ -n "${PROFILE:-}" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu-baseline ${BENCH_ARGS:-}
fi
echo ALLDONE
