#!/bin/bash
# Run named GPU steps, each under its own timeout; stop at the first crash / timeout / abort (any exit code other
# than 0 = ok and 1 = test failures). Usage: tools/gpu_steps.sh "name|timeout|cmd" ...
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  echo "== $name"
  timeout -k 10 "$t" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "rc($name)=$rc"; tail -n 8 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
done
echo ALLDONE
