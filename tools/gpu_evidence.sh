#!/bin/bash
# Round evidence in one GPU session: GPU tests, smoke, every config's bench line + rocprofv3 kernel stats.
# Outputs under gpurun_out/ev/ (copy into profiles/rNN/).
set -u
OUT=gpurun_out/ev; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name 2>&1; local rc=$?; echo "rc($name)=$rc"; \
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP"; exit $rc; fi; }
run pytest_gpu.txt 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run smoke.txt 300 python -c "import __graft_entry__ as g; g.smoke()"
for c in 3 2 4 5; do
  run bench_config$c.txt 300 python bench.py --config $c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c$c -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline > $OUT/prof_c$c.txt 2>&1
  echo "rc(prof $c)=$?"
done
echo ALLDONE
