#!/bin/bash
# Round 4: the pull compiled only into the shapes that use it (outputs gpurun_out/r4pfm/): parity tests, then the
# config 4 / 5 / 3 bench lines with their rocprofv3 kernel stats.
set -u
O=gpurun_out/r4pfm; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cells.py tests/test_gpu_learners.py -k "fused or pull or cell or spec or seeded" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
summ() { python -c "import sys,json; l=[x for x in open('$1').read().splitlines() if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']; print('$1', 'value %.4g ms/step %.4f kernel_ms %.4f frac %.4f alone %.4f frac_alone %.4f' % (d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['kernel_alone_ms'] or 0, r['frac_alone'] or 0))"; }
for c in 4 5 3; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_config$c.json 2>&1 || { tail -20 $O/bench_config$c.json; exit 1; }
  summ $O/bench_config$c.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c$c -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline > $O/prof_c$c.log 2>&1 || exit 1
done
