#!/bin/bash
# The whole GPU suite, smoke, and the config 3 / 4 / 5 bench lines of this tree (gpurun_out/suite2/).
set -u
O=gpurun_out/suite2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
for c in 3 4 5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_config$c.json 2> $O/bench_config$c.err || { tail -20 $O/bench_config$c.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_config$c.json').read().strip().splitlines()[-1]); print('config $c', 'ms/step %.4f' % d['ms_per_step'], '%.4g' % d['value'], 'env launch %.4f' % d['roofline']['kernel_ms'], 'alone', d['roofline'].get('kernel_alone_ms'))"
done
echo ALLDONE
