#!/bin/bash
# Final-tree check: the whole GPU suite + smoke, the config-3 bench line, and the 2-rank rehearsal of the N > 1
# bench path (gloo on cuda:0; gpurun_out/suite3/, gpurun_out/rehearsal/).
set -u
O=gpurun_out/suite3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || { tail -20 $O/driver.err; exit 1; }
python -c "import json; d=json.loads(open('$O/driver.json').read().strip().splitlines()[-1]); print('driver', d['ms_per_step'], d['value'])"
CONFIGS=3 bash tools/gpu_dist_rehearsal.sh || exit 1
echo ALLDONE
