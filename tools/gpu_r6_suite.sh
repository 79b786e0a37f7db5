#!/bin/bash
# Round 6: the GPU suite + smoke + driver-command bench lines on this tree (gpurun_out/r6suite/)
set -o pipefail
O=gpurun_out/r6suite${TAG}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.txt 2>&1 \
  || { tail -60 $O/pytest_gpu.txt; exit 1; }
tail -3 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/driver_$r.json 2> $O/driver_$r.err || { tail $O/driver_$r.err; exit 1; }
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 > $O/s200_$r.json 2> $O/s200_$r.err || { tail $O/s200_$r.err; exit 1; }
  python -c "import json,sys; [print(f, json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step']) for f in sys.argv[1:]]" $O/driver_$r.json $O/s200_$r.json
done
