#!/bin/bash
# Round 6: sparse slot-free events (n_slots >= 5): the pipeline tests, then interleaved config-3 A/B of 3 / 6 / 8 slots
set -o pipefail
O=gpurun_out/r6slots; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_train_loop.py -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2 3; do for n in 3 6 8; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 --sc-slots $n > $O/drv_${n}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 --sc-slots $n > $O/s200_${n}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json,sys; [print(f, round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5)) for f in sys.argv[1:]]" $O/drv_${n}_$r.json $O/s200_${n}_$r.json
done; done
