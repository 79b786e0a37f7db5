#!/bin/bash
# Round 6: the bench's own timing markers on the env stream (FLOCK_BENCH_EV_EVERY: event pair every 4th step = the
# default, 16, 1000 = none in the timed region), interleaved; then one kernel + HIP API trace of the loop (host
# enqueue timing against the GPU timeline)
set -o pipefail
O=gpurun_out/r6ev; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do for e in 4 16 1000; do
  FLOCK_BENCH_EV_EVERY=$e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 > $O/drv_ev${e}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  FLOCK_BENCH_EV_EVERY=$e timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 > $O/s200_ev${e}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json,sys; [print(f, round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5)) for f in sys.argv[1:]]" $O/drv_ev${e}_$r.json $O/s200_ev${e}_$r.json
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/ht -o run -- python bench.py --steps 40 --warmup 10 --policy-steps 0 --no-cpu-baseline > $O/ht.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
ls $O/ht/*/ | head
