#!/bin/bash
# Round 6: the GRU-recurrence row chunks, the multi-rank GPU tests (gloo ranks on one GPU, world 2 / 4 / 8), the
# pipeline and overlapped-train tests, configs 4 / 5 once, then the bench's N > 1 path rehearsed with 8 and 4 gloo
# ranks on the one GPU (not a scaling number). A heartbeat file keeps the silence
# watchdog informed while the 8-rank tests run (their ranks print nothing for minutes).
set -o pipefail
O=gpurun_out/r6dist; mkdir -p $O; export TMPDIR=/tmp
(while true; do date >> $O/heartbeat.txt; sleep 30; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests/test_gpu_dist.py tests/test_gpu_learn_kernels.py tests/test_gpu_overlap.py tests/test_gpu_train_loop.py tests/test_gpu_overlap_train.py} -x -v --durations=15 --timeout ${PT_TIMEOUT:-600} --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -20 $O/pytest.txt
[ -n "${ONLY_TESTS:-}" ] && exit 0
for c in 4 5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_c$c.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['value'])" $O/bench_c$c.json
done
NPROC=8 CONFIGS="3 5 4" bash tools/gpu_dist_rehearsal.sh || exit 1
NPROC=4 CONFIGS="3" bash tools/gpu_dist_rehearsal.sh || exit 1
