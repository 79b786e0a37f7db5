#!/bin/bash
# Round 6: the uw rollout kernel: its tests, config-2 bench lines (rollout 20 / 50 / single steps), rocprofv3 stats
set -o pipefail
O=gpurun_out/r6rollout; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_torch_ops.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for R in 20 50 0; do
  timeout -k 10 200 python bench.py --config 2 --rollout $R --no-cpu-baseline > $O/c2_r$R.json 2> $O/c2_r$R.err || { tail $O/c2_r$R.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], d['value'], r['kernel_ms'], r['frac'])" $O/c2_r$R.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config 2 --no-cpu-baseline > $O/c2_prof.json 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kstats_c2.csv; head -5 $O/kstats_c2.csv | cut -c1-200
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/pytest_dist.txt 2>&1 || { tail -40 $O/pytest_dist.txt; exit 1; }
tail -2 $O/pytest_dist.txt
