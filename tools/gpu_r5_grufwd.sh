#!/bin/bash
# Round 5: the GRU recurrence kernels with each thread's rows' global operands loaded together (base = previous
# head in _ab/base): learner kernel tests in this tree, then config 4's kernel stats in both trees (rocprofv3) and an
# interleaved bench A/B.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/grufwd; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learn_kernels.py \
  tests/test_gpu_learners.py tests/test_gpu_learners_scale.py tests/test_gpu_overlap_train.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for t in base cur; do
  d=_ab/$t; [ $t = cur ] && d=.
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$t -o run --output-format csv -- python3 bench.py --config 4 --no-cpu-baseline > $O/bench_$t.json 2> $O/bench_$t.err) || exit 1
  python - $O/prof_$t <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("gru_seq", "vdn_feat", "step_kernel")):
        print(sys.argv[1].split("/")[-1], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
ABT_OUT=grufwd/ab TREES="base cur" bash tools/gpu_ab_trees.sh 3 "--config 4 --no-cpu-baseline"
