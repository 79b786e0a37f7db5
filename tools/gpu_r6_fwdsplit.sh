#!/bin/bash
# HISTORICAL (round 6): the knob this A/B sets was removed after it measured flat / slower; flock_set_diag now rejects it, so the script fails fast against the current tree.
# Round 6: forward GEMM K slices (flock_set_diag sc_fwd_split 1 / 2 / 4): the pipeline tests, an interleaved config-3
# A/B (driver command + 200 steps) and a kernel trace of each
set -o pipefail
O=gpurun_out/r6fsplit; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do for S in 1 2 4; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 --diag-knob sc_fwd_split=$S > $O/drv_${S}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 --diag-knob sc_fwd_split=$S > $O/s200_${S}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json,sys; [print(f, round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5)) for f in sys.argv[1:]]" $O/drv_${S}_$r.json $O/s200_${S}_$r.json
done; done
for S in 1 2 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$S -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 --diag-knob sc_fwd_split=$S > $O/prof$S.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
done
find $O -name "*kernel_stats.csv" | sort
