#!/bin/bash
# HISTORICAL (round 6): the knob this A/B sets was removed after it measured slower; flock_set_diag now rejects it, so the script fails fast against the current tree.
# Round 6: forward GEMMs as 32 x 64 tiles (flock_set_diag sc_fwd_wide 1) against 32 x 32: the pipeline tests, the
# per-kernel durations of a short traced loop each, and an interleaved config-3 A/B (200 steps + the driver command)
set -o pipefail
O=gpurun_out/r6wide; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for w in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$w -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 --diag-knob sc_fwd_wide=$w > $O/prof$w.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  grep -h "sc_gemm\|sc_k3\|sc_k1\|step_kernel" $(find $O/prof$w -name "*kernel_stats.csv") | cut -d, -f1-4
done
for r in 1 2 3; do for w in 0 1; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 --diag-knob sc_fwd_wide=$w > $O/s200_${w}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 --diag-knob sc_fwd_wide=$w > $O/drv_${w}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json,sys; [print(f.split('/')[-1], round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5)) for f in sys.argv[1:]]" $O/s200_${w}_$r.json $O/drv_${w}_$r.json
done; done
