#!/bin/bash
# Round 6: the learner's ~7-us gap between rounds. Slots freed on the device (sc_gemm stores the consumed snapshot's
# number, the slot's next snapshot polls it; default) against a slot-free event recorded on the learner stream after
# every round (flock_set_diag sc_free_events 1, the round-5 scheme): the pipeline tests, kernel traces with the gap
# before each round listed, and an interleaved config-3 A/B (driver command + 200 steps)
set -o pipefail
O=gpurun_out/r6gaps; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_train_loop.py -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for f in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl$f -o run -- python bench.py --steps 80 --warmup 10 --policy-steps 0 --no-cpu-baseline --diag-knob sc_free_events=$f > $O/tl$f.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python tools/trace_timeline.py $(find $O/tl$f -name "*kernel_trace.csv") > $O/timeline_$f.txt && tail -16 $O/timeline_$f.txt
  python tools/round_gaps.py $(find $O/tl$f -name "*kernel_trace.csv") > $O/gaps_$f.txt && cat $O/gaps_$f.txt
done
for r in 1 2 3; do for f in 0 1; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 --diag-knob sc_free_events=$f > $O/drv_${f}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0 --diag-knob sc_free_events=$f > $O/s200_${f}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json,sys; [print(f, round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'], 5)) for f in sys.argv[1:]]" $O/drv_${f}_$r.json $O/s200_${f}_$r.json
done; done
