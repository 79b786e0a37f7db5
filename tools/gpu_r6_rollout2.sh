#!/bin/bash
# Round 6: the rollout kernel at 2 vs 4 lanes per agent: tests, then interleaved config-2 bench lines
set -o pipefail
O=gpurun_out/r6rollout2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do for spl in 2 4; do for R in 20 50; do
  timeout -k 10 200 python bench.py --config 2 --rollout $R --no-cpu-baseline --diag-knob rollout_spl=$spl > $O/c2_s${spl}_r${R}_$r.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], round(d['ms_per_step']*1e3,3), '%.3g'%d['value'], round(r['kernel_ms']*1e3,3), round(r['frac'],3))" $O/c2_s${spl}_r${R}_$r.json
done; done; done
