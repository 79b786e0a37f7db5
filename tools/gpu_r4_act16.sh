#!/bin/bash
# Round 4: 8-deep chunks / four blocks per CU for the 16 x 16 acting kernel, and the env kernel's L2 pull at config 3
# (outputs gpurun_out/r4a/): acting + pull parity tests, act_bench x3, config 3 bench (default) x2.
set -u
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_act.py tests/test_gpu_cells.py "tests/test_gpu_learners.py::test_shared_critic_choose_action_batched" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2 3; do echo "act r$r: $(timeout -k 10 120 python tools/act_bench.py 2>/dev/null | tail -1)"; done
summ() { python -c "import sys,json; l=[x for x in open('$1').read().splitlines() if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']; pil=d.get('policy_in_loop') or {}; print('$1', 'ms/step %.4f kernel_ms %.4f frac %.4f alone %.4f frac_alone %.4f act_frac %s' % (d['ms_per_step'], r['kernel_ms'], r['frac'], r['kernel_alone_ms'], r['frac_alone'], pil.get('act_mfma_frac')))"; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 200 --warmup 20 > $O/bench3_$r.json 2>&1 || { tail -20 $O/bench3_$r.json; exit 1; }
  summ $O/bench3_$r.json
done
