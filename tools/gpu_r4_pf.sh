#!/bin/bash
# Round 4: the env kernel's L2 pull-ahead and acting-kernel chunk variants (outputs gpurun_out/r4pf/).
#   parity tests (cells incl. the pull, fused inserts); config 5 default (pull on) vs FLOCK_ENV_PF=0; then
#   tools/gpu_c3_pf.sh (config 3) and tools/gpu_act_variants.sh (acting kernel variants) when PHASES asks.
set -u
O=gpurun_out/r4pf; mkdir -p $O
PHASES=${PHASES:-"tests c5 c3 act"}
summ() { python -c "import sys,json; l=[x for x in open('$1').read().splitlines() if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']; print('$1', 'ms/step %.4f kernel_ms %.4f frac %.4f alone %.4f frac_alone %.4f' % (d['ms_per_step'], r['kernel_ms'], r['frac'], r['kernel_alone_ms'], r['frac_alone']))"; }
if [[ $PHASES == *tests* ]]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cells.py tests/test_gpu_learners.py -k "fused or pull or cell or spec or seeded" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
  tail -1 $O/tests.txt
fi
if [[ $PHASES == *c5* ]]; then
  for rep in 1 2; do
    for m in -1 0; do
      FLOCK_ENV_PF=$m timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > $O/bench5_pf${m}_$rep.json 2>&1 || { tail -20 $O/bench5_pf${m}_$rep.json; exit 1; }
      summ $O/bench5_pf${m}_$rep.json
    done
  done
fi
if [[ $PHASES == *c3* ]]; then bash tools/gpu_c3_pf.sh || exit 1; fi
if [[ $PHASES == *act* ]]; then bash tools/gpu_act_variants.sh kc8 kc8w4 kc24w2 kc16w2 || exit 1; fi
