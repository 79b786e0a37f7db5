#!/bin/bash
# Config 3 with the env kernel's L2 pull-ahead (FLOCK_ENV_PF=1: the one-launch step, i.e. the kernel-alone probe;
# 5: also across the step's three launches), interleaved with the default. Outputs gpurun_out/c3pf/.
set -u
O=gpurun_out/c3pf; mkdir -p $O
summ() { python -c "import sys,json; l=[x for x in open('$1').read().splitlines() if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']; print('$1', 'ms/step %.4f kernel_ms %.4f frac %.4f alone %.4f frac_alone %.4f' % (d['ms_per_step'], r['kernel_ms'], r['frac'], r['kernel_alone_ms'], r['frac_alone']))"; }
for rep in 1 2; do
  for m in 0 1 5; do
    FLOCK_ENV_PF=$m timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 200 --warmup 20 > $O/bench3_pf${m}_$rep.json 2>&1 || { tail -20 $O/bench3_pf${m}_$rep.json; exit 1; }
    summ $O/bench3_pf${m}_$rep.json
  done
done
