#!/bin/bash
# Config 3 with and without the env kernel's L2 pull-ahead (FLOCK_ENV_PF=0 off, -1 the default: on in the one-launch
# step, i.e. the kernel-alone probe), interleaved. Outputs gpurun_out/c3pf/. (The round-4 A/B in profiles/r04/pf/ ran
# an earlier knob layout: 1 = the one-launch pull, 2 = also across the step's three launches, since removed.)
set -u
O=gpurun_out/c3pf; mkdir -p $O
summ() { python -c "import sys,json; l=[x for x in open('$1').read().splitlines() if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']; print('$1', 'ms/step %.4f kernel_ms %.4f frac %.4f alone %.4f frac_alone %.4f' % (d['ms_per_step'], r['kernel_ms'], r['frac'], r['kernel_alone_ms'], r['frac_alone']))"; }
for rep in 1 2; do
  for m in 0 -1; do
    FLOCK_ENV_PF=$m timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 200 --warmup 20 > $O/bench3_pf${m}_$rep.json 2>&1 || { tail -20 $O/bench3_pf${m}_$rep.json; exit 1; }
    summ $O/bench3_pf${m}_$rep.json
  done
done
