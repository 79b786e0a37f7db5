#!/bin/bash
# Longer runs as a stability check (the device gate's error word is checked after the timed region by bench.py):
# config 3 with 3000 timed steps, config 4 with 1500, config 5 with 1000 (gpurun_out/long/).
set -u
O=${LONG_OUT:-gpurun_out/long}; mkdir -p $O
for a in "3 3000" "4 1500" "5 1000"; do
  set -- $a
  timeout -k 10 300 python bench.py --config $1 --steps $2 --warmup 20 --no-cpu-baseline --policy-steps 0 > $O/config$1.json 2> $O/config$1.err || { tail -20 $O/config$1.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/config$1.json').read().strip().splitlines()[-1]); print('config $1', d['steps'], 'steps', 'ms/step %.4f' % d['ms_per_step'], '%.4g' % d['value'])"
done
echo ALLDONE
