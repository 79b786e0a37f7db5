#!/bin/bash
# VALU issue PMC pass of the config-3 env kernel (one launch per step) for library variants (swapped over
# _build/libflock_amd.so, "base" = the tree's build). Output: gpurun_out/vab/pmc_<name>.json
set -u
OUT=gpurun_out/vab; mkdir -p $OUT; export TMPDIR=/tmp
B=$PWD/marl_range_flocking_amd/_build
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"
cp $B/libflock_amd.so $B/libflock_amd_base.so
for v in base "$@"; do
  cp $B/libflock_amd_$v.so $B/libflock_amd.so
  timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/pmc_$v -o run --output-format csv -- python3 bench.py --config 3 --no-cpu-baseline --steps 30 --warmup 3 --step-launches 1 --policy-steps 0 > $OUT/pmc_$v.log 2>&1 || { tail -5 $OUT/pmc_$v.log; cp $B/libflock_amd_base.so $B/libflock_amd.so; exit 1; }
  python tools/pmc_sq_json.py $OUT/pmc_$v --kernel step_kernel --out $OUT/pmc_$v.json > /dev/null
  python -c "import json;d=json.load(open('$OUT/pmc_$v.json'));w=d['SQ_WAVES'];print('$v', 'valu/wave %.1f'%(d['SQ_INSTS_VALU']/w), 'act %.0f act2 %.0f'%(d['SQ_ACTIVE_INST_VALU'],d['SQ_ACTIVE_INST_VALU2']), 'wave_cyc/wave %.0f'%(d['SQ_WAVE_CYCLES']/w), 'wait_any %.2f'%(d['SQ_WAIT_ANY']/d['SQ_WAVE_CYCLES']), 'grbm %.0f'%d['GRBM_GUI_ACTIVE'])"
done
cp $B/libflock_amd_base.so $B/libflock_amd.so
