#!/bin/bash
# Config-3 step time against the learner GEMM K-chunk knobs (FLOCK_GEMM_KC: forward / input-gradient GEMMs,
# FLOCK_GRAD_KC: the weight-gradient GEMMs), two interleaved passes. Output gpurun_out/kc/
O=gpurun_out/kc; mkdir -p $O
for r in 1 2; do for kc in "200 128" "128 128" "104 128" "256 128" "200 64" "200 200"; do
  set -- $kc
  FLOCK_GEMM_KC=$1 FLOCK_GRAD_KC=$2 timeout -k 10 120 python bench.py --steps 300 --no-cpu-baseline --policy-steps 0 > $O/kc_$1_$2_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('$O/kc_$1_$2_$r.json').read().strip().splitlines()[-1]);print('fwd_kc $1 grad_kc $2', 'ms/step %.4f'%d['ms_per_step'])"
done; done
