#!/bin/bash
# Config-5 env-kernel variants (pull placement, non-temporal streams; tools/mk_variant.sh trees): interleaved A/B,
# then FETCH_SIZE / WRITE_SIZE passes (one counter per run) of the trees in PMC_TREES. Output: gpurun_out/c5pull/.
set -o pipefail
O=$PWD/gpurun_out/c5pull; mkdir -p $O
ABT_OUT=c5pull/ab TREES="$TREES" bash tools/gpu_ab_trees.sh ${REPS:-2} "--config 5 --no-cpu-baseline" || exit 1
for t in $PMC_TREES; do
  d=_ab/$t; [ $t = cur ] && d=.
  for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd $d && timeout -k 10 240 rocprofv3 --pmc $ctr -d $O/pmc_${t}_$ctr -o run --output-format csv -- python3 bench.py --config 5 --no-cpu-baseline --steps 30 --warmup 3 --step-launches 1 > $O/pmc_${t}_$ctr.log 2>&1) || { echo "pmc $t $ctr failed"; tail -5 $O/pmc_${t}_$ctr.log; exit 1; }
  done
  python tools/pmc_traffic.py $O/pmc_${t}_FETCH_SIZE $O/pmc_${t}_WRITE_SIZE --kernel step_kernel --algorithmic-bytes $(( (93 + 64) * 1024 * 16384 )) --out $O/pmc_$t.json && cat $O/pmc_$t.json && echo
done
echo ALLDONE
