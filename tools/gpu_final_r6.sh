#!/bin/bash
# Round-6 final evidence (gpurun_out/ev6/): GPU suite + smoke (tools/gpu_evidence_r5.sh phase tests), config 2's
# rollout-kernel PMC traffic passes, every config's bench line with rocprofv3 kernel stats, the driver's own command
# twice with its rocprofv3 profile
# Two gpurun calls: PHASES=tests (GPU suite + smoke), then PHASES="pmc bench driver" (the default)
set -u
OUT=gpurun_out/ev6; mkdir -p $OUT; export TMPDIR=/tmp
(while true; do date >> $OUT/heartbeat.txt; sleep 30; done) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
P=${PHASES:-pmc bench driver}
if [[ $P == *tests* ]]; then EV_OUT=$OUT PHASES=tests bash tools/gpu_evidence_r5.sh || exit 1; fi
if [[ $P == *pmc* ]]; then
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/pmc_rollout_$ctr -o run --output-format csv -- python3 bench.py --config 2 --no-cpu-baseline --steps 100 --warmup 50 > $OUT/pmc_rollout_$ctr.log 2>&1 || { tail $OUT/pmc_rollout_$ctr.log; exit 1; }
done
python tools/pmc_traffic.py $OUT/pmc_rollout_FETCH_SIZE $OUT/pmc_rollout_WRITE_SIZE --kernel rollout_uw_kernel --algorithmic-bytes $((77 * 64 * 1024 * 50)) --steps-per-launch 50 --out $OUT/pmc_uw_rollout_N64_E1024.json || exit 1
cp $OUT/pmc_uw_rollout_N64_E1024.json profiles/
fi
P2=${P//tests/}; P2=${P2//pmc/}
if [ -n "${P2// /}" ]; then EV_OUT=$OUT PHASES="$P2" CONFIGS="${CONFIGS:-3 2 4 5}" bash tools/gpu_evidence_r5.sh || exit 1; fi
echo ALLDONE6
