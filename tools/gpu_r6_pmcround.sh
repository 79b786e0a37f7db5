#!/bin/bash
# Round 6: PMC counters of the learner round's kernels (counter collection serialises dispatches: each kernel alone):
# MFMA busy and L2 hit / miss per kernel. One counter group per rocprofv3 pass.
set -o pipefail
O=gpurun_out/r6pmc; mkdir -p $O; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/sq -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --policy-steps 0 > $O/sq.log 2>&1 || { tail $O/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/tcc -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --policy-steps 0 > $O/tcc.log 2>&1 || { tail $O/tcc.log; exit 1; }
python tools/pmc_round.py $O/sq $O/tcc | tee $O/summary.txt
