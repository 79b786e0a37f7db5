#!/bin/bash
# SQ instruction-mix pass for the bench kernel (one rocprofv3 --pmc run; <= 8 SQ counters)
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM -d $OUT/pmc_sq -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 30 --warmup 3 ${BENCH_ARGS:-} > $OUT/pmc_sq.log 2>&1
rc=$?; echo "rc(sq)=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/pmc_summary.py $OUT/pmc_sq --kernel step_kernel
