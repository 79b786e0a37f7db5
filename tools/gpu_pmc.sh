#!/bin/bash
# PMC traffic passes for the bench kernel (separate FETCH_SIZE / WRITE_SIZE runs; kernel-trace stats run).
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-}
TAG=${TAG:-v2_N256_E4096}
ALG=${ALG:-97517568}
run() { local name=$1; shift; timeout -k 10 600 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc($name)=$rc"; tail -n 3 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run pmc_fetch rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 30 --warmup 3 $ARGS
run pmc_write rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 30 --warmup 3 $ARGS
run stats rocprofv3 --kernel-trace --stats -d $OUT/prof_stats -o run --output-format csv -- python bench.py --no-cpu-baseline $ARGS
python tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write --kernel step_kernel --algorithmic-bytes $ALG --out $OUT/pmc_$TAG.json
echo ALLDONE
