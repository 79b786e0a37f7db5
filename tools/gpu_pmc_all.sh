#!/bin/bash
# PMC evidence for the env step kernel of BASELINE configs: FETCH_SIZE and WRITE_SIZE (one pass each, TCC limits)
# and one SQ pass (<= 8 SQ counters). Writes gpurun_out/pmc/pmc_<tag>.json and pmc_sq_<tag>.json (copy into
# profiles/, where bench.py reads them).   CONFIGS="3 2 4 5" bash tools/gpu_pmc_all.sh
set -u
OUT=gpurun_out/pmc; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # tag args...
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 24 --warmup 3 $BARGS > $OUT/$tag.log 2>&1
  local rc=$?; echo "rc($tag)=$rc"; [ $rc -eq 0 ] || exit $rc
}
for c in ${CONFIGS:-3}; do
  case $c in
    2) tag=uw_N64_E1024; alg=9764864 ;;
    3) tag=v2_ring_N256_E4096; alg=164626432 ;;
    4) tag=uw_discrete_N512_E1024; alg=36175872 ;;
    5) tag=v2_ring_N1024_E2048; alg=396361728 ;;
  esac
  BARGS="--config $c ${EXTRA:-}"
  run ${tag}_fetch --pmc FETCH_SIZE -d $OUT/${tag}_fetch
  run ${tag}_write --pmc WRITE_SIZE -d $OUT/${tag}_write
  run ${tag}_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM -d $OUT/${tag}_sq
  python tools/pmc_traffic.py $OUT/${tag}_fetch $OUT/${tag}_write --kernel step_kernel --algorithmic-bytes $alg --out $OUT/pmc_$tag.json > /dev/null
  python tools/pmc_sq_json.py $OUT/${tag}_sq --kernel step_kernel --out $OUT/pmc_sq_$tag.json > /dev/null
done
echo ALLDONE
