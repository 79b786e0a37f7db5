#!/bin/bash
# PMC traffic (FETCH_SIZE, WRITE_SIZE: one pass each) of the env step kernel for BASELINE configs 2, 4, 5;
# outputs gpurun_out/pmc_<variant>[_ring]_N<N>_E<E>.json (copy into profiles/, where bench.py reads them)
set -u
OUT=gpurun_out/pmcc; mkdir -p $OUT; export TMPDIR=/tmp
pass() {  # config tag alg
  local c=$1 tag=$2 alg=$3
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr -d $OUT/${tag}_$ctr -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --steps 30 --warmup 3 > $OUT/${tag}_$ctr.log 2>&1
    local rc=$?; echo "rc($tag $ctr)=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python tools/pmc_traffic.py $OUT/${tag}_FETCH_SIZE $OUT/${tag}_WRITE_SIZE --kernel step_kernel --algorithmic-bytes $alg --out $OUT/pmc_$tag.json
}
# algorithmic bytes per launch: (SURVEY 8(d) bytes + the fused insert's bytes) x agents per launch
for c in ${CONFIGS:-3 2 4 5}; do
  case $c in
    3) pass 3 v2_ring_N256_E4096 $(( (93 + 64) * 256 * 4096 )) ;;
    2) pass 2 uw_N64_E1024 $(( 149 * 64 * 1024 )) ;;
    4) pass 4 uw_discrete_ring_N512_E8192 $(( (69 + 56) * 512 * 8192 )) ;;
    5) pass 5 v2_ring_N1024_E16384 $(( (93 + 96) * 1024 * 16384 )) ;;
  esac
done
echo ALLDONE
