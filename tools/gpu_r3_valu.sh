#!/bin/bash
# VALU roofline evidence (round 3), outputs under gpurun_out/valu/ (copy the summaries into profiles/):
#   1. tools/ubench_valu: cycles per wave64 instruction per SIMD of the env kernel's opcodes -> ubench_valu.json
#   2. the same ubench under one PMC pass (SQ_ACTIVE_INST_VALU / _VALU2 per opcode kernel: what the dual-issue
#      counter means on a known instruction stream)
#   3. two SQ passes of the config-3 env kernel (one launch per step): the VALU class mix and the issue counters
# PHASES="ubench pmc bench tests" selects parts; CONFIGS="3 2 4 5" the configs of the PMC passes.
set -u
OUT=gpurun_out/valu; mkdir -p $OUT; export TMPDIR=/tmp
PHASES=${PHASES:-"ubench pmc"}
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name 2>&1; local rc=$?; echo "rc($name)=$rc";
  if [ $rc -ne 0 ]; then tail -20 $OUT/$name; exit $rc; fi; }
tag_of() { case $1 in 3) echo v2_ring_N256_E4096;; 2) echo uw_N64_E1024;; 4) echo uw_discrete_ring_N512_E8192;;
  5) echo v2_ring_N1024_E16384;; esac; }
PASS_A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE"
PASS_B="SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
if [[ $PHASES == *tests* ]]; then
  step pytest_gpu.txt 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
  tail -2 $OUT/pytest_gpu.txt
fi
if [[ $PHASES == *ubench* ]]; then
  [ -x tools/ubench_valu ] || hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -o tools/ubench_valu tools/ubench_valu.hip
  step ubench_valu.json 120 tools/ubench_valu
  step ubench_pmc.log 120 rocprofv3 --pmc $PASS_B -d $OUT/ubench_pmc -o run --output-format csv -- tools/ubench_valu
  python tools/ubench_summary.py $OUT/ubench_valu.json $OUT/ubench_pmc --out $OUT/ubench_valu_merged.json > /dev/null
fi
if [[ $PHASES == *bench* ]]; then
  step bench_config3.json 300 python bench.py --config 3
  tail -c 1500 $OUT/bench_config3.json; echo
fi
if [[ $PHASES == *pmc* ]]; then
  for c in ${CONFIGS:-3}; do
    t=$(tag_of $c)
    step pmc_valuA_$t.log 240 rocprofv3 --pmc $PASS_A -d $OUT/pmc_valuA_$t -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --steps 30 --warmup 3 --step-launches 1
    step pmc_valuB_$t.log 240 rocprofv3 --pmc $PASS_B -d $OUT/pmc_valuB_$t -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --steps 30 --warmup 3 --step-launches 1
    python tools/pmc_sq_json.py $OUT/pmc_valuA_$t $OUT/pmc_valuB_$t --kernel step_kernel --out $OUT/pmc_valu_$t.json
  done
fi
echo ALLDONE
