#!/bin/bash
# Round evidence in one GPU session (outputs under gpurun_out/ev5/; copy the summaries into profiles/r05/):
#   GPU tests, smoke, every config's bench line + rocprofv3 kernel stats, and the env kernel's PMC passes
#   (FETCH_SIZE, WRITE_SIZE: one pass each, MI355X_MICROARCH.md; SQ instruction mix) -> pmc_*.json. The PMC passes
#   run the step as one launch (--step-launches 1), so a dispatch's counters are one whole step's.
# PHASES="tests bench pmc" selects parts. Every GPU step has its own time limit; the script stops at a failure.
set -u
OUT=${EV_OUT:-gpurun_out/ev5}; mkdir -p $OUT; export TMPDIR=/tmp
PHASES=${PHASES:-"tests pmc bench driver ab"}
PASS_A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE"
PASS_B="SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name 2>&1; local rc=$?; echo "rc($name)=$rc";
  if [ $rc -ne 0 ]; then tail -20 $OUT/$name; exit $rc; fi; }
tag_of() { case $1 in 3) echo v2_ring_N256_E4096;; 2) echo uw_N64_E1024;; 4) echo uw_discrete_ring_N512_E8192;;
  5) echo v2_ring_N1024_E16384;; esac; }
alg_of() { case $1 in 3) echo $(( (93 + 64) * 256 * 4096 ));; 2) echo $(( 149 * 64 * 1024 ));;
  4) echo $(( (69 + 56) * 512 * 8192 ));; 5) echo $(( (93 + 64) * 1024 * 16384 ));; esac; }
if [[ $PHASES == *tests* ]]; then
  step pytest_gpu.txt 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  tail -2 $OUT/pytest_gpu.txt
  step smoke.txt 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $PHASES == *pmc* ]]; then
  for c in ${CONFIGS:-3 2 4 5}; do
    t=$(tag_of $c)
    for ctr in FETCH_SIZE WRITE_SIZE; do  # (SQ VALU passes: tools/gpu_r3_valu.sh)
      step pmc_${t}_$ctr.log 240 rocprofv3 --pmc $ctr -d $OUT/pmc_${t}_$ctr -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --steps 30 --warmup 3 --step-launches 1
    done
    python tools/pmc_traffic.py $OUT/pmc_${t}_FETCH_SIZE $OUT/pmc_${t}_WRITE_SIZE --kernel step_kernel --algorithmic-bytes $(alg_of $c) --out $OUT/pmc_$t.json
    step pmc_sq_$t.log 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM -d $OUT/pmc_sq_$t -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --steps 30 --warmup 3 --step-launches 1
    python tools/pmc_sq_json.py $OUT/pmc_sq_$t --kernel step_kernel --out $OUT/pmc_sq_$t.json
    step pmc_valuA_$t.log 240 rocprofv3 --pmc $PASS_A -d $OUT/pmc_valuA_$t -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --steps 30 --warmup 3 --step-launches 1
    step pmc_valuB_$t.log 240 rocprofv3 --pmc $PASS_B -d $OUT/pmc_valuB_$t -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --steps 30 --warmup 3 --step-launches 1
    python tools/pmc_sq_json.py $OUT/pmc_valuA_$t $OUT/pmc_valuB_$t --kernel step_kernel --out $OUT/pmc_valu_$t.json
  done
  cp $OUT/pmc_*.json profiles/  # the bench lines below read them (copy them into the repo afterwards)
fi
if [[ $PHASES == *bench* ]]; then
  for c in ${CONFIGS:-3 2 4 5}; do
    if [ $c = 3 ]; then step bench_config$c.json 400 python bench.py --config $c; else step bench_config$c.json 400 python bench.py --config $c --no-cpu-baseline; fi
    tail -c 400 $OUT/bench_config$c.json; echo
    step prof_c$c.log 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_c$c -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline
  done
fi

# the driver's exact command twice (BENCH_rNN.json is one such line), and its rocprofv3 kernel summary
if [[ $PHASES == *driver* ]]; then
  step driver_1.json 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
  step driver_2.json 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
  step prof_driver.log 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_driver -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
fi
# same-box A/B of the round-3 head, the round-4 head and this tree (verdict r4 item 1), both commands
if [[ $PHASES == *ab* ]]; then
  ABT_OUT=ev5/ab TREES="89c4346 c2589f5 cur" tools/gpu_ab_trees.sh 3 \
    "--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0" \
    "--steps 200 --warmup 20 --no-cpu-baseline --policy-steps 0" || exit 1
fi
echo ALLDONE2
