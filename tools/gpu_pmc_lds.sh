#!/bin/bash
# LDS PMC pass of the config-3 env kernel (one launch per step): LDS instructions, bank-conflict and LDS-array
# cycles, issue stalls on LDS, against the waves' cycles. Output: gpurun_out/lds/pmc_lds_<tag>.json
set -u
OUT=gpurun_out/lds; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-base}
CTRS="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/pmc_$TAG -o run --output-format csv -- python3 bench.py --config 3 --no-cpu-baseline --steps 30 --warmup 3 --step-launches 1 --policy-steps 0 > $OUT/pmc_$TAG.log 2>&1 || { tail -5 $OUT/pmc_$TAG.log; exit 1; }
python tools/pmc_sq_json.py $OUT/pmc_$TAG --kernel step_kernel --out $OUT/pmc_lds_$TAG.json && cat $OUT/pmc_lds_$TAG.json
