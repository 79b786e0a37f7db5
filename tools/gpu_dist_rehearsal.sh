#!/bin/bash
# Rehearsal of bench.py's N > 1 path on ONE GPU (gloo, NPROC ranks on cuda:0, default 2): the barrier, max-over-ranks
# timing, the global env split (configs 4 / 5) and the multi-rank learners (data-parallel shared critic, agent-sharded
# MADDPG critics) run end to end. Not a scaling measurement. Outputs under gpurun_out/rehearsal$NPROC/.
set -u
NP=${NPROC:-2}
OUT=gpurun_out/rehearsal$NP; mkdir -p $OUT
export FLOCK_DIST_BACKEND=gloo
run() { local name=$1; shift; timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP \
  --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus $NP --no-cpu-baseline "$@" \
  > $OUT/$name.json 2> $OUT/$name.err; local rc=$?; echo "rc($name)=$rc"; tail -c 700 $OUT/$name.json; echo;
  [ $rc -eq 0 ] || { tail -20 $OUT/$name.err; exit $rc; }; }
for c in ${CONFIGS:-3 5 4}; do
  case $c in
    3) run config3 --config 3 --steps 40 --warmup 5 ;;
    5) run config5 --config 5 --steps 250 --warmup 5 ;;
    4) run config4 --config 4 --steps 150 --warmup 5 ;;
  esac
done
