#!/bin/bash
# Kernel traces of the data-parallel loop at one rank over RCCL: the unsplit and the split rounds (direct RCCL)
# (gpurun_out/splittrace/).
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/splittrace; mkdir -p $O
for v in "DP unsplit, RCCL:unsplit" "DP split, RCCL:split"; do
  name=${v%%:*}; tag=${v##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- python3 tools/rccl_host_cost.py --only "$name" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  grep "per step" $O/$tag.log
done
echo ALLDONE
