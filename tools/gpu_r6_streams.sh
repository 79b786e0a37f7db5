#!/bin/bash
# Round 6: stream placement (5 instances per process, own vs pool streams, high vs normal priority) and the CU split
set -o pipefail
O=gpurun_out/r6streams; mkdir -p $O
for m in "own high" "own normal" "pool high"; do
  set -- $m
  MODE=$1 PRIORITY=$2 GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python tools/stream_probe.py > $O/streams_$1_$2.txt 2>&1 || { tail -20 $O/streams_$1_$2.txt; exit 1; }
  grep instance $O/streams_$1_$2.txt
done
KEEP=${KEEP:-32,48,64} timeout -k 10 400 python tools/cu_split_probe.py > $O/split.txt 2>&1 || { tail -20 $O/split.txt; exit 1; }
cat $O/split.txt | grep -v amdgpu.ids
