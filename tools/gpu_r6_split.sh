#!/bin/bash
# CU-partition probe: learner stream on X CU bits, env stream on the complement (tools/learner_mask_probe.py MODE=split)
set -o pipefail
O=gpurun_out/r6split; mkdir -p $O
MODE=split KEEP=${KEEP:-32,64,96,128} REPS=${REPS:-2} timeout -k 10 500 python tools/learner_mask_probe.py > $O/split.txt 2>&1 || { tail -20 $O/split.txt; exit 1; }
cat $O/split.txt
