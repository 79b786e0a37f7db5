#!/bin/bash
# env step alone / learner alone / both per tree (r5c vs cur), interleaved
set -o pipefail
O=gpurun_out/it4b; mkdir -p $O
for r in 1 2 3; do
  for t in r5c cur; do
    d=$PWD/_ab/$t; [ $t = cur ] && d=$PWD
    FLOCK_TREE=$d timeout -k 10 120 python tools/round_alone.py > $O/alone_${t}_$r.txt 2>&1 || { tail $O/alone_${t}_$r.txt; exit 1; }
    echo "$t rep $r: $(grep us/call $O/alone_${t}_$r.txt | tr -s ' ' | tr '\n' ';')"
  done
done
