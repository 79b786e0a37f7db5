#!/bin/bash
# Round 5: fused Adam variants (tools/mk_variant.sh trees: nt = non-temporal streams, u2 = two float4 per thread
# and iteration) against this tree at config 5's critic size, interleaved.
set -o pipefail
O=gpurun_out/adam; mkdir -p $O
for r in 1 2; do
  for t in ${ADAM_TREES:-cur nt u2 ntu2}; do
    d=_ab/$t; [ $t = cur ] && d=.
    [ -d $d/marl_range_flocking_amd ] || { echo "no tree $d"; exit 1; }
    FLOCK_ROOT=$PWD/$d timeout -k 10 120 python tools/adam_bw.py > $O/${t}_$r.txt 2>&1 || { cat $O/${t}_$r.txt; exit 1; }
    echo "$t rep $r: $(tr '\n' ' ' < $O/${t}_$r.txt)"
  done
done
