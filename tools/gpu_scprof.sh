#!/bin/bash
# Per-block learner-round timeline (tools/sc_block_prof.py) with the -DFLOCK_SC_PROF build swapped in for
# _build/libflock_amd.so (the torch ops link it), alone and beside env steps; restores the build after.
set -u
B=$PWD/marl_range_flocking_amd/_build; O=gpurun_out/scprof; mkdir -p $O
cp $B/libflock_amd.so $B/libflock_amd_base.so && cp $B/libflock_amd_scprof.so $B/libflock_amd.so
SWAPPED=1 timeout -k 10 200 python tools/sc_block_prof.py > $O/alone.txt 2>&1; r1=$?
SWAPPED=1 timeout -k 10 200 python tools/sc_block_prof.py --corun > $O/corun.txt 2>&1; r2=$?
cp $B/libflock_amd_base.so $B/libflock_amd.so
grep -v "^    blocks" $O/alone.txt; grep -v "^    blocks" $O/corun.txt
exit $((r1 | r2))
