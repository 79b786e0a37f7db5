#!/bin/bash
# Run GPU test files against a libflock_amd.so variant (copied over the tree's build for the run, restored after).
#   tools/gpu_variant_tests.sh NAME "tests/..." ; outputs gpurun_out/vtests/NAME.txt
set -u
B=$PWD/marl_range_flocking_amd/_build; O=gpurun_out/vtests; mkdir -p $O
name=$1; shift
cp $B/libflock_amd.so $B/libflock_amd_base.so
cp $B/libflock_amd_$name.so $B/libflock_amd.so
timeout -k 10 600 python -u -m pytest $@ -x -q --timeout 120 --timeout-method thread > $O/$name.txt 2>&1; rc=$?
cp $B/libflock_amd_base.so $B/libflock_amd.so
tail -3 $O/$name.txt
exit $rc
