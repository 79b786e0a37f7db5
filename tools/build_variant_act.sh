#!/bin/bash
# Build an A/B variant of libflock_amd.so with extra defines for flock_act.hip (diagnostics).
#   tools/build_variant_act.sh NAME -DFOO ...   ->  marl_range_flocking_amd/_build/libflock_amd_NAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
B=marl_range_flocking_amd/_build
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 "$@" -c -I include \
    -o $B/flock_act_$name.o marl_range_flocking_amd/csrc/flock_act.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -shared -o $B/libflock_amd_$name.so \
    $B/flock_env.hip.o $B/flock_act_$name.o $B/flock_learn.hip.o $B/flock_sc.hip.o
