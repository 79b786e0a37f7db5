#!/bin/bash
# Copy this working tree (sources, tests, bench; no _ab/, gpurun_out/, profiles/, .git) to _ab/<name>/ with
# compile-time defines prepended to one .hip file, and build it in place on the CPU, for a same-box A/B with
# tools/gpu_ab_trees.sh (TREES="<name> ... cur").
# Usage: tools/mk_variant.sh <name> <file under marl_range_flocking_amd/csrc> "DEF1=v" ["DEF2=v" ...]
set -eu
name=$1; file=$2; shift 2
d=_ab/$name
rm -rf "$d"; mkdir -p "$d"
tar --exclude=./_ab --exclude=./gpurun_out --exclude=./profiles --exclude=./.git --exclude='*.o' -cf - . | tar -xf - -C "$d"
mkdir -p $d/profiles; cp profiles/*.json $d/profiles/
f=$d/marl_range_flocking_amd/csrc/$file
tmp=$(mktemp)
for kv in "$@"; do echo "#define ${kv%%=*} ${kv#*=}" >> "$tmp"; done
cat "$f" >> "$tmp"; mv "$tmp" "$f"
(cd "$d" && python -c "from marl_range_flocking_amd import build; build.build(force=True)" > build.log 2>&1) || { tail -20 "$d/build.log"; exit 1; }
echo "built $d with $*"
