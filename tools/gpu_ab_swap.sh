#!/bin/bash
# Same-box A/B of libflock_amd.so variants on the bench path that libflock_torch.so links (ScTrainLoop): each run
# copies _build/libflock_amd_<NAME>.so over _build/libflock_amd.so ("base" = the tree's own build), interleaved.
# Usage: tools/gpu_ab_swap.sh "bench args" NAME...   (results in gpurun_out/abs/)
set -o pipefail
B=$PWD/marl_range_flocking_amd/_build
O=$PWD/gpurun_out/abs
mkdir -p $O
args=$1; shift
cp $B/libflock_amd.so $B/libflock_amd_base.so
for r in 1 2 3; do
  for v in base "$@"; do
    cp $B/libflock_amd_$v.so $B/libflock_amd.so
    timeout -k 10 200 python bench.py $args > $O/${v}_$r.json 2> $O/${v}_$r.err || { cp $B/libflock_amd_base.so $B/libflock_amd.so; exit 1; }
  done
done
cp $B/libflock_amd_base.so $B/libflock_amd.so
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/abs/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f.split("/")[-1], "ms/step %.4f" % d["ms_per_step"], "kernel_ms %.4f" % r.get("kernel_ms", 0),
          "alone_ms %.4f" % (r.get("kernel_alone_ms") or 0), "value %.3e" % d["value"])
PY
