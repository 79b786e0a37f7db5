#!/bin/bash
# Same-box A/B of bench.py lines: the tree in _prev/ (an earlier commit, exported with git archive and built in place)
# against this tree, interleaved. Usage: tools/gpu_ab_prev.sh [bench args...]   (results in gpurun_out/abp/)
set -o pipefail
O=$PWD/gpurun_out/abp
mkdir -p $O
for r in 1 2 3; do
  (cd _prev && timeout -k 10 200 python bench.py "$@" > $O/prev_$r.json 2> $O/prev_$r.err) || exit 1
  timeout -k 10 200 python bench.py "$@" > $O/cur_$r.json 2> $O/cur_$r.err || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/abp/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f.split("/")[-1], "ms/step %.4f" % d["ms_per_step"], "kernel_ms %.4f" % r.get("kernel_ms", 0),
          "alone_ms %.4f" % r.get("kernel_alone_ms", 0), "value %.3e" % d["value"])
PY
