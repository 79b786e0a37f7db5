#!/bin/bash
# Same-box interleaved A/B of bench.py across source trees exported from earlier commits (git archive into _ab/<sha>/,
# built in place on the CPU) and this tree. Usage: tools/gpu_ab_trees.sh REPS "<bench args>" [more bench-arg sets...]
# Results: gpurun_out/abt/<set>_<tree>_<rep>.json, summary in gpurun_out/abt/summary.txt
set -o pipefail
O=$PWD/gpurun_out/${ABT_OUT:-abt}
mkdir -p $O
rm -f $O/s*_*.json
REPS=$1; shift
TREES="${TREES:-$(ls _ab) cur}"  # TREES="<sha> ... cur": a subset
s=0
for args in "$@"; do
  s=$((s + 1))
  for r in $(seq 1 $REPS); do
    for t in $TREES; do
      d=_ab/$t; [ $t = cur ] && d=.
      (cd $d && timeout -k 10 240 python bench.py $args > $O/s${s}_${t}_$r.json 2> $O/s${s}_${t}_$r.err) || exit 1
      echo "set $s ($args) tree $t rep $r done"
    done
  done
done
python - "$@" <<'PY' | tee $O/summary.txt
import json, glob, sys, collections
rows = collections.defaultdict(list)
import os
for f in sorted(glob.glob("gpurun_out/%s/s*_*.json" % os.environ.get("ABT_OUT", "abt"))):
    name = f.split("/")[-1][:-5]
    s, rest = name.split("_", 1)
    t, r = rest.rsplit("_", 1)
    d = json.loads(open(f).read().strip().splitlines()[-1])
    rows[(s, t)].append((d["ms_per_step"], (d.get("roofline") or {}).get("kernel_ms")))
for (s, t), v in sorted(rows.items()):
    ks = [k for _, k in v if k]
    print(f"{s} ({sys.argv[int(s[1:])]}) {t:8s} ms/step " + " ".join("%.4f" % x for x, _ in v) +
          "  min %.4f" % min(x for x, _ in v) + ("  env launch ms " + " ".join("%.4f" % k for k in ks) if ks else ""))
PY
