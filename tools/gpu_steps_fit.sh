#!/bin/bash
# The bench's timed-region cost as a function of the step count K (verdict r3 item 5: the driver's 20-step line vs
# longer runs): K in $KS (default 10 20 40 200), warmup W in $WS (default 5, the driver's), $REPS runs each, interleaved; prints
# ms_per_step, the GPU-side span per step (HIP events at the region's ends) and the host enqueue time per step, then
# a least-squares fit el(K) = a + b K over the W = 5 runs. Extra bench args: $ARGS. Outputs: gpurun_out/stepsfit/.
set -u
OUT=gpurun_out/stepsfit; mkdir -p $OUT; export TMPDIR=/tmp
KS=${KS:-"10 20 40 200"}
for r in $(seq 1 ${REPS:-2}); do
  for w in ${WS:-5}; do
    for k in $KS; do
      f=$OUT/k${k}_w${w}_$r.json
      timeout -k 10 200 python3 bench.py --steps $k --warmup $w --no-cpu-baseline --policy-steps 0 ${ARGS:-} > $f 2> $OUT/k${k}_w${w}_$r.err || { echo "FAIL K=$k"; tail -5 $OUT/k${k}_w${w}_$r.err; exit 1; }
    done
  done
done
python3 - <<'EOF'
import glob, json
import numpy as np
ks, els = [], []
for f in sorted(glob.glob("gpurun_out/stepsfit/k*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    K = d["steps"]
    print(f"{f.split('/')[-1]:16s} K={K:4d} W={d['warmup']:4d} ms/step {d['ms_per_step']:.5f} gpu span/step {d.get('gpu_span_ms_per_step', 0):.5f} "
          f"host/step {d['host_ms_per_step']:.5f}")
    if d["warmup"] == 5:
        ks.append(K)
        els.append(d["ms_per_step"] * K)
A = np.stack([np.ones(len(ks)), np.array(ks, float)], 1)
(a, b), *_ = np.linalg.lstsq(A, np.array(els), rcond=None)
print(f"fit: el(K) = {a:.4f} ms + {b:.5f} ms x K")
EOF
echo ALLDONE
