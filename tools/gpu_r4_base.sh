#!/bin/bash
# Round-4 baseline on one box: the driver's exact bench command next to longer runs, so the driver's 0.0916 ms and the
# builder's 0.082 ms per step can be compared on the same box (verdict r3 item 5), and the learner round alone.
set -u
OUT=gpurun_out/r4base; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$name 2>&1; local rc=$?; echo "rc($name)=$rc";
  if [ $rc -ne 0 ]; then tail -25 $OUT/$name; exit $rc; fi; }
step driver_cmd.json 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
for i in 1 2; do
  step short_$i.json 200 python3 bench.py --steps 20 --warmup 5 --policy-steps 0 --no-cpu-baseline
  step long_$i.json 200 python3 bench.py --steps 200 --warmup 20 --policy-steps 0 --no-cpu-baseline
  step shortw_$i.json 200 python3 bench.py --steps 20 --warmup 200 --policy-steps 0 --no-cpu-baseline
done
step round_alone.txt 200 python3 tools/round_alone.py
python3 - <<'EOF'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4base/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f, d["steps"], d["warmup"], round(d["ms_per_step"], 5), round(d["roofline"]["kernel_alone_ms"], 5))
    except Exception as e:
        print(f, "?", e)
EOF
cat $OUT/round_alone.txt
echo ALLDONE
