#!/bin/bash
# Diagnostics of the driver's 20-step line: a sleep kernel opening the timed region (the host enqueues
# ahead) and a GPU kept busy before the warmup (clock / power state). Outputs gpurun_out/ps_*.json.
for r in 1 2; do
for a in "--diag-presleep-us 0" "--diag-prewarm-ms 300" "--diag-prewarm-ms 1000"; do
  tag=$(echo "$a" | tr ' ' '_')
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --policy-steps 0 $a > gpurun_out/ps_${tag}_$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ps_${tag}_$r.json').read().strip().splitlines()[-1]);print('$a r$r ms/step', round(d['ms_per_step'],5), 'span', round(d['gpu_span_ms_per_step'],5), 'host', round(d['host_ms_per_step'],5))"
done; done
