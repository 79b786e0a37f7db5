#!/bin/bash
# A/B of the device-side snapshot gate (default) against the cross-queue event wait (FLOCK_SC_GATE=0), same build,
# interleaved, config 3 (three env launches). Then the pipeline tests.
O=gpurun_out/gate; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_torch_ops.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for g in 1 0; do
  FLOCK_SC_GATE=$g timeout -k 10 120 python bench.py --steps 300 --no-cpu-baseline --policy-steps 0 > $O/g${g}_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('$O/g${g}_$r.json').read().strip().splitlines()[-1]);print('gate=$g', 'ms/step %.4f'%d['ms_per_step'], 'host %.4f'%d.get('host_ms_per_step',0))"
done; done
