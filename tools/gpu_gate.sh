# device-side snapshot gate of the learn() pipeline: bitwise pipeline tests, then bench A/B against the event waits
set -o pipefail
mkdir -p gpurun_out/gate
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_overlap.py tests/test_gpu_train_loop.py > gpurun_out/gate/pytest.txt 2>&1 || { tail -40 gpurun_out/gate/pytest.txt; exit 1; }
tail -2 gpurun_out/gate/pytest.txt
for r in 1 2 3; do
  for v in 0 1; do
    FLOCK_SC_GATE=$v timeout -k 10 200 python bench.py --steps 200 --policy-steps 0 --no-cpu-baseline > gpurun_out/gate/b_${v}_$r.json 2>gpurun_out/gate/b_${v}_$r.err || { tail -5 gpurun_out/gate/b_${v}_$r.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/gate/b_${v}_$r.json').read().strip().splitlines()[-1]);print('gate=$v', round(d['ms_per_step']*1000,2), 'us/step', round(d['roofline']['kernel_ms']*1000,1), 'env us')"
  done
done
