# fc1 folded into the forward GEMM (sc_gemm_fc1): shared-critic GPU tests, then bench A/B against the separate row launch
set -o pipefail
mkdir -p gpurun_out/fc1g
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_learners.py tests/test_gpu_overlap.py tests/test_gpu_train_loop.py tests/test_gpu_learners_scale.py tests/test_gpu_torch_ops_learn.py tests/test_gpu_dist.py > gpurun_out/fc1g/pytest.txt 2>&1 || { tail -40 gpurun_out/fc1g/pytest.txt; exit 1; }
tail -2 gpurun_out/fc1g/pytest.txt
for r in 1 2 3; do
  for v in 0 1; do
    FLOCK_SC_FC1_GEMM=$v timeout -k 10 200 python bench.py --steps 200 --policy-steps 0 --no-cpu-baseline > gpurun_out/fc1g/b_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/fc1g/b_${v}_$r.json').read().strip().splitlines()[-1]);print('fc1_gemm=$v', round(d['ms_per_step']*1000,2), 'us/step', round(d['roofline']['kernel_ms']*1000,1), 'env us')"
  done
done
