set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_torch_ops.py -v --timeout 250 --timeout-method thread > gpurun_out/torch_ops.txt 2>&1; echo "rc(ops)=$?"
timeout -k 10 120 python tools/host_cost_ops.py > gpurun_out/host_cost_ops.txt 2>&1; echo "rc(host)=$?"
