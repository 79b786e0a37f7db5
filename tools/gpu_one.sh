timeout -k 10 300 python -u -m pytest tests/test_gpu_checkpoints.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ckpt.txt 2>&1; tail -3 gpurun_out/pytest_ckpt.txt
