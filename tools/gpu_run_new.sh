mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_reset.py tests/test_gpu_learners_scale.py tests/test_gpu_checkpoints.py tests/test_gpu_dropin_drivers.py -v --timeout 300 --timeout-method thread > gpurun_out/new_tests.txt 2>&1
