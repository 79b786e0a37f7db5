set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_learners.py -v --timeout 250 --timeout-method thread > gpurun_out/overlap.txt 2>&1; echo "rc(tests)=$?"
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench3p.json 2> gpurun_out/bench3p.err; echo "rc(bench)=$?"
FLOCK_LEARN_PIPELINE=0 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench3s.json 2> gpurun_out/bench3s.err; echo "rc(bench0)=$?"
