set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_learners_scale.py -v --timeout 250 --timeout-method thread > gpurun_out/scale.txt 2>&1; echo "rc(scale)=$?"
timeout -k 10 200 python bench.py > gpurun_out/bench3.json 2> gpurun_out/bench3.err; echo "rc(bench)=$?"
CONFIGS="3" bash tools/gpu_pmc_all.sh
