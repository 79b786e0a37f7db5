set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1; echo "rc(tests)=$?"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1; echo "rc(smoke)=$?"
timeout -k 10 200 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; echo "rc(bench)=$?"
timeout -k 10 120 python tools/host_parts.py > gpurun_out/host_parts.txt 2>&1; echo "rc(host)=$?"
