timeout -k 10 300 python -u -m pytest tests/test_gpu_cells.py tests/test_gpu_env_parity.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_one.txt 2>&1; rc=$?; tail -3 gpurun_out/pytest_one.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/phase_prof.py > gpurun_out/phase.txt 2>&1 && cat gpurun_out/phase.txt
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; cat gpurun_out/bench_default.json
