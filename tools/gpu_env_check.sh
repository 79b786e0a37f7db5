# Env-kernel change check: parity tests, phase profile of the small-N (uw 64 x 1024) step, config-2 and -3 bench lines
set -o pipefail
O=gpurun_out/envc; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_env_parity.py tests/test_gpu_cells.py tests/test_gpu_dropin_drivers.py > $O/pytest.txt 2>&1 && \
timeout -k 10 120 python tools/phase_prof.py --variant uw --E 1024 --N 64 > $O/ph_uw.txt 2>&1 && \
timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline > $O/b2.txt 2>&1 && \
timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline > $O/b3.txt 2>&1
echo rc=$?
