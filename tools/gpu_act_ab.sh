set -o pipefail
for v in 0 1 0 1; do FLOCK_ACT_STAGE=$v timeout -k 10 120 python tools/act_bench.py || exit 1; done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_act.py 2>&1 | tail -2
