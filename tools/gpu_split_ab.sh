# A/B: the config-3 step as 1 / 2 / 4 / 8 env-range launches (FLOCK_ENV_LAUNCHES), overlapped with learn()
set -o pipefail
O=gpurun_out/split; mkdir -p $O
FLOCK_ENV_LAUNCHES=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cells.py -k specialised > $O/pytest.txt 2>&1 || exit 1
for n in 1 2 4 8 1 4; do
  FLOCK_ENV_LAUNCHES=$n timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline > $O/b3_$n.txt 2>&1 || exit 1
  tail -1 $O/b3_$n.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['value']/1e9,3), round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_ms']*1e3,1))"
done
