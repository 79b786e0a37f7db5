# two env blocks per workgroup (FLOCK_ENV_REP=2) for the config-3 step: bitwise tests, then bench A/B (alone + loop)
set -o pipefail
mkdir -p gpurun_out/rep
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cells.py -k "two_envs or launches" > gpurun_out/rep/pytest.txt 2>&1 || { tail -30 gpurun_out/rep/pytest.txt; exit 1; }
tail -1 gpurun_out/rep/pytest.txt
for r in 1 2; do
  for cfg in "1 2" "2 1" "2 2"; do
    set -- $cfg
    FLOCK_ENV_REP=$1 timeout -k 10 200 python bench.py --steps 200 --policy-steps 0 --no-cpu-baseline --step-launches $2 > gpurun_out/rep/b_$1_$2_$r.json 2>gpurun_out/rep/err || { tail -5 gpurun_out/rep/err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/rep/b_$1_$2_$r.json').read().strip().splitlines()[-1]);r=d['roofline'];print('rep=$1 launches=$2', round(d['ms_per_step']*1000,2), 'us/step; env in loop', round(r['kernel_ms']*1000,1), 'alone', round(r['kernel_alone_ms']*1000,1))"
  done
done
