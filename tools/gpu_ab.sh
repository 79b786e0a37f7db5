# A/B of library builds through bench.py (config 3 default): alternate runs, kernel_ms of each
# HISTORICAL (rounds 1-2): selected builds through FLOCK_LIB, which the library no longer reads; tools/gpu_ab_swap.sh copies a variant over _build/libflock_amd.so instead.
set -e
for r in 1 2; do
  for lib in "$@"; do
    FLOCK_LIB=$PWD/marl_range_flocking_amd/_build/$lib timeout -k 10 200 python bench.py --steps 100 > gpurun_out/ab_$lib.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/ab_$lib.json'));print('$lib', round(d['roofline']['kernel_ms']*1000,2), 'us kernel', round(d['ms_per_step']*1000,1), 'us/step')"
  done
done
