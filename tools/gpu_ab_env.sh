# A/B of an environment variable through bench.py: tools/gpu_ab_env.sh VAR "valA valB" [bench args]
set -e
var=$1; vals=$2; shift 2
for r in 1 2; do
  for v in $vals; do
    env $var=$v timeout -k 10 200 python bench.py "$@" > gpurun_out/ab_env_$v.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/ab_env_$v.json'));print('$var=$v', round(d['roofline']['kernel_ms']*1000,2), 'us kernel', round(d['ms_per_step']*1000,1), 'us/step', '%.3g'%d['value'])"
  done
done
