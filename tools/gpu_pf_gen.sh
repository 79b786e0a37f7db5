set -u
summ() { python -c "import sys,json; l=[x for x in open('$1').read().splitlines() if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']; print('$1', 'ms/step %.4f kernel_ms %.4f frac %.4f alone %.4f' % (d['ms_per_step'], r['kernel_ms'], r['frac'], r['kernel_alone_ms']))"; }
mkdir -p gpurun_out/gen
for r in 1 2; do for g in 1 2; do FLOCK_ENV_PF_GEN=$g timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline > gpurun_out/gen/c5_g${g}_$r.json 2>&1 || exit 1; summ gpurun_out/gen/c5_g${g}_$r.json; done; done
