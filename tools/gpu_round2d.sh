set -u
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_p$i.json 2> gpurun_out/b_p$i.err; echo "rc=$?"
python -c "
import json; d=json.load(open('gpurun_out/b_p$i.json')); print('run $i', round(d['value']/1e9,3), 'e9', round(d['ms_per_step'],4), 'ms', round(d['roofline']['kernel_ms'],4))"
done
ORDER=pg,pg timeout -k 10 300 python tools/pipe_bench_probe.py
