#!/bin/bash
# Config 5's bench line and rocprofv3 kernel stats with the default train() in line (gpurun_out/c5line/).
set -u
export TMPDIR=/tmp
O=gpurun_out/c5line; mkdir -p $O
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > $O/bench_config5.json 2> $O/bench_config5.err || { tail -20 $O/bench_config5.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 bench.py --config 5 --no-cpu-baseline > $O/prof_c5.log 2>&1 || { tail -20 $O/prof_c5.log; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_config5.json').read().strip().splitlines()[-1]); r=d['roofline']; print('config 5', d['ms_per_step'], d['value'], r['kernel_ms'], r['frac'], r['kernel_alone_ms'], r['frac_alone'])"
echo ALLDONE
