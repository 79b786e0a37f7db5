#!/bin/bash
# Configs 4 / 5 with train() on its own stream beside the following env steps (OverlappedTrain): the bitwise tests,
# then bench lines with --overlap 1 / 0 interleaved on one box (gpurun_out/trainov/).
set -u
O=gpurun_out/trainov; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap_train.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  for c in 4 5; do
    for ov in 1 0; do
      timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --overlap $ov > $O/c${c}_ov${ov}_$r.json 2> $O/c${c}_ov${ov}_$r.err || { tail -20 $O/c${c}_ov${ov}_$r.err; exit 1; }
      python -c "import json,sys; d=json.loads(open('$O/c${c}_ov${ov}_$r.json').read().strip().splitlines()[-1]); print('config $c overlap $ov rep $r', 'ms/step %.4f' % d['ms_per_step'], '%.4g' % d['value'], 'env launch %.4f' % d['roofline']['kernel_ms'])"
    done
  done
done
echo ALLDONE
