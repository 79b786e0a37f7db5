#!/bin/bash
# Round 5: the uw / uw_discrete phase-2 tree's rounds s < 64 in registers (wave shuffles) instead of LDS rounds with
# a block barrier each (base = previous head in _ab/base). The whole GPU suite in this tree, then an interleaved
# same-box A/B on configs 4 and 2, and the config-4 phase profile.
set -o pipefail
O=gpurun_out/wavetail; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
ABT_OUT=wavetail/ab TREES="base cur" bash tools/gpu_ab_trees.sh 3 "--config 4" "--config 2" || exit 1
timeout -k 10 120 python tools/phase_prof.py --variant uwd --seeds --E 8192 --N 512 --k 4 --steps 20 > $O/phase_uwd.txt 2>&1
