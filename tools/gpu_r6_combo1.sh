#!/bin/bash
set -o pipefail
bash tools/gpu_r6_rollout.sh && bash tools/gpu_r6_evscope.sh
