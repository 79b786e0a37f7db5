#!/bin/bash
# Round-5 final evidence (gpurun_out/ev5b/): GPU suite + smoke, the env kernel's PMC passes (configs 3-5), every
# config's bench line with rocprofv3 kernel stats, the driver's own command twice with its rocprofv3 profile
# (tools/gpu_evidence_r5.sh phases "tests pmc bench driver").
set -u
EV_OUT=${EV_OUT:-gpurun_out/ev5b} PHASES="${PHASES:-tests pmc bench driver}" CONFIGS="${CONFIGS:-3 4 5 2}" bash tools/gpu_evidence_r5.sh || exit 1
echo ALLDONE3
