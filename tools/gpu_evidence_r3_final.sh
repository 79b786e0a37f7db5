#!/bin/bash
# Round-3 final evidence: the env kernel's VALU PMC passes (-> profiles/pmc_valu_*.json, read by bench.py), then
# tools/gpu_evidence_r3.sh (GPU tests, smoke, traffic + SQ PMC passes, every config's bench line + rocprofv3 stats).
set -u
PHASES=pmc CONFIGS="3 2 4 5" bash tools/gpu_r3_valu.sh || exit 1
cp gpurun_out/valu/pmc_valu_*.json profiles/
PHASES="tests pmc bench" bash tools/gpu_evidence_r3.sh
