#!/bin/bash
# round-3 check: GPU suite, smoke, bench line, rocprof kernel stats of the bench, hs_straus PMC passes
# (HBM traffic for roofline.traffic) and the Merkle PMC passes of the default leaf kernel
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
T=${1:-r03h}
bash scripts/gpu_multi.sh "$T" \
  "bash scripts/pmc.sh gpurun_out/$T/pmc" \
  "bash scripts/pmc_merkle.sh gpurun_out/$T/pmc_merkle"
