#!/bin/bash
# round-3 session 1: check suite + bench + rocprof, then the scalars-split and leaf-kernel A/Bs and
# the Merkle PMC passes
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
T=${1:-r03a}
bash scripts/gpu_multi.sh "$T" \
  "timeout -k 10 300 python -u tools/knob_ab.py --n 1000000 --msg 300 --rounds 5 base: split33:cvk_set_scalars_split=1/3/3 split43:cvk_set_scalars_split=1/4/3 split42:cvk_set_scalars_split=1/4/2 split44:cvk_set_scalars_split=1/4/4" \
  "for r in 1 2 3; do for m in 0 1; do timeout -k 10 120 python -u tools/merkle_probe.py --ntx 1000000 --reps 5 --leaf-mode \$m || exit 1; done; done" \
  "bash scripts/pmc_merkle.sh gpurun_out/$T/pmc_merkle" \
  "timeout -k 10 240 python -u tools/notary_probe.py --sizes 256,4096,16384 --reps 40 --rounds 3 --variants 'base: seq:cvk_set_lat_seq=3'"
