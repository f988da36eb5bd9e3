#!/bin/bash
# round-3 session 1: check suite + bench + rocprof, then the scalars-split / drain-split and leaf-kernel A/Bs
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
T=${1:-r03a}
shift
bash scripts/gpu_multi.sh "$T" "$@" \
  "timeout -k 10 400 python -u tools/knob_ab.py --n 1000000 --msg 300 --rounds 5 base: split33:cvk_set_scalars_split=1/3/3 split43:cvk_set_scalars_split=1/4/3 split42:cvk_set_scalars_split=1/4/2 split44:cvk_set_scalars_split=1/4/4 'half1:cvk_set_split_mode=1;cvk_set_split_pct=50' 'half2:cvk_set_split_mode=2;cvk_set_split_pct=50' 'tail30:cvk_set_split_mode=2;cvk_set_split_pct=30'" \
  "for r in 1 2 3; do for m in 0 1; do timeout -k 10 120 python -u tools/merkle_probe.py --ntx 1000000 --reps 5 --leaf-mode \$m || exit 1; done; done"
