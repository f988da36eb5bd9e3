#!/bin/bash
# Round-5 GPU session: the hs_straus translation unit under three LLVM scheduler options against the product
# flags (tools/ab_build_hss.sh variants), C2 1M, alternating fresh processes.   usage: r05_flags_ab.sh TAG [ROUNDS]
set -o pipefail
TAG=$1; R=${2:-2}
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
for i in $(seq 1 "$R"); do
  for V in base trk rlx nohr; do
    CV_LIB_PATH=ab/$V/libcv.so timeout -k 10 120 python -u tools/ab_lib.py --tag $V >> "$OUT/ab.log" 2>&1 || { tail -5 "$OUT/ab.log"; exit 1; }
  done
done
grep "^{" "$OUT/ab.log" | python3 -c "
import json,sys
for ln in sys.stdin:
    d=json.loads(ln); print(d['tag'], round(d['median_ms'],3), d['phase_ms'])"
