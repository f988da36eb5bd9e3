#!/bin/bash
# Interleaved A/B of two engine builds on one box (C2 device path, HIP-event kernel phases); optional keyed pool.
#   usage: scripts/r05_ab.sh TAG LIB_A LIB_B [ROUNDS] [KEYED_POOL]
set -o pipefail
TAG=$1; A=$2; B=$3; R=${4:-3}; K=${5:-0}
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
for i in $(seq $R); do
  for L in "$A" "$B"; do
    CV_LIB_PATH=$L timeout -k 10 120 python tools/ab_lib.py --tag "$L" >> "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
    if [ "$K" != "0" ]; then
      CV_LIB_PATH=$L timeout -k 10 120 python tools/ab_lib.py --tag "$L" --keyed $K >> "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
    fi
  done
done
grep "^{" "$OUT/ab.log" | cut -c1-220
