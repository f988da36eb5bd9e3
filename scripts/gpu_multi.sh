#!/bin/bash
# Several GPU steps in one box session: scripts/gpu_check.sh TAG (tests, smoke, bench, rocprof
# stats), then each extra command given as a further argument (a string run by bash with its own
# time limit, output under gpurun_out/TAG/extra_K.log).  Stops at the first failing step.
#   usage: scripts/gpu_multi.sh TAG [--skip-check] ['timeout -k 10 300 python tools/x.py ...' ...]
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$1" = "--skip-check" ]; then shift; else bash scripts/gpu_check.sh "$TAG" || exit $?; fi
k=0
for cmd in "$@"; do
  k=$((k+1))
  echo "[gpu_multi] step $k: $cmd"
  bash -o pipefail -c "$cmd" > "$OUT/extra_$k.log" 2>&1
  rc=$?
  tail -20 "$OUT/extra_$k.log"
  [ $rc -ne 0 ] && { echo "step $k failed rc=$rc"; exit $rc; }
done
echo "[gpu_multi] done"
