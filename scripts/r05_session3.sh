#!/bin/bash
# Round-5 GPU session: the mirror's host overhead, a kernel + copy timeline of synchronous pinned C2 calls, and an
# interleaved A/B of two engine builds.   usage: scripts/r05_session3.sh TAG LIB_A LIB_B
set -o pipefail
TAG=$1; A=$2; B=$3
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
echo "[r05] host overhead"
timeout -k 10 300 python -u tools/host_overhead_probe.py > "$OUT/overhead.log" 2>&1 || { tail -20 "$OUT/overhead.log"; exit 1; }
tail -1 "$OUT/overhead.log"
echo "[r05] timeline: synchronous pinned C2"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/tl" -o tl --output-format csv -- \
    python3 tools/host_timeline.py --shape c2 --pinned 1 --calls 3 > "$OUT/tl.log" 2>&1 || { tail -20 "$OUT/tl.log"; exit 1; }
grep "^call" "$OUT/tl.log"
TL_GAP_MS=3 python3 tools/host_timeline.py --summarize "$OUT/tl" > "$OUT/tl_summary.txt" 2>&1
tail -3 "$OUT/tl_summary.txt"
timeout -k 10 120 python3 tools/host_timeline.py --shape c2 --pinned 1 --calls 4 > "$OUT/tl_noprof.log" 2>&1 || exit 1
grep "^call" "$OUT/tl_noprof.log"
echo "[r05] A/B $A vs $B"
for i in 1 2 3; do
  for L in "$A" "$B"; do
    CV_LIB_PATH=$L timeout -k 10 120 python tools/ab_lib.py --tag "$L" >> "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
  done
done
grep "^{" "$OUT/ab.log" | cut -c1-200
echo "[r05] done"
