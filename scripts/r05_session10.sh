#!/bin/bash
# Round-5 GPU session: host CPU probe of two builds at HIP's default 4 hardware queues with 0-3 streams
# created first (which queues the engine's streams share).    usage: scripts/r05_session10.sh TAG LIB_A LIB_B
set -o pipefail
TAG=$1; A=$2; B=$3; SC=c2_async_wait,c2_sync,keyed_async,keyed_sync
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
for P in 0 2 3; do
  for L in "$A" "$B"; do
    echo "[r05] $L pre-streams $P"
    CV_LIB_PATH=$L timeout -k 10 300 python -u tools/host_cpu_probe.py --calls 6 --pre-streams $P --scenarios "$SC" >> "$OUT/q.log" 2>&1 || { tail -20 "$OUT/q.log"; exit 1; }
  done
done
grep '^{"scenario' "$OUT/q.log" | python3 -c "
import json,sys
for ln in sys.stdin:
    d=json.loads(ln); print(d['lib'], 'pre', d['pre_streams'], d['scenario'], round(d['wall_ms_per_call'],2), d['host_ms_per_call'])"
echo "[r05] done"
