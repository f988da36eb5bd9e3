#!/bin/bash
# Round-5 GPU session: does the hardware queue an engine stream lands on explain the host-call effects?
# The host CPU probe with 0-3 torch streams created first, at HIP's default 4 hardware queues and at 8.
#     usage: scripts/r05_session9.sh TAG
set -o pipefail
TAG=$1; SC=c2_async_wait,c2_sync,keyed_async,keyed_sync
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
for Q in 4 8; do
  for P in 0 1 2 3; do
    echo "[r05] queues $Q pre-streams $P"
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python -u tools/host_cpu_probe.py --calls 6 --pre-streams $P --scenarios "$SC" >> "$OUT/q.log" 2>&1 || { tail -20 "$OUT/q.log"; exit 1; }
  done
done
grep '^{"scenario' "$OUT/q.log" | python3 -c "
import json,sys
for ln in sys.stdin:
    d=json.loads(ln); print('q', d['gpu_max_hw_queues'], 'pre', d['pre_streams'], d['scenario'], round(d['wall_ms_per_call'],2), d['host_ms_per_call'])"
echo "[r05] done"
