#!/bin/bash
# Round-5 GPU session: the host CPU probe on the round-4 package (_r4pkg: its Python mirror and library)
# against this tree, alternating fresh processes.    usage: scripts/r05_session8.sh TAG [ROUNDS]
set -o pipefail
TAG=$1; R=${2:-2}; SC=c2_async_wait,c2_async_sleep,c2_sync,keyed_async,keyed_sync
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
for i in $(seq 1 "$R"); do
  for P in _r4pkg ""; do
    echo "[r05] pkg '${P:-tree}' round $i"
    CV_PKG_ROOT=$P timeout -k 10 300 python -u tools/host_cpu_probe.py --scenarios "$SC" >> "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
  done
done
grep '^{"scenario' "$OUT/ab.log" | python3 -c "
import json,sys
for ln in sys.stdin:
    d=json.loads(ln); print(d['lib'], d['scenario'], round(d['wall_ms_per_call'],2), 'cpu', round(d['cpu_ms_per_call'],1), d['top_threads_cpu_ms_per_call'][:3], d['host_ms_per_call'])"
echo "[r05] done"
