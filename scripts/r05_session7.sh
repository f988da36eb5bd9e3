#!/bin/bash
# Round-5 GPU session: host CPU probe A/B of two builds (alternating fresh processes).
#     usage: scripts/r05_session7.sh TAG LIB_A LIB_B [ROUNDS] [SCENARIOS]
set -o pipefail
TAG=$1; A=$2; B=$3; R=${4:-2}; SC=${5:-c2_async_wait,c2_async_sleep,c2_sync,keyed_async,keyed_sync}
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
for i in $(seq 1 "$R"); do
  for L in "$A" "$B"; do
    echo "[r05] $L round $i"
    CV_LIB_PATH=$L timeout -k 10 300 python -u tools/host_cpu_probe.py --scenarios "$SC" >> "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
  done
done
grep '^{"scenario' "$OUT/ab.log" | python3 -c "
import json,sys
for ln in sys.stdin:
    d=json.loads(ln); print(d['lib'], d['scenario'], round(d['wall_ms_per_call'],2), 'cpu', round(d['cpu_ms_per_call'],1), d['top_threads_cpu_ms_per_call'][:3], d['host_ms_per_call'])"
echo "[r05] done"
