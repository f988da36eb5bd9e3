#!/bin/bash
# Round-5 GPU session: parity tests on the product build, an interleaved A/B of two builds, and the mid-size
# notary probe (pageable and pinned host inputs, host phases).    usage: scripts/r05_session4.sh TAG LIB_A LIB_B
set -o pipefail
TAG=$1; A=$2; B=$3
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
echo "[r05] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"
[ $rc -ne 0 ] && { grep -E "FAIL|Error" "$OUT/pytest.log" | head -20; tail -40 "$OUT/pytest.log"; exit $rc; }
echo "[r05] A/B"
bash scripts/r05_ab.sh "$TAG" "$A" "$B" 3 || exit 1
echo "[r05] notary mid-size"
timeout -k 10 300 python -u tools/notary_probe.py --sizes 4096,16384,32768,65536 --reps 60 --pinned > "$OUT/midsize.log" 2>&1 || { tail -20 "$OUT/midsize.log"; exit 1; }
grep "^{" "$OUT/midsize.log" | python3 -c "
import json,sys
for ln in sys.stdin:
    d=json.loads(ln); print(d['n'], 'host', [round(x,3) for x in d['host_p50_p99_ms']], 'pinned', [round(x,3) for x in d['pinned_p50_p99_ms']], 'dev', [round(x,3) for x in d['device_p50_p99_ms']], d['host_phases_us_mean'], d['pinned_host_phases_us_mean'])"
echo "[r05] done"
