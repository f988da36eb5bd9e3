#!/bin/bash
# Round-5 GPU session: parity tests on the product build, then the mid-size notary probe of two builds,
# alternating fresh processes.    usage: scripts/r05_session12.sh TAG LIB_A LIB_B [ROUNDS]
set -o pipefail
TAG=$1; A=$2; B=$3; R=${4:-2}
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
echo "[r05] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"
[ $rc -ne 0 ] && { grep -E "FAIL|Error" "$OUT/pytest.log" | head -20; tail -40 "$OUT/pytest.log"; exit $rc; }
for i in $(seq 1 "$R"); do
  for L in "$A" "$B"; do
    CV_LIB_PATH=$L timeout -k 10 300 python -u tools/notary_probe.py --sizes 16384,32768,65536 --reps 80 --pinned > "$OUT/np.log" 2>&1 || { tail -5 "$OUT/np.log"; exit 1; }
    grep "^{" "$OUT/np.log" | python3 -c "
import json,sys
for ln in sys.stdin:
    d=json.loads(ln); print('$L', d['n'], 'host', [round(x,3) for x in d['host_p50_p99_ms']], 'pinned', [round(x,3) for x in d['pinned_p50_p99_ms']], d['host_phases_us_mean'], d['pinned_host_phases_us_mean'])"
  done
done
echo "[r05] done"
