#!/bin/bash
# Round-5 GPU session: parity tests on the product build, then the mid-size notary probe (pageable and
# pinned host inputs, host phases).    usage: scripts/r05_session5.sh TAG [skip-tests]
set -o pipefail
TAG=$1
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
if [ "$2" != "skip-tests" ]; then
    echo "[r05] pytest -m gpu"
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
    rc=$?; tail -2 "$OUT/pytest.log"
    [ $rc -ne 0 ] && { grep -E "FAIL|Error" "$OUT/pytest.log" | head -20; tail -40 "$OUT/pytest.log"; exit $rc; }
fi
echo "[r05] notary mid-size"
timeout -k 10 400 python -u tools/notary_probe.py --sizes ${SIZES:-4096,16384,32768,65536} --reps 60 --pinned --variants "${VARIANTS:-base:}" --rounds ${ROUNDS:-1} > "$OUT/midsize.log" 2>&1 || { tail -20 "$OUT/midsize.log"; exit 1; }
grep "^{" "$OUT/midsize.log" | python3 -c "
import json,sys
for ln in sys.stdin:
    d=json.loads(ln); print(d['variant'], d['round'], d['n'], 'host', [round(x,3) for x in d['host_p50_p99_ms']], 'pinned', [round(x,3) for x in d['pinned_p50_p99_ms']], 'dev', [round(x,3) for x in d['device_p50_p99_ms']], d['host_phases_us_mean'], d['pinned_host_phases_us_mean'])"
echo "[r05] done"
