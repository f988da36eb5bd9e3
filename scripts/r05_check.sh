#!/bin/bash
# Round-5 GPU check: parity tests, smoke, the --gpus 2 refusal on a 1-GPU box, and a short bench with the
# c_abi_multi sub-line forced at N = 1.   usage: scripts/r05_check.sh TAG
set -o pipefail
TAG=${1:-r05}; shift
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
echo "[r05] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"
[ $rc -ne 0 ] && { grep -E "FAIL|Error|error" "$OUT/pytest.log" | head -30; tail -60 "$OUT/pytest.log"; exit $rc; }
echo "[r05] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "[r05] --gpus 2 on a 1-GPU box"
timeout -k 10 120 python -u bench.py --gpus 2 --steps 1 > "$OUT/gpus2.out" 2> "$OUT/gpus2.err"
echo "exit $? (expect 2)"; tail -2 "$OUT/gpus2.err"
echo "[r05] bench"
timeout -k 10 600 python -u bench.py --c-abi-multi --no-notary --no-keyed "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "[r05] done"
