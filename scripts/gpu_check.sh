#!/bin/bash
# One GPU session on the box: GPU parity tests, the default bench line, and a rocprofv3 kernel-trace
# summary of the same bench command.  Every GPU step has its own time limit; the script stops at the
# first failure.   usage: scripts/gpu_check.sh TAG [bench args...]
set -o pipefail
TAG=${1:-check}
shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
[ -z "$GRAFT_REPO_ROOT" ] && OUT=$(pwd)/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1

echo "[gpu_check] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; tail -40 "$OUT/pytest.log"; exit $rc; }

echo "[gpu_check] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"

echo "[gpu_check] bench"
timeout -k 10 400 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"

echo "[gpu_check] rocprofv3 kernel stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o prof --output-format csv -- \
    python3 bench.py --no-cpu --no-notary --steps 5 --warmup 1 "$@" > "$OUT/prof.log" 2>&1 || { tail -30 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-4 "$OUT/kernel_stats.csv" | head -12
echo "[gpu_check] done"
