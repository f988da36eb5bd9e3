#!/bin/bash
# Round-5 final GPU session on one box: parity tests, smoke, the --gpus 2 refusal, the default bench line, the same
# bench command under rocprofv3 --kernel-trace --stats, and the PMC passes of the throughput kernels.
#     usage: scripts/r05_final.sh TAG [skip-pmc]
set -o pipefail
TAG=$1
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
echo "[final] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"
[ $rc -ne 0 ] && { grep -E "FAIL|Error" "$OUT/pytest.log" | head -20; tail -40 "$OUT/pytest.log"; exit $rc; }
echo "[final] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "[final] --gpus 2 on a 1-GPU box"
timeout -k 10 120 python -u bench.py --gpus 2 --steps 1 > "$OUT/gpus2.out" 2> "$OUT/gpus2.err"
echo "exit $? (expect 2)"; tail -1 "$OUT/gpus2.err"
echo "[final] bench"
timeout -k 10 900 python -u bench.py --detail "$OUT/bench_detail.json" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "[final] bench under rocprofv3 --kernel-trace --stats"
timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o prof --output-format csv -- \
    python3 -u bench.py --detail "$OUT/prof_bench_detail.json" > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { tail -30 "$OUT/prof_bench.err"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
KT=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
[ -n "$KT" ] && python3 tools/trace_by_shape.py "$KT" > "$OUT/trace_by_shape.txt" 2>&1
find "$OUT/prof" -name "*kernel_trace.csv" -delete
cut -d, -f1-4 "$OUT/kernel_stats.csv" | head -14
if [ "$2" != "skip-pmc" ]; then
  echo "[final] PMC passes"
  bash scripts/pmc.sh "$OUT/pmc" > "$OUT/pmc.log" 2>&1 || { tail -20 "$OUT/pmc.log"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc" 1000000 --kernel cv_hs_straus_kernel > "$OUT/pmc_summary.txt" 2>&1
  find "$OUT/pmc" -name "*.csv" -size +2M -delete
  tail -22 "$OUT/pmc_summary.txt"
fi
echo "[final] done"
