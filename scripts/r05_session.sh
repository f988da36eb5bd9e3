#!/bin/bash
# Round-5 GPU session: interleaved A/B of two engine builds (plain C2 device path, keyed device path, notary
# latency sizes), then the GPU parity tests on the product build, a short bench with the c_abi_multi sub-line
# forced at N = 1, and the PMC passes of the verify kernels.  Every GPU step has its own time limit; the script
# stops at the first failure.     usage: scripts/r05_session.sh TAG LIB_A LIB_B [skip-ab]
set -o pipefail
TAG=$1; A=$2; B=$3; SKIP=$4
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
if [ "$SKIP" != "skip-ab" ]; then
  echo "[r05] A/B $A vs $B"
  for i in 1 2 3; do
    for L in "$A" "$B"; do
      CV_LIB_PATH=$L timeout -k 10 120 python tools/ab_lib.py --tag "$L" >> "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
      CV_LIB_PATH=$L timeout -k 10 120 python tools/ab_lib.py --tag "$L" --keyed 1024 >> "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
    done
  done
  grep "^{" "$OUT/ab.log"
  for L in "$A" "$B"; do
    CV_LIB_PATH=$L timeout -k 10 180 python tools/notary_probe.py --sizes 4096,16384,65536 --reps 60 >> "$OUT/notary_ab.log" 2>&1 || { tail -20 "$OUT/notary_ab.log"; exit 1; }
    echo "lib $L done" >> "$OUT/notary_ab.log"
  done
  grep -E "^\{|^lib" "$OUT/notary_ab.log" | cut -c1-220
fi
echo "[r05] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"
[ $rc -ne 0 ] && { grep -E "FAIL|Error" "$OUT/pytest.log" | head -20; tail -40 "$OUT/pytest.log"; exit $rc; }
echo "[r05] bench"
timeout -k 10 600 python -u bench.py --c-abi-multi --no-notary --no-keyed > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "[r05] pmc"
bash scripts/pmc.sh "$OUT/pmc" || exit 1
python3 tools/pmc_summary.py "$OUT/pmc" 1000000 --kernel cv_hs_straus_kernel > "$OUT/pmc_summary.txt" 2>&1
tail -30 "$OUT/pmc_summary.txt"
echo "[r05] done"
