#!/bin/bash
# One GPU session on the box, steps chosen on the command line (replaces the round-5 one-off wrappers).
#   usage: scripts/session.sh TAG STEP [STEP ...]
# Steps (each with its own time limit; the session stops at the first failing step):
#   tests            pytest -m gpu (one process)                      -> OUT/pytest.log
#   smoke            __graft_entry__.smoke()                          -> OUT/smoke.log
#   gpus2            bench.py --gpus 2 on a 1-GPU box (expects exit 2) -> OUT/gpus2.err
#   bench[:ARGS]     bench.py ARGS (commas become spaces)             -> OUT/bench.json, OUT/bench_detail.json
#   prof[:ARGS]      the same bench command under rocprofv3 --kernel-trace --stats
#                    -> OUT/kernel_stats.csv, OUT/trace_by_shape.txt
#   pmc[:N]          PMC passes of the throughput kernels at N signatures (scripts/pmc.sh) -> OUT/pmc_N/, summary
#   issue            tools/microbench issue_cost (VALU issue cost at exactly k waves per SIMD) -> OUT/issue_cost.txt
#   ab:LIBA:LIBB[:R] interleaved A/B of two engine builds (tools/ab_lib.py), R rounds -> OUT/ab.log
#   notary[:SIZES]   tools/notary_probe.py over the sizes (pageable + pinned) -> OUT/notary.log
#   cmd:STRING       any command (run by bash -c, 600 s limit)        -> OUT/cmd_K.log
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
k=0
for step in "$@"; do
  k=$((k + 1))
  name=${step%%:*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*:}
  echo "[session $TAG] step $k: $step"
  case $name in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
      rc=$?; tail -2 "$OUT/pytest.log"
      [ $rc -ne 0 ] && { grep -E "FAIL|Error" "$OUT/pytest.log" | head -20; tail -40 "$OUT/pytest.log"; exit $rc; } ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
      tail -1 "$OUT/smoke.log" ;;
    gpus2)
      timeout -k 10 120 python -u bench.py --gpus 2 --steps 1 > "$OUT/gpus2.out" 2> "$OUT/gpus2.err"
      echo "exit $? (expect 2)"; tail -1 "$OUT/gpus2.err" ;;
    bench)
      timeout -k 10 900 python -u bench.py --detail "$OUT/bench_detail.json" ${arg//,/ } > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    prof)
      timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o prof --output-format csv -- \
          python3 -u bench.py --detail "$OUT/prof_bench_detail.json" ${arg//,/ } > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { tail -30 "$OUT/prof_bench.err"; exit 1; }
      find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
      KT=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
      [ -n "$KT" ] && python3 tools/trace_by_shape.py "$KT" > "$OUT/trace_by_shape.txt" 2>&1
      find "$OUT/prof" -name "*kernel_trace.csv" -delete
      cut -d, -f1-4 "$OUT/kernel_stats.csv" | head -14 ;;
    pmc)
      N=${arg:-1000000}
      CV_PMC_N=$N bash scripts/pmc.sh "$OUT/pmc_$N" > "$OUT/pmc_$N.log" 2>&1 || { tail -20 "$OUT/pmc_$N.log"; exit 1; }
      python3 tools/pmc_summary.py "$OUT/pmc_$N" "$N" --kernel cv_hs_straus_kernel > "$OUT/pmc_summary_$N.txt" 2>&1
      find "$OUT/pmc_$N" -name "*.csv" -size +2M -delete
      tail -30 "$OUT/pmc_summary_$N.txt" ;;
    issue)
      timeout -k 10 300 tools/microbench/_bin/issue_cost > "$OUT/issue_cost.txt" 2>&1 || { tail -20 "$OUT/issue_cost.txt"; exit 1; }
      cat "$OUT/issue_cost.txt" ;;
    ab)
      IFS=: read -r A B R <<< "$arg"
      for i in $(seq "${R:-3}"); do
        for L in "$A" "$B"; do
          CV_LIB_PATH=$L timeout -k 10 120 python -u tools/ab_lib.py --tag "$L" >> "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
        done
      done
      grep "^{" "$OUT/ab.log" | cut -c1-240 ;;
    notary)
      timeout -k 10 600 python -u tools/notary_probe.py --sizes "${arg:-4096,16384,32768,65536}" --reps 100 --pinned > "$OUT/notary.log" 2>&1 || { tail -20 "$OUT/notary.log"; exit 1; }
      grep "^{" "$OUT/notary.log" | cut -c1-400 ;;
    cmd)
      timeout -k 10 600 bash -o pipefail -c "$arg" > "$OUT/cmd_$k.log" 2>&1
      rc=$?; tail -25 "$OUT/cmd_$k.log"
      [ $rc -ne 0 ] && { echo "step $k failed rc=$rc"; exit $rc; } ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo "[session $TAG] done"
