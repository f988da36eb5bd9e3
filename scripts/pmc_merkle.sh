#!/bin/bash
# PMC passes over the Merkle tx-id kernels (leaf SHA-256 + tree) on the C3 leaf shape, one counter
# group per rocprofv3 run, then the record bench.py's c3.merkle_roofline reads.
#   usage: scripts/pmc_merkle.sh [OUT_DIR] [NTX] [LEAF_MODE]
set -e
OUT=${1:-gpurun_out/pmc_merkle}
NTX=${2:-1000000}
LM=${3:--1}
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p "$OUT"
export TMPDIR=/tmp
K="--kernel-include-regex (leaf_hash|merkle_tree)"
timeout -k 10 120 python3 tools/merkle_probe.py --ntx "$NTX" --reps 3 --leaf-mode "$LM" > "$OUT/probe.json" 2> "$OUT/probe.err"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD $K -d "$OUT/p1" -o p1 --output-format csv -- python3 tools/merkle_probe.py --ntx "$NTX" --reps 1 --leaf-mode "$LM" > "$OUT/p1.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE $K -d "$OUT/p2" -o p2 --output-format csv -- python3 tools/merkle_probe.py --ntx "$NTX" --reps 1 --leaf-mode "$LM" > "$OUT/p2.log" 2>&1
python3 tools/merkle_pmc.py "$OUT" "$OUT/probe.json" --out "$OUT/pmc_merkle.json" > "$OUT/summary.txt"
echo merkle pmc done
