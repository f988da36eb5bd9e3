#!/bin/bash
# round-3 session 7: pipeline sub-chunk plan sweep (2 slots; ramp on/off; chunk size), C2 and C5
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
T=${1:-r03g}
O=gpurun_out/$T
bash scripts/gpu_multi.sh "$T" --skip-check \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread" \
  "for ch in 262144 393216 524288; do for r in 1 0; do for p in 1 0; do timeout -k 10 120 python3 tools/host_timeline.py --shape c2 --pinned \$p --ramp \$r --first 32768 --chunk \$ch --calls 5 | sed \"s/^/c2 chunk=\$ch ramp=\$r pinned=\$p /\" || exit 1; done; done; done" \
  "for ch in 262144 524288 1048576; do for p in 1 0; do timeout -k 10 120 python3 tools/host_timeline.py --shape c5 --pinned \$p --first 32768 --chunk \$ch --calls 4 | sed \"s/^/c5 chunk=\$ch pinned=\$p /\" || exit 1; done; done" \
  "timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_pin -o t --output-format csv -- python3 tools/host_timeline.py --shape c2 --pinned 1" \
  "python3 tools/host_timeline.py --summarize $O/tl_pin > $O/tl_pin.txt" || exit $?
bash scripts/gpu_multi.sh "${T}_lat" --skip-check \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k 'latency_field_forms or quad_and_tri' --timeout 120 --timeout-method thread" \
  "timeout -k 10 300 python -u tools/notary_probe.py --sizes 256,4096,16384 --reps 40 --rounds 3 --variants 'seq3:cvk_set_lat_seq=3 seq7:cvk_set_lat_seq=7'"
