#!/bin/bash
# round-3 session 6: pipeline slot count vs hardware-queue sharing (GPU_MAX_HW_QUEUES=4): timelines and
# call times of pinned / pageable C2 and C5 host calls with 2 and 3 compute slots
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
T=${1:-r03f}
O=gpurun_out/$T
bash scripts/gpu_multi.sh "$T" --skip-check \
  "timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_pin2 -o t --output-format csv -- python3 tools/host_timeline.py --shape c2 --pinned 1 --slots 2" \
  "python3 tools/host_timeline.py --summarize $O/tl_pin2 > $O/tl_pin2.txt" \
  "for sl in 2 3; do for ch in 131072 262144; do for p in 1 0; do timeout -k 10 120 python3 tools/host_timeline.py --shape c2 --pinned \$p --slots \$sl --first 32768 --chunk \$ch --calls 4 | sed \"s/^/c2 slots=\$sl chunk=\$ch pinned=\$p /\" || exit 1; done; done; done" \
  "for sl in 2 3; do for p in 1 0; do timeout -k 10 120 python3 tools/host_timeline.py --shape c5 --pinned \$p --slots \$sl --calls 3 | sed \"s/^/c5 slots=\$sl pinned=\$p /\" || exit 1; done; done"
