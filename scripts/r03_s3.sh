#!/bin/bash
# round-3 session 3: table-builder A/B (ab/base vs ab/tab), GPU parity suite on the new build, and
# timelines of pinned / pageable host calls under rocprofv3 (kernels + memory copies)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
T=${1:-r03c}
O=gpurun_out/$T
bash scripts/gpu_multi.sh "$T" --skip-check \
  "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bash tools/ab_lib.sh ab/base/libcv.so ab/tab/libcv.so 3" \
  "timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_pin3 -o t --output-format csv -- python3 tools/host_timeline.py --shape c2 --pinned 1 --first 32768 --chunk 131072" \
  "timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_pin4 -o t --output-format csv -- python3 tools/host_timeline.py --shape c2 --pinned 1 --first 32768 --chunk 131072 --slots 4" \
  "timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_page -o t --output-format csv -- python3 tools/host_timeline.py --shape c2 --pinned 0 --first 32768 --chunk 131072 --threads 16" \
  "python3 tools/host_timeline.py --summarize $O/tl_pin3 > $O/tl_pin3.txt && python3 tools/host_timeline.py --summarize $O/tl_pin4 > $O/tl_pin4.txt && python3 tools/host_timeline.py --summarize $O/tl_page > $O/tl_page.txt"
