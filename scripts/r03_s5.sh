#!/bin/bash
# round-3 session 5: host pipeline without the copy-queue fill kernel: pipeline tests, host probe, timelines
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
T=${1:-r03e}
O=gpurun_out/$T
bash scripts/gpu_multi.sh "$T" --skip-check \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread" \
  "timeout -k 10 400 python -u tools/host_pipe_probe.py --reps 3" \
  "timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_pin -o t --output-format csv -- python3 tools/host_timeline.py --shape c2 --pinned 1" \
  "python3 tools/host_timeline.py --summarize $O/tl_pin > $O/tl_pin.txt"
