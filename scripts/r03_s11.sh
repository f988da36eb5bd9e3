#!/bin/bash
# round-3 session 11: async sub-chunk size sweep (C2, C5), pipeline tests
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
T=${1:-r03l}
bash scripts/gpu_multi.sh "$T" --skip-check \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread" \
  "timeout -k 10 200 python -u tools/async_probe.py --shape c2 --chunks 262144,524288,1048576 --calls 8" \
  "timeout -k 10 300 python -u tools/async_probe.py --shape c5 --chunks 524288,1048576,2097152 --calls 4"
