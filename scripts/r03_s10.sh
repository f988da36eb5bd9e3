#!/bin/bash
# round-3 session 10: async pipeline with the host-side join: pipeline tests, short bench, timeline of
# three async C2 calls in flight
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
T=${1:-r03k}
O=gpurun_out/$T
bash scripts/gpu_multi.sh "$T" --skip-check \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread" \
  "timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --no-cpu --no-keyed --no-notary > $O/bench_short.json"
