#!/bin/bash
# round-3 session 8: pipeline tests (direct small-path threshold), Merkle PMC of the pair leaf kernel,
# notary latency with pinned and pageable inputs
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
T=${1:-r03i}
bash scripts/gpu_multi.sh "$T" --skip-check \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread" \
  "bash scripts/pmc_merkle.sh gpurun_out/$T/pmc_merkle" \
  "timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu --no-sub --no-keyed > gpurun_out/$T/bench_small.json"
