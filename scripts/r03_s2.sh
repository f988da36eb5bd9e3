#!/bin/bash
# round-3 session 2: pipeline tests (pinned direct-DMA inputs), host pipeline probe, Merkle PMC
# passes and the latency-form / small-batch packing A/B (no full check suite)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
T=${1:-r03b}
bash scripts/gpu_multi.sh "$T" --skip-check \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread" \
  "timeout -k 10 400 python -u tools/host_pipe_probe.py --reps 3" \
  "bash scripts/pmc_merkle.sh gpurun_out/$T/pmc_merkle" \
  "timeout -k 10 300 python -u tools/notary_probe.py --sizes 256,4096,16384 --reps 40 --rounds 3 --variants 'base: seq:cvk_set_lat_seq=3 pool2k:cvk_set_small_pool_min=2048'"
