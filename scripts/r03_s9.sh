#!/bin/bash
# round-3 session 9: pipeline + async tests, short bench (host_api async/sync/pageable, notary), a
# timeline of a 4,096-signature notary-sized host call
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
T=${1:-r03j}
O=gpurun_out/$T
bash scripts/gpu_multi.sh "$T" --skip-check \
  "timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread" \
  "timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --no-cpu --no-keyed > $O/bench_short.json" \
  "timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_4096 -o t --output-format csv -- python3 tools/host_timeline.py --shape c5 --n 4096 --pinned 0 --calls 6" \
  "TL_GAP_MS=2 python3 tools/host_timeline.py --summarize $O/tl_4096 > $O/tl_4096.txt" \
  "bash scripts/pmc_merkle.sh $O/pmc_merkle"
