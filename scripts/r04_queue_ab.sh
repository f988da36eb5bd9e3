#!/bin/bash
# round 4: same-box A/B of the C2 bench line at GPU_MAX_HW_QUEUES = 4 (HIP's default) vs 8, three
# alternating rounds, each in a fresh process (the queue count is read when the HIP runtime starts).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
OUT=gpurun_out/${1:-r04_qab}
mkdir -p "$OUT"
for r in 1 2 3; do
  for q in 4 8; do
    echo "[queue_ab] round $r queues $q"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-notary \
      --no-keyed --no-sub --no-host > "$OUT/q${q}_r${r}.json" 2> "$OUT/q${q}_r${r}.err" || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('queues', sys.argv[2], 'ms_per_step', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d.items() if k.endswith('stream_ms_per_step')})" "$OUT/q${q}_r${r}.json" $q
  done
done
echo "[queue_ab] done"
