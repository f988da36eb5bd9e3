#!/bin/bash
# Mid-size notary batches: host-buffer p50 (pageable and pinned inputs), device p50 and kernel
# phases at 16,384 / 32,768 / 65,536 signatures (1/16 adversarial), for the launch forms the options select.
set -o pipefail
TAG=${1:-r05m}
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
timeout -k 10 500 python -u tools/notary_probe.py --sizes 16384,32768,65536 --reps 80 --rounds 2 --pinned \
  --variants "base: quad64:quad_max=65536 pipe:pipe_min=16384,pipe_first=8192 pipeq:pipe_min=16384,pipe_first=8192,quad_max=65536" \
  > "$OUT/midsize.log" 2>&1 || { tail -20 "$OUT/midsize.log"; exit 1; }
python3 - "$OUT/midsize.log" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln)
        print(d["variant"], d["round"], d["n"], "host", [round(x, 3) for x in d["host_p50_p99_ms"]],
              "pinned", [round(x, 3) for x in (d["pinned_p50_p99_ms"] or [])], "device",
              [round(x, 3) for x in d["device_p50_p99_ms"]], {k: round(v, 3) for k, v in d["phase_ms"].items()})
PY
