#!/bin/bash
# Round-5 GPU session: what in the bench's sequence slows the keyed host call (bench line 9.25 ms per step vs
# 7.4-7.6 in tools/host_cpu_probe.py)?  bench sub-sets, then the standalone probe.   usage: r05_session11.sh TAG
set -o pipefail
TAG=$1
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
for V in "--no-sub --no-notary --no-cpu" "--no-notary --no-cpu"; do
  echo "[r05] bench $V"
  timeout -k 10 600 python -u bench.py $V --detail "$OUT/d.json" > "$OUT/b.json" 2> "$OUT/b.err" || { tail -20 "$OUT/b.err"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); k=d['host_api'].get('keyed'); print('keyed host', k)"
done
echo "[r05] probe"
timeout -k 10 300 python -u tools/host_cpu_probe.py --calls 8 --scenarios keyed_async,keyed_sync > "$OUT/p.log" 2>&1 || { tail -20 "$OUT/p.log"; exit 1; }
grep '^{"scenario' "$OUT/p.log" | cut -c1-200
echo "[r05] done"
