#!/bin/bash
# Round-5 GPU session: host CPU time and cgroup throttling of the host-buffer calls (tools/host_cpu_probe.py),
# without and then under rocprofv3 --kernel-trace (the keyed call ran faster under the profiler in round 4).
#     usage: scripts/r05_session6.sh TAG [SCENARIOS]
set -o pipefail
TAG=$1; SC=${2:-c2_async_wait,c2_async_sleep,c2_sync,keyed_async,keyed_async_sleep,keyed_sync}
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
echo "[r05] host cpu probe"
timeout -k 10 400 python -u tools/host_cpu_probe.py --scenarios "$SC" > "$OUT/cpu.log" 2>&1 || { tail -20 "$OUT/cpu.log"; exit 1; }
grep "^{" "$OUT/cpu.log"
echo "[r05] host cpu probe under rocprofv3 --kernel-trace"
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof" -o kt --output-format csv -- \
    python3 -u tools/host_cpu_probe.py --scenarios "$SC" > "$OUT/cpu_prof.log" 2>&1 || { tail -20 "$OUT/cpu_prof.log"; exit 1; }
grep "^{" "$OUT/cpu_prof.log"
rm -rf "$OUT/prof"
echo "[r05] done"
