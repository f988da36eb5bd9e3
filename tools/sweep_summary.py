#!/usr/bin/env python3
"""One line per (round, setting) of tools/sync_pipe_sweep.py output: call time, device time, host phases and the
GPU timeline (CV_OPT_TIMELINE).    python tools/sweep_summary.py LOG [LOG ...]"""
import json
import sys

for f in sys.argv[1:]:
    print(f)
    for ln in open(f):
        if not ln.startswith("{"):
            continue
        d = json.loads(ln)
        t, h = d.get("timeline", {}), d.get("host_ms", {})
        print(f'{d["round"]} {d["setting"]:8s} call {d["sync_pinned_ms"]:7.3f} dev {d["device_ms"]:6.3f} '
              f'r {d["ratio"]:.3f} | plan {h.get("plan", 0):.2f} pack {h.get("pack", 0):.2f} '
              f'enq {h.get("enqueue", 0):.2f} sync {h.get("sync", 0):.2f} sub {h.get("subchunks", 0):.0f} | '
              f'ramp {t.get("ramp_ms", 0):.2f} dma {t.get("dma_end_ms", 0):.2f} span {t.get("span_ms", 0):.2f} '
              f'busy {t.get("busy_ms", 0):.2f} idle {t.get("idle_ms", 0):.2f} tail {t.get("tail_ms", 0):.2f} | '
              f'host pre {t.get("host_pre_ms", 0):.2f} post {t.get("host_post_ms", 0):.2f}')
