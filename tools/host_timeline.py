#!/usr/bin/env python3
"""Timeline of host-buffer verify calls (for rocprofv3 --kernel-trace --memory-copy-trace): a C2- or
C5-shaped batch verified by cv_ed25519_verify_batch from pinned (or pageable) inputs, `--calls` times,
with optional pipeline settings.  Then `--summarize DIR` prints the last call's kernels and copies per
stream, relative to its first event.

    rocprofv3 --kernel-trace --memory-copy-trace -d OUT -o t --output-format csv -- \\
        python3 tools/host_timeline.py --shape c2 --pinned 1 --first 32768 --chunk 131072
    python tools/host_timeline.py --summarize OUT
"""
import argparse
import csv
import ctypes
import glob
import os
import sys
import time

import numpy as np


def summarize(d, gap_ms=3.0):
    gap_ms = float(os.environ.get("TL_GAP_MS", gap_ms))
    ev = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K s" + r["Stream_Id"],
                       r["Kernel_Name"].split("(")[0][-28:], r["Grid_Size_X"]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + r.get("Direction", "?")[:14],
                       r.get("Source_Agent_Id", "") + "->" + r.get("Destination_Agent_Id", ""), r.get("Size", "")))
    ev.sort()
    # the last call: events after the last gap of more than gap_ms
    start = 0
    for i in range(1, len(ev)):
        if ev[i][0] - max(e[1] for e in ev[max(0, i - 50):i]) > gap_ms * 1e6:
            start = i
    t0 = ev[start][0]
    busy = 0
    for e in ev[start:]:
        print(f"{(e[0] - t0) / 1e3:9.1f} {(e[1] - t0) / 1e3:9.1f} {(e[1] - e[0]) / 1e3:8.1f}  {e[2]:18s} {e[3]:30s} {e[4]}")
    print("call span ms", (max(e[1] for e in ev[start:]) - t0) / 1e6)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--summarize", default="")
    ap.add_argument("--shape", default="c2")
    ap.add_argument("--pinned", type=int, default=1)
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--n", type=int, default=0, help="signatures (overrides the shape's)")
    ap.add_argument("--key-pool", type=int, default=0, help="signers from a pool of this many keys (keyed path)")
    ap.add_argument("--async-calls", type=int, default=0, help="after the timed calls: this many async calls, "
                                                               "two in flight (the summary's last window)")
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize)
        return
    import torch  # noqa: F401
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from corda_amd import native, workload
    eng = native.Engine(1)
    for k, v in (("pipe_first", a.first), ("pipe_chunk", a.chunk), ("host_threads", a.threads)):
        if v:
            eng.set_option(k, v)
    n, ml = (1_000_000, 300) if a.shape == "c2" else (8_000_000, 32)
    if a.n:
        n = a.n
    b = workload.make_batch(eng, 0, n, ml, seed=11, key_pool=a.key_pool or None)
    arrs = b.to_host()
    del b
    if a.pinned:
        arrs = tuple(eng.host_copy(x) for x in arrs)
    for k in range(a.calls):
        time.sleep(0.01)                      # a gap between calls (the summary takes the last one)
        eng.stats("pipe", reset=True)
        t = time.perf_counter()
        bm, _ = eng.verify_batch(*arrs, want_status=False)
        dt = (time.perf_counter() - t) * 1e3
        st = eng.stats("pipe", reset=True)
        print(f"call {k}: {dt:.2f} ms  host ms: " + " ".join(f"{n[:-2]}={v * 1e3:.2f}" for n, v in st.items()
                                                            if n.endswith("_s")), flush=True)
    assert native.bitmap_to_bools(bm, n).all()
    if a.async_calls:
        time.sleep(0.01)
        t = time.perf_counter()
        pend = []
        for _ in range(a.async_calls):
            pend.append(eng.verify_batch_async(*arrs, want_status=False))
            if len(pend) == 2:
                bm, _ = eng.wait(pend.pop(0))
        for tk in pend:
            bm, _ = eng.wait(tk)
        print(f"async: {(time.perf_counter() - t) / a.async_calls * 1e3:.2f} ms per call", flush=True)
        assert native.bitmap_to_bools(bm, n).all()
    eng.close()


if __name__ == "__main__":
    main()
