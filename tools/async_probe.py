#!/usr/bin/env python3
"""Rate of host-buffer calls with two in flight (cv_ed25519_verify_batch_async / cv_wait) against the
synchronous call, on a C2- or C5-shaped batch from pinned or pageable buffers, for a list of async
sub-chunk sizes (CV_OPT_ASYNC_CHUNK).  One JSON line per setting.

    python tools/async_probe.py --shape c2 --chunks 262144,524288,1048576 --calls 8
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="c2")
    ap.add_argument("--chunks", default="262144,524288,1048576")
    ap.add_argument("--calls", type=int, default=8)
    a = ap.parse_args()
    import torch  # noqa: F401
    from corda_amd import native, workload
    eng = native.Engine(1)
    if os.environ.get("PIPE_SLOTS"):                  # compute streams of the pipelined calls (CV_OPT_PIPE_SLOTS)
        eng.set_option("pipe_slots", int(os.environ["PIPE_SLOTS"]))
    n, ml = (1_000_000, 300) if a.shape == "c2" else (8_000_000, 32)
    b = workload.make_batch(eng, 0, n, ml, seed=11)
    page = b.to_host()
    del b
    pin = tuple(eng.host_copy(x) for x in page)
    for name, arrs in (("pinned", pin), ("pageable", page)):
        eng.verify_batch(*arrs, want_status=False)
        t = time.perf_counter()
        for _ in range(a.calls):
            bm, _ = eng.verify_batch(*arrs, want_status=False)
        sync_ms = (time.perf_counter() - t) / a.calls * 1e3
        assert native.bitmap_to_bools(bm, n).all()
        for ch in (int(x) for x in a.chunks.split(",")):
            eng.set_option("async_chunk", ch)
            eng.wait(eng.verify_batch_async(*arrs, want_status=False))
            t = time.perf_counter()
            pend = []
            for _ in range(a.calls):
                pend.append(eng.verify_batch_async(*arrs, want_status=False))
                if len(pend) == 2:
                    bm, _ = eng.wait(pend.pop(0))
            for tk in pend:
                bm, _ = eng.wait(tk)
            ms = (time.perf_counter() - t) / a.calls * 1e3
            assert native.bitmap_to_bools(bm, n).all()
            print(json.dumps({"shape": a.shape, "inputs": name, "pipe_slots": eng.get_option("pipe_slots"),
                              "async_chunk": ch, "async_ms_per_call": ms,
                              "sync_ms_per_call": sync_ms}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
