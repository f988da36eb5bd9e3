#!/usr/bin/env python3
"""Where the synchronous host call's kernel time goes: the same 1M C2 batch verified from HBM
  whole      one 1M verify per call, calls dealt over two streams (the bench's device step)
  sub S      each call cut into sub-chunks of S records dealt alternately over two streams, as the synchronous
             pipeline deals its sub-chunks — once with a device synchronize after every call (the synchronous call's
             shape, tail included), once back to back (steady state)
(--streams: over that many streams instead) beside the synchronous host call itself from pinned buffers (cv_ed25519_verify_batch).  If the sub-chunked
device calls are as slow as the host call, its kernel time is the sub-chunk granularity, not the DMA.

    python tools/subchunk_probe.py [--sizes 62528,131072,196608] [--calls 8]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--sizes", default="62528,131072,196608")
    ap.add_argument("--first", type=int, default=0, help="first sub-chunk size (0: same as the others)")
    ap.add_argument("--calls", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--host", type=int, default=1)
    ap.add_argument("--streams", type=int, default=2)
    a = ap.parse_args()
    n = a.n
    eng = native.Engine(1)
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in range(a.streams)]
    b = workload.make_batch(eng, 0, n, 300, seed=11, stream=streams[0].cuda_stream)
    torch.cuda.synchronize(dev)
    bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)

    def verify(c0, c1, st):
        eng.verify_device(0, c1 - c0, b.pk.data_ptr() + 32 * c0, b.sig.data_ptr() + 64 * c0, b.arena.data_ptr(),
                          b.off.data_ptr() + 8 * c0, b.len.data_ptr() + 4 * c0, bm.data_ptr() + 8 * (c0 // 64), 0,
                          st.cuda_stream)

    def cuts(S):
        c, x = [0], a.first or S
        while c[-1] < n:
            c.append(min(n, c[-1] + x))
            x = S
        return c

    def run(S, sync_each):
        c = cuts(S) if S else [0, n]
        k = 0
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for call in range(a.calls):
            for j in range(len(c) - 1):
                verify(c[j], c[j + 1], streams[k % len(streams)])
                k += 1
            if sync_each:
                torch.cuda.synchronize(dev)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) / a.calls * 1e3, len(c) - 1

    sizes = [int(x) for x in a.sizes.split(",")]
    for S in [0] + sizes:                                          # warm every launch shape
        run(S, False)
    host = None
    if a.host:
        pinned = tuple(eng.host_copy(x) for x in b.to_host())
        for _ in range(2):
            eng.verify_batch(*pinned, want_status=False)
    for rnd in range(a.rounds):
        for S in [0] + sizes:
            for sync_each in (True, False):
                ms, parts = run(S, sync_each)
                print(json.dumps({"round": rnd, "form": "whole" if not S else f"sub {S}", "first": a.first or S,
                                  "streams": len(streams),
                                  "subchunks": parts, "sync_each_call": sync_each, "ms_per_call": round(ms, 3)}),
                      flush=True)
        if a.host:
            t = time.perf_counter()
            for _ in range(a.calls):
                bmh, _ = eng.verify_batch(*pinned, want_status=False)
            host = (time.perf_counter() - t) / a.calls * 1e3
            assert native.bitmap_to_bools(bmh, n).all()
            print(json.dumps({"round": rnd, "form": "host sync pinned", "ms_per_call": round(host, 3)}), flush=True)
    assert bool((bm == -1).all()), "a device verify rejected an honest signature"
    eng.close()


if __name__ == "__main__":
    main()
