#!/usr/bin/env python3
"""Tuning probe of the host-buffer pipeline (cv_ed25519_verify_batch above the pipeline threshold) and
of the device API's stream/slot plan: C2 (1M x 300 B) and C5 (8M x 32 B) shapes, each setting timed
over a few calls, printed as one JSON line per setting.

    python tools/host_pipe_probe.py [--n2 1000000] [--n5 8000000] [--reps 4]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402

SETTINGS = [  # (first, chunk, threads)
    (65536, 262144, 8), (65536, 262144, 16), (65536, 262144, 12), (32768, 131072, 16), (131072, 524288, 16),
    (65536, 262144, 24),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n2", type=int, default=1_000_000)
    ap.add_argument("--n5", type=int, default=8_000_000)
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    eng = native.Engine(1)

    def set_pipe(first, chunk, threads):
        eng.set_option("pipe_first", first)
        eng.set_option("pipe_chunk", chunk)
        eng.set_option("host_threads", threads)
    dev = torch.device("cuda", 0)
    for name, n, ml in (("c2", a.n2, 300), ("c5", a.n5, 32)):
        b = workload.make_batch(eng, 0, n, ml, seed=11)
        # device API: one stream vs two streams (independent calls)
        words = (n + 63) // 64
        ss = [torch.cuda.Stream(dev) for _ in range(2)]
        bms = [torch.zeros(words, dtype=torch.int64, device=dev) for _ in range(2)]
        for ns in (1, 2, 1, 2):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for k in range(6):
                eng.verify_device(0, n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                                  b.len.data_ptr(), bms[k % ns].data_ptr(), 0, ss[k % ns].cuda_stream)
            torch.cuda.synchronize()
            print(json.dumps({"shape": name, "device_streams": ns, "ms_per_call": (time.perf_counter() - t) / 6 * 1e3}),
                  flush=True)
        pk, sig, arena, off, ln = b.to_host()
        del b
        torch.cuda.empty_cache()
        h = torch.empty(256 << 20, dtype=torch.uint8, pin_memory=True)
        dd = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dd.copy_(h, non_blocking=True)
            e1.record()
            e1.synchronize()
            print(json.dumps({"h2d_pinned_gb_per_s": (256 << 20) / e0.elapsed_time(e1) / 1e6}), flush=True)
        del h, dd
        for first, chunk, th in SETTINGS + SETTINGS[:1]:
            set_pipe(first, chunk, th)
            eng.verify_batch(pk, sig, arena, off, ln, want_status=False)
            eng.stats("pipe", reset=True)
            ts = []
            for _ in range(a.reps):
                t = time.perf_counter()
                bm, _ = eng.verify_batch(pk, sig, arena, off, ln, want_status=False)
                ts.append(time.perf_counter() - t)
            assert native.bitmap_to_bools(bm, n).all()
            st = list(eng.stats("pipe", reset=True).values())
            calls = max(st[5], 1)
            print(json.dumps({"shape": name, "first": first, "chunk": chunk, "threads": th,
                              "ms_med": float(np.median(ts) * 1e3), "ms_min": float(np.min(ts) * 1e3),
                              "host_ms_per_call": {k: st[i] / calls * 1e3 for i, k in
                                                   enumerate(("plan", "pack", "wait", "enqueue", "sync"))},
                              "subchunks_per_call": st[6] / calls}), flush=True)
        # the same call from pinned inputs (cv_host_alloc): sub-chunks DMAed in place, no packing
        pinned = [eng.host_copy(x) for x in (pk, sig, arena, off, ln)]
        for first, chunk in ((65536, 262144), (131072, 524288), (32768, 131072)):
            set_pipe(first, chunk, 8)
            eng.verify_batch(*pinned, want_status=False)
            ts = []
            for _ in range(a.reps):
                t = time.perf_counter()
                bm, _ = eng.verify_batch(*pinned, want_status=False)
                ts.append(time.perf_counter() - t)
            assert native.bitmap_to_bools(bm, n).all()
            print(json.dumps({"shape": name, "pinned_inputs": True, "first": first, "chunk": chunk,
                              "ms_med": float(np.median(ts) * 1e3), "ms_min": float(np.min(ts) * 1e3)}), flush=True)
        del pinned
        # pack-only and copy-only rates of the host (what bounds the pipeline besides the GPU)
        t = time.perf_counter()
        _ = np.concatenate([pk.reshape(-1), sig.reshape(-1), arena])
        print(json.dumps({"shape": name, "host_numpy_concat_gb_per_s": (pk.nbytes + sig.nbytes + arena.nbytes) /
                          (time.perf_counter() - t) / 1e9}), flush=True)
        set_pipe(32768, 262144, 8)
    eng.close()


if __name__ == "__main__":
    main()
