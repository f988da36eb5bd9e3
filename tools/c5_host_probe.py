#!/usr/bin/env python3
"""C5-shaped host-buffer calls (8M signatures over 32-byte ids, 1.12 GB of inputs per call) through
bench.py's host_api_rate, in a fresh process or after the bench's device-API work (--dirty: C2 device
calls dealt over two torch streams first, which creates the engine's split-helper streams and the
caller's streams before the host pipeline runs).  --lazy: the engine creates its pipeline streams on
first use instead of at cv_open (cvk_set_eager_streams(0)).  One JSON line per repetition:
[async pinned, sync pinned, async pageable, sync pageable] ms per call.

    python tools/c5_host_probe.py [--dirty] [--lazy]
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from corda_amd import native, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dirty", action="store_true")
    ap.add_argument("--lazy", action="store_true")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    lib = native.load()
    lib.cvk_set_eager_streams.argtypes = [ctypes.c_int]
    lib.cvk_set_eager_streams(0 if a.lazy else 1)
    eng = native.Engine(1)
    if a.dirty:
        dev = torch.device("cuda", 0)
        c2 = workload.make_batch(eng, 0, 1_000_000, 300, seed=3)
        streams = [torch.cuda.Stream(dev) for _ in range(2)]
        bms = [torch.zeros(15625, dtype=torch.int64, device=dev) for _ in streams]
        for k in range(8):
            eng.verify_device(0, c2.n, c2.pk.data_ptr(), c2.sig.data_ptr(), c2.arena.data_ptr(), c2.off.data_ptr(),
                              c2.len.data_ptr(), bms[k % 2].data_ptr(), 0, streams[k % 2].cuda_stream)
        torch.cuda.synchronize(dev)
        del c2
    b = workload.make_batch(eng, 0, 8_000_000, 32, seed=5)
    for r in range(a.reps):
        h = bench.host_api_rate(eng, b, 3, 1.0, "c5", async_steps=8)
        print(json.dumps({"dirty": a.dirty, "lazy": a.lazy, "rep": r,
                          "ms": [h["ms_per_step"], h["sync_pinned"]["ms_per_step"],
                                 h["async_pageable"]["ms_per_step"], h["pageable"]["ms_per_step"]]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
