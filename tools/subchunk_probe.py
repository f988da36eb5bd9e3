#!/usr/bin/env python3
"""GPU efficiency of sub-chunked verification, separated from the host: a device-resident C5-shaped batch
(8M x 32 B) verified as sub-chunks of m signatures dealt round-robin over S streams (each stream takes
its own workspace slot), against one whole call; then the host pipeline with 2/3/4 slots.  One JSON
line per setting.  Run it once per GPU_MAX_HW_QUEUES setting to see whether streams share hardware
queues.

    python tools/subchunk_probe.py [--n 8000000]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8_000_000)
    ap.add_argument("--msg", type=int, default=32)
    ap.add_argument("--host", action="store_true")
    a = ap.parse_args()
    lib = native.load()
    lib.cvk_set_pipe.argtypes = [ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]
    lib.cvk_set_pipe_slots.argtypes = [ctypes.c_int]
    lib.cvk_pipe_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    eng = native.Engine(1)
    dev = torch.device("cuda", 0)
    n = a.n
    b = workload.make_batch(eng, 0, n, a.msg, seed=11)
    words = (n + 63) // 64
    bm = torch.zeros(words, dtype=torch.int64, device=dev)
    env = os.environ.get("GPU_MAX_HW_QUEUES", "default")
    streams = [torch.cuda.Stream(dev) for _ in range(4)]

    def run(m, ns, reps=3):
        ts = []
        for r in range(reps + 1):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for j, c0 in enumerate(range(0, n, m)):
                mm = min(m, n - c0)
                st = streams[j % ns]
                eng.verify_device(0, mm, b.pk.data_ptr() + 32 * c0, b.sig.data_ptr() + 64 * c0, b.arena.data_ptr(),
                                  b.off.data_ptr() + 8 * c0, b.len.data_ptr() + 4 * c0, bm.data_ptr() + c0 // 8, 0,
                                  st.cuda_stream)
            torch.cuda.synchronize()
            if r:
                ts.append(time.perf_counter() - t)
        assert native.bitmap_to_bools(bm.cpu().numpy().view(np.uint64), n).all()
        return float(np.median(ts) * 1e3)

    print(json.dumps({"hw_queues": env, "whole_call_ms": run(n, 1)}), flush=True)
    for m in (131072, 262144, 524288, 1048576):
        for ns in (1, 2, 3, 4):
            print(json.dumps({"hw_queues": env, "subchunk": m, "streams": ns, "ms": run(m, ns)}), flush=True)
    if a.host:
        pk, sig, arena, off, ln = b.to_host()
        for slots in (2, 3, 4):
            for first, chunk in ((32768, 131072), (65536, 262144), (131072, 524288)):
                lib.cvk_set_pipe_slots(slots)
                lib.cvk_set_pipe(131072, first, chunk, 8)
                eng.verify_batch(pk, sig, arena, off, ln, want_status=False)
                lib.cvk_pipe_stats(None, 1)
                ts = []
                for _ in range(3):
                    t = time.perf_counter()
                    hb, _ = eng.verify_batch(pk, sig, arena, off, ln, want_status=False)
                    ts.append(time.perf_counter() - t)
                st = (ctypes.c_double * 7)()
                lib.cvk_pipe_stats(st, 1)
                print(json.dumps({"hw_queues": env, "host_slots": slots, "first": first, "chunk": chunk,
                                  "ms": float(np.median(ts) * 1e3),
                                  "host_ms": {k: st[i] / 3 * 1e3 for i, k in
                                              enumerate(("plan", "pack", "wait", "enqueue", "sync"))}}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
