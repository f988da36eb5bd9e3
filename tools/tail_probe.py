#!/usr/bin/env python3
"""Tail-effect probe: per-phase verify times (HIP events on the launch stream) at batch sizes around
whole resident rounds of the half-size Straus kernel, and the small-batch (quad / regular) forms for
the leftover signatures of a 1M batch.

    python tools/tail_probe.py [n ...]
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [983040, 1000000, 1032192, 16960, 33920]
    eng = native.Engine(1)
    lib = native.load()
    lib.cvk_set_quad_max.argtypes = [ctypes.c_uint32]
    stream = torch.cuda.Stream(0)
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    b = workload.make_batch(eng, 0, max(sizes), 300, seed=1, stream=sh)
    bm = torch.zeros((max(sizes) + 63) // 64, dtype=torch.int64, device="cuda:0")
    rows = []
    if os.environ.get("CV_SPLIT_SWEEP"):
        # whole-call time (torch events around verify_device) for the two-stream sub-chunk overlap
        lib.cvk_set_split_mode.argtypes = [ctypes.c_int]
        lib.cvk_set_split_pct.argtypes = [ctypes.c_int]
        for n in [n for n in sizes if n > 32768]:
            for mode, pct in [(0, 25), (3, 25), (1, 25), (0, 25), (3, 25)]:
                lib.cvk_set_split_mode(mode)
                lib.cvk_set_split_pct(pct)
                ts = []
                for r in range(9):
                    bm.zero_()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    eng.verify_device(0, n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                                      b.len.data_ptr(), bm.data_ptr(), 0, sh)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    full = torch.full_like(bm[: (n + 63) // 64], -1)
                    if n % 64:
                        full[-1] = (1 << (n % 64)) - 1
                    assert torch.equal(bm[: (n + 63) // 64], full), (n, mode, pct)
                    if r:
                        ts.append(e0.elapsed_time(e1))
                med = float(np.median(ts))
                print(json.dumps({"n": n, "split_mode": mode, "pct": pct, "median_ms": round(med, 4),
                                  "min_ms": round(float(np.min(ts)), 4), "Mverifies_s": round(n / med / 1e3, 2)}),
                      flush=True)
        lib.cvk_set_split_mode(0)
        eng.close()
        return
    for n in sizes:
        for qmax in ([32768, 0] if n <= 32768 else [32768]):
            lib.cvk_set_quad_max(qmax)
            ph = []
            for r in range(8):
                p = eng.verify_device_timed(0, n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(),
                                            b.off.data_ptr(), b.len.data_ptr(), bm.data_ptr(), sh)
                if r:
                    ph.append(p)
            ph = np.median(np.array(ph), axis=0)
            rows.append({"n": n, "quad_max": qmax, "phase_ms": [round(float(x), 4) for x in ph],
                         "total_ms": round(float(ph.sum()), 4), "Mverifies_s": round(n / ph.sum() / 1e3, 2)})
            print(json.dumps(rows[-1]), flush=True)
    lib.cvk_set_quad_max(32768)
    eng.close()


if __name__ == "__main__":
    main()
