#!/usr/bin/env python3
"""A/B the Straus kernel occupancy variants (waves/SIMD register budget) in ONE process, interleaved
rounds (methodology rule: perf deltas only from interleaved A/B on one device).

    python tools/ab_straus.py [--n 1000000] [--rounds 5]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--msg", type=int, default=300)
    args = ap.parse_args()
    lib = native.load()
    lib.cvk_set_straus_waves.argtypes = [ctypes.c_int]
    eng = native.Engine(1)
    stream = torch.cuda.Stream(0)
    torch.cuda.set_stream(stream)
    b = workload.make_batch(eng, 0, args.n, args.msg, seed=1, stream=stream.cuda_stream)
    bm = torch.zeros((args.n + 63) // 64, dtype=torch.int64, device="cuda:0")
    res = {w: [] for w in (2, 3, 4)}
    for r in range(args.rounds):
        for w in (2, 3, 4):
            lib.cvk_set_straus_waves(w)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            eng.verify_device(0, args.n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                              b.len.data_ptr(), bm.data_ptr(), 0, stream.cuda_stream)
            e0.record(stream)
            eng.verify_device(0, args.n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                              b.len.data_ptr(), bm.data_ptr(), 0, stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            assert bool((bm == -1).all()) or args.n % 64, "honest batch rejected"
            res[w].append(e0.elapsed_time(e1))
    out = {f"waves{w}": {"median_ms": float(np.median(v)), "min_ms": float(np.min(v)),
                         "verifies_per_s": args.n / (np.median(v) * 1e-3)} for w, v in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
