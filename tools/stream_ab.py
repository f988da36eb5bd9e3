#!/usr/bin/env python3
"""Interleaved A/B of how bench.py deals its C2 steps: K device calls of the same 1M batch over S
streams (each stream its own workspace slot), with the engine's drain-overlap split (cvk_set_split_mode)
on or off.  Every round runs every variant once; prints one JSON line per (variant, round).

    python tools/stream_ab.py --n 1000000 --msg 300 --steps 20 --rounds 4
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402

VARIANTS = [("s1_split", 1, 3), ("s2_split", 2, 3), ("s2_nosplit", 2, 0), ("s1_nosplit", 1, 0), ("s3_split", 3, 3)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000000)
    ap.add_argument("--msg", type=int, default=300)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=4)
    args = ap.parse_args()
    lib = native.load()
    lib.cvk_set_split_mode.argtypes = [ctypes.c_int]
    eng = native.Engine(1)
    dev = torch.device("cuda", 0)
    sh = torch.cuda.Stream(dev)
    b = workload.make_batch(eng, 0, args.n, args.msg, seed=20261015, stream=sh.cuda_stream)
    torch.cuda.synchronize(dev)
    words = (args.n + 63) // 64
    streams = [sh] + [torch.cuda.Stream(dev) for _ in range(2)]
    bms = [torch.zeros(words, dtype=torch.int64, device=dev) for _ in streams]

    def run(ns, k):
        eng.verify_device(0, args.n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                          b.len.data_ptr(), bms[k % ns].data_ptr(), 0, streams[k % ns].cuda_stream)

    for name, ns, split in VARIANTS:      # warm every slot / helper stream
        lib.cvk_set_split_mode(split)
        for k in range(2 * ns):
            run(ns, k)
    torch.cuda.synchronize(dev)
    for r in range(args.rounds):
        for name, ns, split in VARIANTS:
            lib.cvk_set_split_mode(split)
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            for k in range(args.steps):
                run(ns, k)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t
            for bm in bms[:ns]:
                assert bool((bm == -1).all()), "rejected an honest signature"
            print(json.dumps({"variant": name, "round": r, "ms_per_step": dt / args.steps * 1e3}), flush=True)
    lib.cvk_set_split_mode(3)
    eng.close()


if __name__ == "__main__":
    main()
