#!/usr/bin/env python3
"""Workload for the PMC passes (scripts/pmc.sh): the C2 batch (1M signatures, 300-byte messages)
through verify_device_timed — whole-chunk launches of scalars | points | hs_straus, no two-stream
split — so each kernel's counters describe one whole-batch dispatch.

    python tools/pmc_probe.py [--n 1000000] [--reps 2]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--msg", type=int, default=300)
    args = ap.parse_args()
    eng = native.Engine(1)
    s = torch.cuda.Stream(0)
    torch.cuda.set_stream(s)
    b = workload.make_batch(eng, 0, args.n, args.msg, seed=1, stream=s.cuda_stream)
    bm = torch.zeros((args.n + 63) // 64, dtype=torch.int64, device="cuda:0")
    for _ in range(args.reps):
        ph = eng.verify_device_timed(0, args.n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                                     b.len.data_ptr(), bm.data_ptr(), s.cuda_stream)
        print("phase_ms", [round(float(x), 3) for x in ph], flush=True)
    assert bool((bm == -1).all()) or args.n % 64
    eng.close()


if __name__ == "__main__":
    main()
