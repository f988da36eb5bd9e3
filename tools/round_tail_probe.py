#!/usr/bin/env python3
"""hs_straus launched whole over n signatures for n at whole rounds of resident waves (3 waves per SIMD x 1,024
SIMDs x 64 = 196,608 signatures per round) and just past them: separates the kernel's steady-state rate from the
cost of a launch's partly filled last round.  HIP-event phases of verify_device_timed.

    python tools/round_tail_probe.py [--sizes 983040,1000000,1179648] [--reps 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402

W_MAC = 130460


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="786432,983040,1000000,1179648")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    sizes = [int(x) for x in a.sizes.split(",")]
    eng = native.Engine(1)
    s = torch.cuda.Stream(0)
    torch.cuda.set_stream(s)
    mad_rate, _ = eng.calibrate(0)
    b = workload.make_batch(eng, 0, max(sizes), 300, seed=3, stream=s.cuda_stream)
    bm = torch.zeros((max(sizes) + 63) // 64, dtype=torch.int64, device="cuda:0")
    for n in sizes:
        eng.verify_device_timed(0, n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                                b.len.data_ptr(), bm.data_ptr(), s.cuda_stream)
    for rnd in range(2):
        for n in sizes:
            ph = np.median(np.array([eng.verify_device_timed(0, n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(),
                                                             b.off.data_ptr(), b.len.data_ptr(), bm.data_ptr(),
                                                             s.cuda_stream) for _ in range(a.reps)]), axis=0)
            hs = float(ph[2])
            print(json.dumps({"round": rnd, "n": n, "rounds_of_waves": n / 196608, "hs_straus_ms": round(hs, 4),
                              "ns_per_verify": round(hs * 1e6 / n, 3), "frac": round(n * W_MAC / (hs * 1e-3) / mad_rate, 4),
                              "phase_ms": [round(float(x), 4) for x in ph]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
