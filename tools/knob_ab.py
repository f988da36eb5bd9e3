#!/usr/bin/env python3
"""In-process interleaved A/B of the library's internal launch knobs on one batch: every round runs
each variant once (whole device call, HIP events on the launch stream) plus its per-phase times
(cv_ed25519_verify_device_timed), and checks the verdict bitmap each time.

    python tools/knob_ab.py --n 1000000 --msg 300 --rounds 5 \\
        'base:' 'split34:cvk_set_scalars_split=1/3/4'

A variant is NAME:SETTER=A/B/C;SETTER=... (integer arguments separated by '/'); before each variant
the setters named by ANY variant are reset to the values given with --reset (same syntax, default
the library defaults listed in RESET below).
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

RESET = {"cvk_set_scalars_split": (0, 3, 3), "cvk_set_split_mode": (3,), "cvk_set_split_pct": (10,),
         "cvk_set_hs_waves": (3,), "cvk_set_points_mode": (3,), "cvk_set_scalars_waves": (3,),
         "cvk_set_prep_tp": (0,)}


def parse(spec):
    name, _, body = spec.partition(":")
    sets = []
    for kv in filter(None, body.split(";")):
        k, v = kv.split("=")
        sets.append((k, tuple(int(x) for x in v.split("/"))))
    return name, sets


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--msg", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    lib = native.load()
    variants = [parse(v) for v in a.variants]
    used = {k for _, s in variants for k, _ in s}

    def apply(sets):
        for k in used:
            args = RESET[k]
            getattr(lib, k).argtypes = [ctypes.c_int] * len(args)
            getattr(lib, k)(*args)
        for k, args in sets:
            getattr(lib, k).argtypes = [ctypes.c_int] * len(args)
            getattr(lib, k)(*args)

    eng = native.Engine(1)
    stream = torch.cuda.Stream(0)
    torch.cuda.set_stream(stream)
    b = workload.make_batch(eng, 0, a.n, a.msg, seed=1, stream=stream.cuda_stream)
    bm = torch.zeros((a.n + 63) // 64, dtype=torch.int64, device="cuda:0")
    full = torch.full_like(bm, -1)
    if a.n % 64:
        full[-1] = (1 << (a.n % 64)) - 1
    ptrs = (b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(), b.len.data_ptr())
    res = {name: {"call": [], "phases": []} for name, _ in variants}
    for r in range(a.rounds + 1):
        for name, sets in variants:
            apply(sets)
            bm.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            eng.verify_device(0, a.n, *ptrs, bm.data_ptr(), 0, stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            assert torch.equal(bm, full), f"{name}: honest batch rejected"
            ph = eng.verify_device_timed(0, a.n, *ptrs, bm.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            assert torch.equal(bm, full), f"{name}: honest batch rejected (timed)"
            if r:                                   # round 0 is warmup
                res[name]["call"].append(e0.elapsed_time(e1))
                res[name]["phases"].append(list(ph))
    apply([])
    for name, d in res.items():
        c = np.array(d["call"])
        p = np.median(np.array(d["phases"]), axis=0)
        print(json.dumps({"variant": name, "n": a.n, "msg": a.msg, "call_median_ms": float(np.median(c)),
                          "call_min_ms": float(c.min()), "phase_median_ms": [round(float(x), 4) for x in p],
                          "rounds": a.rounds}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
