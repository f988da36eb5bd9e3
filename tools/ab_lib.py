#!/usr/bin/env python3
"""Time one build of the engine (CV_LIB_PATH selects the .so) on the C2 workload: median and min of
`--rounds` verify launches of the whole batch, HIP events on the launch stream.  Run two builds
alternately in separate processes on one box (tools/ab_lib.sh) to A/B a kernel change.

    CV_LIB_PATH=ab/old/libcv_old.so python tools/ab_lib.py --tag old
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--msg", type=int, default=300)
    ap.add_argument("--tag", default=os.environ.get("CV_LIB_PATH", "default"))
    ap.add_argument("--keyed", type=int, default=0, help="key pool size: time the keyed device path")
    args = ap.parse_args()
    eng = native.Engine(1)
    # CV_OPTS="quad_max=0,drain_split=2": per-context options (cv_set_option) for this run
    for kv in filter(None, os.environ.get("CV_OPTS", "").split(",")):
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    if args.keyed:
        return keyed(eng, args)
    stream = torch.cuda.Stream(0)
    torch.cuda.set_stream(stream)
    b = workload.make_batch(eng, 0, args.n, args.msg, seed=1, stream=stream.cuda_stream)
    bm = torch.zeros((args.n + 63) // 64, dtype=torch.int64, device="cuda:0")
    ts = []
    for r in range(args.rounds + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        eng.verify_device(0, args.n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                          b.len.data_ptr(), bm.data_ptr(), 0, stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        assert bool((bm == -1).all()) or args.n % 64, "honest batch rejected"
        if r:
            ts.append(e0.elapsed_time(e1))
    out = {"tag": args.tag, "median_ms": float(np.median(ts)), "min_ms": float(np.min(ts)),
           "verifies_per_s": args.n / (np.median(ts) * 1e-3)}
    if hasattr(native.load(), "cv_ed25519_verify_device_timed"):
        ph = [eng.verify_device_timed(0, args.n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(),
                                      b.off.data_ptr(), b.len.data_ptr(), bm.data_ptr(), stream.cuda_stream)
              for _ in range(3)]
        out["phase_ms"] = [round(float(x), 3) for x in np.median(np.array(ph), axis=0)]
    print(json.dumps(out), flush=True)


def keyed(eng, args):
    stream = torch.cuda.Stream(0)
    torch.cuda.set_stream(stream)
    b = workload.make_batch(eng, 0, args.n, args.msg, seed=1, key_pool=args.keyed, stream=stream.cuda_stream)
    bm = torch.zeros((args.n + 63) // 64, dtype=torch.int64, device="cuda:0")
    a = (0, args.n, b.nkeys, b.pk.data_ptr(), b.key_index.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(),
         b.off.data_ptr(), b.len.data_ptr(), bm.data_ptr(), 0, stream.cuda_stream)
    eng.verify_device_keyed(*a, timed=True)
    ph = np.array([eng.verify_device_keyed(*a, timed=True) for _ in range(args.rounds)])
    assert bool((bm == -1).all()) or args.n % 64, "honest batch rejected"
    med = np.median(ph, axis=0)
    print(json.dumps({"tag": args.tag, "keyed_pool": args.keyed, "phase_ms": [round(float(x), 3) for x in med],
                      "total_ms": float(med.sum()), "verifies_per_s": args.n / (med.sum() * 1e-3)}), flush=True)


if __name__ == "__main__":
    main()
