#!/usr/bin/env python3
"""Time the device Merkle-id call (leaf SHA-256 + per-tx tree) on the C3 leaf shape, for A/B of the
leaf-hash kernel (CV_LIB_PATH selects the .so).  --sort-leaves hashes the same leaves ordered by
length (the ids are then not transaction ids: a divergence experiment, timing only).

    CV_LIB_PATH=ab/x/libcv.so python tools/merkle_probe.py --ntx 1000000
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ntx", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--sort-leaves", action="store_true")
    ap.add_argument("--tag", default=os.environ.get("CV_LIB_PATH", "default"))
    ap.add_argument("--leaf-mode", type=int, default=-1, help="(ignored: one leaf kernel since round 4)")
    args = ap.parse_args()
    eng = native.Engine(1)
    tb = workload.make_tx_batch(eng, 0, args.ntx, signers=1)
    off, ln = tb.leaf_off, tb.leaf_len
    if args.sort_leaves:
        order = torch.argsort(ln, stable=True)
        off, ln = off[order].contiguous(), ln[order].contiguous()
    nleaves = int(ln.numel())
    ws = torch.empty(nleaves * 32, dtype=torch.uint8, device="cuda:0")
    ids = torch.empty((args.ntx, 32), dtype=torch.uint8, device="cuda:0")
    ts = []
    st = torch.cuda.Stream(0)          # the call runs on this stream, so the events bracket it
    torch.cuda.synchronize()
    for r in range(args.reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        eng.merkle_device(0, args.ntx, nleaves, tb.leaf_arena.data_ptr(), off.data_ptr(), ln.data_ptr(),
                          tb.tx_begin.data_ptr(), ws.data_ptr(), ids.data_ptr(), 0, st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        if r:
            ts.append(e0.elapsed_time(e1))
    same = bool(torch.equal(ids, tb.ids)) if not args.sort_leaves else None
    import bench  # the repo root is on sys.path
    comp = bench.merkle_compressions(ln, tb.tx_begin)
    print(json.dumps({"tag": args.tag, "leaf_mode": args.leaf_mode, "ntx": args.ntx, "sorted": args.sort_leaves,
                      "median_ms": float(np.median(ts)), "min_ms": float(np.min(ts)),
                      "ids_match_generation": same, "compressions": comp,
                      "ids_sha256": hashlib.sha256(ids.cpu().numpy().tobytes()).hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
