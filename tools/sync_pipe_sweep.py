#!/usr/bin/env python3
"""Synchronous host-buffer calls (cv_ed25519_verify_batch, default C2: 1M x 300-B records in pinned buffers) under
pipeline settings given as per-context options, interleaved over rounds so box drift hits every setting
alike; one JSON line per (round, setting) with the median call time and the device-API time of the same batch.

    python tools/sync_pipe_sweep.py [--settings "pipe_first=32768,pipe_chunk=262144 pipe_chunk=524288"] [--rounds 3]
"""
import argparse
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
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--msg", type=int, default=300, help="message bytes (C2 300, C5 32)")
    ap.add_argument("--settings", default="base: chunk512:pipe_chunk=524288 chunk1m:pipe_chunk=1048576 "
                                          "first64k:pipe_first=65536,pipe_chunk=524288 nosplit:drain_split=0")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--pageable", type=int, default=0, help="pageable numpy inputs (host threads pack them)")
    a = ap.parse_args()
    eng = native.Engine(1)
    variants = []
    for v in a.settings.split():
        name, _, body = v.partition(":")
        variants.append((name, [(k, int(x)) for k, x in (kv.split("=") for kv in filter(None, body.split(",")))]))
    used = {k for _, sets in variants for k, _ in sets}
    defaults = {k: eng.get_option(k) for k in used}
    b = workload.make_batch(eng, 0, a.n, a.msg, seed=11)
    dev = torch.device("cuda", 0)
    bm_d = torch.zeros((a.n + 63) // 64, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream(dev)
    pinned = list(b.to_host()) if a.pageable else [eng.host_copy(x) for x in b.to_host()]
    for rnd in range(a.rounds):
        for name, sets in variants:
            for k in used:
                eng.set_option(k, defaults[k])
            for k, x in sets:
                eng.set_option(k, x)
            eng.verify_batch(*pinned, want_status=False)
            eng.stats("pipe", reset=True)
            ts = []
            for _ in range(a.reps):
                t = time.perf_counter()
                bm, _ = eng.verify_batch(*pinned, want_status=False)
                ts.append(time.perf_counter() - t)
            assert native.bitmap_to_bools(bm, a.n).all()
            ps = eng.stats("pipe", reset=True)
            calls = max(1.0, ps["calls"])
            host = {k[:-2]: round(ps[k] / calls * 1e3, 3) for k in ("plan_s", "pack_s", "wait_s", "enqueue_s", "sync_s")}
            host["subchunks"] = ps["subchunks"] / calls
            eng.set_option("timeline", 1)
            eng.stats("timeline", reset=True)
            for _ in range(2):
                eng.verify_batch(*pinned, want_status=False)
            tl = eng.stats("timeline", reset=True)
            eng.set_option("timeline", 0)
            tl = {k: round(v / max(1.0, tl["calls"]), 3) for k, v in tl.items() if k != "calls"}
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(3):
                eng.verify_device(0, a.n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                                  b.len.data_ptr(), bm_d.data_ptr(), 0, s.cuda_stream)
            s.synchronize()
            dev_ms = (time.perf_counter() - t) / 3 * 1e3
            med = float(np.median(ts) * 1e3)
            print(json.dumps({"n": a.n, "msg": a.msg, "pageable": a.pageable, "round": rnd, "setting": name, "sync_pinned_ms": round(med, 3),
                              "device_ms": round(dev_ms, 3), "ratio": round(dev_ms / med, 4), "host_ms": host,
                              "timeline": tl}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
