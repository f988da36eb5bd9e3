#!/usr/bin/env python3
"""How much of a host-buffer call is the Python mirror's own work (argument checks, the message-extent scan)
rather than the C-ABI call: a C2 batch (1M x 300 B, pinned) through Engine.verify_batch against the same call
made directly through ctypes with the pointers computed once (what a JVM shim with prebuilt buffers does), and
the extent scan alone at C2 (1M records) and C3 leaf (6M) sizes.

    python tools/host_overhead_probe.py [--reps 8]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    import torch  # noqa: F401
    eng = native.Engine(1)
    lib = native.load()
    out = {}
    for n in (1_000_000, 6_000_000):
        off = np.arange(n, dtype=np.uint64) * 32
        ln = np.full(n, 32, np.uint32)
        native._msg_end(lib, off, ln)
        t = time.perf_counter()
        for _ in range(a.reps):
            native._msg_end(lib, off, ln)
        out[f"msg_extent_us_{n}"] = (time.perf_counter() - t) / a.reps * 1e6
    b = workload.make_batch(eng, 0, 1_000_000, 300, seed=3)
    pk, sig, arena, off, ln = (eng.host_copy(x) for x in b.to_host())
    del b
    n = pk.shape[0]
    bm = np.zeros((n + 63) // 64, np.uint64)
    ptrs = [native._p(x) for x in (pk, sig, arena, off, ln)]
    for _ in range(2):
        eng.verify_batch(pk, sig, arena, off, ln, want_status=False)

    def direct():
        rc = lib.cv_ed25519_verify_batch(eng._h, n, *ptrs, native._p(bm), None)
        assert rc == 0

    for name, f in (("python_mirror", lambda: eng.verify_batch(pk, sig, arena, off, ln, want_status=False)),
                    ("direct_c_abi", direct), ("python_mirror_2", lambda: eng.verify_batch(pk, sig, arena, off, ln,
                                                                                              want_status=False)),
                    ("direct_c_abi_2", direct)):
        ts = []
        for _ in range(a.reps):
            t = time.perf_counter()
            f()
            ts.append(time.perf_counter() - t)
        out[f"c2_sync_pinned_ms_{name}"] = float(np.median(ts) * 1e3)
    assert native.bitmap_to_bools(bm, n).all()
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
