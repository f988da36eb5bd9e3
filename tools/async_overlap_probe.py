#!/usr/bin/env python3
"""Does the GPU keep working on an asynchronous host-buffer call while the calling thread is busy before its
next API call?  C2 (1M x 300 B, pinned) async calls with two in flight; after each submit the thread spins
(busy, no API call) for --busy-ms before waiting on the previous call.  With real overlap the period stays at
the GPU time until busy-ms exceeds it.

    python tools/async_overlap_probe.py [--key-pool 0] [--calls 12]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key-pool", type=int, default=0)
    ap.add_argument("--calls", type=int, default=12)
    ap.add_argument("--busy", default="0,1,3,6")
    ap.add_argument("--sleep", type=int, default=0, help="sleep instead of spinning")
    ap.add_argument("--depth", type=int, default=2, help="calls in flight (the engine keeps up to 4 per device)")
    a = ap.parse_args()
    eng = native.Engine(1)
    b = workload.make_batch(eng, 0, 1_000_000, 300, seed=11, key_pool=a.key_pool or None)
    arrs = tuple(eng.host_copy(x) for x in b.to_host())
    del b
    for _ in range(2):
        eng.verify_batch(*arrs, want_status=False)
    for busy in (float(x) for x in a.busy.split(",")):
        t = time.perf_counter()
        pend = []
        for _ in range(a.calls):
            pend.append(eng.verify_batch_async(*arrs, want_status=False))
            if busy:
                if a.sleep:
                    time.sleep(busy / 1e3)
                else:
                    t1 = time.perf_counter() + busy / 1e3
                    while time.perf_counter() < t1:
                        pass
            if len(pend) == a.depth:
                eng.wait(pend.pop(0))
        for tk in pend:
            eng.wait(tk)
        print(f"key_pool {a.key_pool} depth {a.depth} busy {busy} ms{' (sleep)' if a.sleep else ''}: "
              f"{(time.perf_counter() - t) / a.calls * 1e3:.2f} ms per call", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
