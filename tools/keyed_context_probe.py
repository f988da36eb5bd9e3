#!/usr/bin/env python3
"""Why the keyed host call is slower inside bench.py than alone: one engine, the keyed host
call (C2, 1,024-key pool, pinned, two async calls in flight) measured fresh, then again after each step of the
bench's sequence — a device-resident keyed run on a torch stream (bench.py keyed_rate), a device-resident
C2 run on two torch streams, C2 host calls from pinned or pageable buffers (bench.py host_api_rate) — with the
host pipeline's phase times per call (--order picks the sequence).

    python tools/keyed_context_probe.py [--calls 8]
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
    ap.add_argument("--calls", type=int, default=8)
    ap.add_argument("--order", default="host,c2_host_pinned,host,c2_host_pageable,host")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = native.Engine(1)
    sh = torch.cuda.Stream(dev)
    n = 1_000_000
    b = workload.make_batch(eng, 0, n, 300, seed=4243, key_pool=1024, stream=sh.cuda_stream)
    host = tuple(eng.host_copy(x) for x in b.to_host())
    del b
    torch.cuda.empty_cache()

    def host_keyed(tag):
        tw = [0.0, 0.0]

        def loop(k):
            pend, bm = [], None
            for _ in range(k):
                t0 = time.perf_counter()
                pend.append(eng.verify_batch_async(*host, want_status=False))
                t1 = time.perf_counter()
                tw[0] += t1 - t0
                if len(pend) == 2:
                    bm, _ = eng.wait(pend.pop(0))
                    tw[1] += time.perf_counter() - t1
            for t in pend:
                bm, _ = eng.wait(t)
            return bm
        loop(2)
        eng.stats("pipe", reset=True)
        tw[0] = tw[1] = 0.0
        t = time.perf_counter()
        bm = loop(a.calls)
        dt = (time.perf_counter() - t) / a.calls
        st = eng.stats("pipe", reset=True)
        assert native.bitmap_to_bools(bm, n).all()
        print(json.dumps({"step": tag, "keyed_host_async_ms_per_call": dt * 1e3,
                          "submit_ms_per_call": tw[0] / a.calls * 1e3, "wait_ms_per_call": tw[1] / a.calls * 1e3,
                          "host_ms_per_call": {k[:-2]: round(v / a.calls * 1e3, 3) for k, v in st.items()
                                               if k.endswith("_s")}}), flush=True)

    def dev_keyed():
        kb = workload.make_batch(eng, 0, n, 300, seed=4242, key_pool=1024, stream=sh.cuda_stream)
        bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
        args = (0, n, kb.nkeys, kb.pk.data_ptr(), kb.key_index.data_ptr(), kb.sig.data_ptr(), kb.arena.data_ptr(),
                kb.off.data_ptr(), kb.len.data_ptr(), bm.data_ptr(), 0, sh.cuda_stream)
        for _ in range(6):
            eng.verify_device_keyed(*args, timed=True)
        torch.cuda.synchronize()
        del kb, bm
        torch.cuda.empty_cache()

    def dev_c2():
        cb = workload.make_batch(eng, 0, n, 300, seed=77, stream=sh.cuda_stream)
        streams = [sh, torch.cuda.Stream(dev)]
        bms = [torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev) for _ in streams]
        torch.cuda.synchronize()
        for k in range(12):
            s = streams[k % 2]
            eng.verify_device(0, n, cb.pk.data_ptr(), cb.sig.data_ptr(), cb.arena.data_ptr(), cb.off.data_ptr(),
                              cb.len.data_ptr(), bms[k % 2].data_ptr(), 0, s.cuda_stream)
        torch.cuda.synchronize()
        del cb, bms
        torch.cuda.empty_cache()

    def c2_host_one(sync_form, nn=None):
        def run():
            cb = workload.make_batch(eng, 0, nn or n, 300, seed=81, stream=sh.cuda_stream)
            pin = tuple(eng.host_copy(x) for x in cb.to_host())
            del cb
            if sync_form:
                for _ in range(4):
                    eng.verify_batch(*pin, want_status=False)
            else:
                pend = []
                for _ in range(4):
                    pend.append(eng.verify_batch_async(*pin, want_status=False))
                    if len(pend) == 2:
                        eng.wait(pend.pop(0))
                for t in pend:
                    eng.wait(t)
            del pin
            torch.cuda.empty_cache()
        return run

    def c2_host_calls(pinned_form, pageable_form):
        def run():
            cb = workload.make_batch(eng, 0, n, 300, seed=78, stream=sh.cuda_stream)
            page = cb.to_host()
            del cb
            torch.cuda.empty_cache()
            if pageable_form:
                for _ in range(4):
                    eng.verify_batch(*page, want_status=False)
            if pinned_form:
                pin = tuple(eng.host_copy(x) for x in page)
                for _ in range(4):
                    eng.verify_batch(*pin, want_status=False)
                pend = []
                for _ in range(4):
                    pend.append(eng.verify_batch_async(*pin, want_status=False))
                    if len(pend) == 2:
                        eng.wait(pend.pop(0))
                for t in pend:
                    eng.wait(t)
                del pin
            if pageable_form:
                pend = []
                for _ in range(4):
                    pend.append(eng.verify_batch_async(*page, want_status=False))
                    if len(pend) == 2:
                        eng.wait(pend.pop(0))
                for t in pend:
                    eng.wait(t)
        return run

    import bench  # noqa: E402  (the bench's own steps, for fidelity)

    def set_stream():
        torch.cuda.set_stream(sh)

    def calibrate():
        eng.calibrate(0)
        eng.calibrate_cycles(0)

    def pcie():
        bench.pcie_h2d_probe(dev)

    def bench_c2_host():
        cb = workload.make_batch(eng, 0, n, 300, seed=79, stream=sh.cuda_stream)
        bench.host_api_rate(eng, cb, 6, 1e8, "c2")
        del cb
        torch.cuda.empty_cache()

    def bench_dev_keyed():
        bench.keyed_rate(eng, 0, n, 300, 5, sh.cuda_stream)
        torch.cuda.empty_cache()

    def c2_host_other_engine():
        # the C2 host calls on a second context, then closed: is the slow state per context or per process?
        other = native.Engine(1)
        cb = workload.make_batch(other, 0, n, 300, seed=80, stream=sh.cuda_stream)
        page = cb.to_host()
        del cb
        pin = tuple(other.host_copy(x) for x in page)
        for _ in range(4):
            other.verify_batch(*pin, want_status=False)
        pend = []
        for _ in range(4):
            pend.append(other.verify_batch_async(*pin, want_status=False))
            if len(pend) == 2:
                other.wait(pend.pop(0))
        for t in pend:
            other.wait(t)
        del pin
        other.close()
        torch.cuda.empty_cache()

    hbuf = torch.empty(4 << 20, dtype=torch.uint8, pin_memory=True)
    dbuf = torch.empty(4 << 20, dtype=torch.uint8, device=dev)

    def dma1():
        # one 4 MB host-to-device copy outside the engine: does the DMA engine a copy lands on rotate per copy?
        dbuf.copy_(hbuf, non_blocking=True)
        torch.cuda.synchronize()

    def c2_async_small_chunks():
        # the asynchronous form with sync-like sub-chunk sizes (many launches per call on the same streams)
        old = eng.get_option("async_chunk")
        eng.set_option("async_chunk", 65536)
        c2_host_one(False)()
        eng.set_option("async_chunk", old)

    def with_opts(fn, **kw):
        def run():
            old = {k: eng.get_option(k) for k in kw}
            for k, v in kw.items():
                eng.set_option(k, v)
            fn()
            for k, v in old.items():
                eng.set_option(k, v)
        return run

    def c2_async_serial():
        # asynchronous calls joined one at a time (the synchronous call's completion pattern)
        cb = workload.make_batch(eng, 0, n, 300, seed=82, stream=sh.cuda_stream)
        pin = tuple(eng.host_copy(x) for x in cb.to_host())
        del cb
        for _ in range(4):
            eng.wait(eng.verify_batch_async(*pin, want_status=False))
        del pin
        torch.cuda.empty_cache()

    steps = {"c2_async_serial": c2_async_serial, "c2_async_quad": with_opts(c2_host_one(False), async_chunk=32768),
             "c2_sync_noquad": with_opts(c2_host_one(True), quad_max=0),
             "c2_async_small": c2_async_small_chunks, "c2_sync_only": c2_host_one(True), "c2_async_only": c2_host_one(False),
             "c2_async_5sub": c2_host_one(False, 5 * 262144), "dma1": dma1, "c2_host_other_engine": c2_host_other_engine, "dev_keyed": dev_keyed, "dev_c2": dev_c2, "c2_host_pinned": c2_host_calls(True, False),
             "c2_host_pageable": c2_host_calls(False, True), "set_stream": set_stream, "calibrate": calibrate,
             "pcie": pcie, "bench_c2_host": bench_c2_host, "bench_dev_keyed": bench_dev_keyed}
    for i, st in enumerate(a.order.split(",")):
        if st == "host":
            host_keyed(f"host#{i}")
        else:
            steps[st]()
            print(json.dumps({"step": st, "done": True}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
