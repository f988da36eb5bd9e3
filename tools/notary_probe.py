#!/usr/bin/env python3
"""Where a notary batch's latency goes (C4, BASELINE.json configs[3]): for n in 256 / 4096 / 65536
signatures over 32-byte tx ids (distinct keys, 1/16 adversarial from the golden corpus), p50 of
  host      the host-buffer C-ABI call (cv_ed25519_verify_batch: H2D + kernels + D2H), as the JVM shim
  device    the device-pointer call on resident inputs + stream sync (kernels + launch overhead)
  phases    per-kernel HIP-event times of the same launch group (hash | prep | straus)
so host - device = transfers + host-side work, device - sum(phases) = launch / sync overhead.

    python tools/notary_probe.py [--reps 100]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

from corda_amd import native  # noqa: E402
from notary_sweep import adversarial_pool, build  # noqa: E402


def p50(f, reps):
    ts = []
    for r in range(reps + 5):
        t = time.perf_counter()
        f()
        dt = time.perf_counter() - t
        if r >= 5:
            ts.append(dt)
    return float(np.percentile(ts, 50) * 1e3), float(np.percentile(ts, 99) * 1e3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--sizes", default="256,4096,65536")
    ap.add_argument("--variants", default="base:",
                    help="space-separated 'NAME:OPTION=V,OPTION=V' (cv_set_option names, e.g. small:small_zero_copy=1); "
                         "rounds interleave them")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--pinned", action="store_true", help="also time the host call from pinned (cv_host_alloc) inputs")
    args = ap.parse_args()
    # variants: "name:option=value,option=value ..." (per-context options, cv_set_option names)
    variants = []
    for v in args.variants.split():
        name, _, body = v.partition(":")
        variants.append((name, [(k, int(a)) for k, a in (kv.split("=") for kv in filter(None, body.split(",")))]))
    used = {k for _, sets in variants for k, _ in sets}

    def apply(sets):
        for k in used:
            eng.set_option(k, defaults[k])
        for k, a in sets:
            eng.set_option(k, a)
    eng = native.Engine(1)
    defaults = {k: eng.get_option(k) for k in used}
    adv = adversarial_pool()
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    for n in (int(x) for x in args.sizes.split(",")):
        pk, sig, arena, off, ln, expect = build(eng, n, None, adv)
        for rnd in range(args.rounds):
            for vname, sets in variants:
                apply(sets)
                eng.stats("small", reset=True)
                host = p50(lambda: eng.verify_batch(pk, sig, arena, off, ln, want_status=False), args.reps)
                st = eng.stats("small", reset=True)
                zc_us = {k: round(st[k + "_s"] / max(st["calls"], 1) * 1e6, 1) for k in
                         ("setup", "pack", "launch", "sync", "assemble")} if st["calls"] else None
                pinned = pin_us = None
                if args.pinned:
                    pin = [eng.host_copy(x) for x in (pk, sig, arena, off, ln)]
                    eng.stats("small", reset=True)
                    pinned = p50(lambda: eng.verify_batch(*pin, want_status=False), args.reps)
                    st = eng.stats("small", reset=True)
                    pin_us = {k: round(st[k + "_s"] / max(st["calls"], 1) * 1e6, 1) for k in
                              ("setup", "pack", "launch", "sync", "assemble")} if st["calls"] else None
                    del pin
                bm_h, _ = eng.verify_batch(pk, sig, arena, off, ln, want_status=False)
                assert np.array_equal(native.bitmap_to_bools(bm_h, n), expect)
                d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
                     (("pk", pk), ("sig", sig), ("arena", arena), ("off", off.view(np.int64)), ("len", ln.view(np.int32)))}
                bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
                torch.cuda.synchronize()

                def dev_call():
                    eng.verify_device(0, n, d["pk"].data_ptr(), d["sig"].data_ptr(), d["arena"].data_ptr(),
                                      d["off"].data_ptr(), d["len"].data_ptr(), bm.data_ptr(), 0, s.cuda_stream)
                    s.synchronize()

                device = p50(dev_call, args.reps)
                assert np.array_equal(native.bitmap_to_bools(bm.cpu().numpy().view(np.uint64), n), expect)
                ph = np.median(np.array([eng.verify_device_timed(0, n, d["pk"].data_ptr(), d["sig"].data_ptr(),
                                                                 d["arena"].data_ptr(), d["off"].data_ptr(),
                                                                 d["len"].data_ptr(), bm.data_ptr(), s.cuda_stream)
                                         for _ in range(20)]), axis=0)
                nbytes = pk.nbytes + sig.nbytes + arena.nbytes + off.nbytes + ln.nbytes
                print(json.dumps({"variant": vname, "round": rnd, "n": n, "host_p50_p99_ms": host,
                                  "pinned_p50_p99_ms": pinned,
                                  "device_p50_p99_ms": device,
                                  "phase_ms": {"hash": float(ph[0]), "prep": float(ph[1]), "straus": float(ph[2])},
                                  "input_bytes": int(nbytes), "host_phases_us_mean": zc_us,
                                  "pinned_host_phases_us_mean": pin_us}), flush=True)
        apply([])
    eng.close()


if __name__ == "__main__":
    main()
