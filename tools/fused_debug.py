#!/usr/bin/env python3
"""Diagnostic for cv_verify_transactions at C3 size: which transactions a call rejects (honest batch), whether
their ids or their signatures fail, and under which sub-chunk settings.  One JSON line per call.

    python tools/fused_debug.py [--ntx 1000000] [--settings "base: chunk512:pipe_chunk=524288"]
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


def bench_seq(ntx):
    """The sequence of tools/host_paths_probe.py --what c3f: bench.host_c3_fused_rate async (its own batch, freed
    at return), then a fresh batch through the synchronous call — with the separate verify of the same host
    arrays over the claimed ids beside it, to tell bad inputs from a bad fused call."""
    import bench  # noqa: E402
    eng = native.Engine(1)
    r = bench.host_c3_fused_rate(eng, 0, 0, ntx, 2, 1.0, 50.0)
    print(json.dumps({"async_ms_per_step": r["ms_per_step"]}), flush=True)
    signers = 8
    tb = workload.make_tx_batch(eng, 0, ntx, signers, seed=20261016)
    n = ntx * signers
    pin = lambda t: eng.host_copy(t.cpu().numpy())  # noqa: E731
    arena, leaf_off = pin(tb.leaf_arena), eng.host_copy(tb.leaf_off.cpu().numpy().astype(np.uint64))
    leaf_len = eng.host_copy(tb.leaf_len.cpu().numpy().astype(np.uint32))
    tx_begin = eng.host_copy(tb.tx_begin.cpu().numpy().astype(np.uint32))
    claimed = tb.ids.cpu().numpy()
    pk, sig = pin(tb.sigs.pk), pin(tb.sigs.sig)
    del tb
    torch.cuda.empty_cache()
    sig_begin = eng.host_copy(np.arange(0, n + 1, signers, dtype=np.uint32))
    args = (arena, leaf_off, leaf_len, tx_begin, pk, sig, sig_begin)
    msg = np.concatenate([claimed.reshape(-1), np.zeros(16, np.uint8)])
    bm, _ = eng.verify_batch(pk, sig, msg, (np.arange(n, dtype=np.uint64) // signers) * 32,
                             np.full(n, 32, np.uint32), want_status=False)
    sep_bad = np.nonzero(~native.bitmap_to_bools(bm, n))[0]
    for rep in range(3):
        for kw in (dict(want_status=False), dict(want_status=True, want_sig_status=True)):
            out = eng.verify_transactions(*args, ids=eng.host_empty((ntx, 32)), **kw)
            bad = np.nonzero(out[0] == 0)[0]
            sst = out[3]
            print(json.dumps({"rep": rep, "kw": str(kw), "separate_bad_sigs": int(sep_bad.size),
                              "separate_first": sep_bad[:6].tolist(), "fused_rejected": int(bad.size),
                              "fused_first": bad[:6].tolist(), "fused_last": bad[-3:].tolist(),
                              "ids_wrong": int((out[1] != claimed).any(axis=1).sum()),
                              "sig_status_nonzero": None if sst is None else int((sst != 0).sum())}), flush=True)
    eng.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ntx", type=int, default=1_000_000)
    ap.add_argument("--settings", default="base:")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--forms", default="sync,async")
    ap.add_argument("--outs", default="sst=1,st=1,pin=0 sst=0,st=0,pin=1 sst=0,st=1,pin=0 sst=1,st=0,pin=1",
                    help="output variants: sig status, tx status, ids into pinned memory")
    ap.add_argument("--bench-seq", action="store_true")
    a = ap.parse_args()
    if a.bench_seq:
        return bench_seq(a.ntx)
    eng = native.Engine(1)
    signers = 8
    ntx = a.ntx
    tb = workload.make_tx_batch(eng, 0, ntx, signers, seed=20261016)
    eng.synchronize(0)          # the batch is signed on the engine's stream, which torch's copies do not wait for
    n = ntx * signers
    pin = lambda t: eng.host_copy(t.cpu().numpy())  # noqa: E731
    arena, leaf_off = pin(tb.leaf_arena), eng.host_copy(tb.leaf_off.cpu().numpy().astype(np.uint64))
    leaf_len = eng.host_copy(tb.leaf_len.cpu().numpy().astype(np.uint32))
    tx_begin = eng.host_copy(tb.tx_begin.cpu().numpy().astype(np.uint32))
    claimed = tb.ids.cpu().numpy()
    pk, sig = pin(tb.sigs.pk), pin(tb.sigs.sig)
    del tb
    torch.cuda.empty_cache()
    sig_begin = eng.host_copy(np.arange(0, n + 1, signers, dtype=np.uint32))
    args = (arena, leaf_off, leaf_len, tx_begin, pk, sig, sig_begin)
    defaults = {k: eng.get_option(k) for k in native.OPTIONS}
    for v in a.settings.split():
        name, _, body = v.partition(":")
        for k, x in defaults.items():
            eng.set_option(k, x)
        for kv in filter(None, body.split(",")):
            k, x = kv.split("=")
            eng.set_option(k, int(x))
        for form in a.forms.split(","):
          for ov in a.outs.split():
            fl = {k: int(x) for k, x in (kv.split("=") for kv in ov.split(","))}
            kw = dict(want_sig_status=bool(fl["sst"]), want_status=bool(fl["st"]))
            for rep in range(a.reps):
                idb = eng.host_empty((ntx, 32)) if fl["pin"] else None
                t_call = time.perf_counter()
                if form == "sync":
                    ok, ids, st, sst = eng.verify_transactions(*args, ids=idb, **kw)
                else:
                    t1 = eng.verify_transactions_async(*args, **kw)
                    t2 = eng.verify_transactions_async(*args, ids=idb, **kw)
                    eng.wait(t1)
                    ok, (ids, st, sst) = eng.wait(t2)
                ms = (time.perf_counter() - t_call) * 1e3
                st = np.zeros(1) if st is None else st
                sst = np.zeros(1) if sst is None else sst
                bad = np.nonzero(ok == 0)[0]
                idbad = np.nonzero((ids != claimed).any(axis=1))[0]
                print(json.dumps({"setting": name, "form": form, "outs": ov, "rep": rep, "ms": round(ms, 2), "rejected": int(bad.size),
                                  "ids_wrong": int(idbad.size), "status_nonzero": int((st != 0).sum()),
                                  "sig_status_nonzero": int((sst != 0).sum()),
                                  "first_rejected": bad[:12].tolist(), "first_ids_wrong": idbad[:12].tolist(),
                                  "rejected_ranges": [int(bad.min()), int(bad.max())] if bad.size else None}),
                      flush=True)
    eng.close()


if __name__ == "__main__":
    main()
