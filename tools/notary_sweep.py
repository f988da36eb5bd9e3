#!/usr/bin/env python3
"""C4: notary-batch latency sweep (BASELINE.json configs[3]).

Batches of 2^k signatures (k = 8..16) over 32-byte tx ids, 8 signers per transaction, with every
16th item replaced by an adversarial signature from the golden corpus (cycling through its rejected
classes: non-canonical / off-curve / small-order R and A, S >= L, carry loss, cofactored-only,
wrong message or key).  Each repetition is the notary's end-to-end step through the host-buffer
C-ABI: H2D + verify kernels + D2H + per-transaction AND (cv_tx_verdicts).  Reports p50 / p99 over
`--reps` repetitions per size, with signer keys distinct or from a 64-party pool (keyed path), and
the CPU restatement (oracle/, 16 threads) at the same sizes for comparison.

    python tools/notary_sweep.py [--reps 200] [--out gpurun_out/notary_sweep.json]
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
sys.path.insert(0, os.path.join(REPO, "oracle"))

from corda_amd import native, workload  # noqa: E402


def adversarial_pool():
    z = np.load(os.path.join(REPO, "tests", "golden", "ed25519_corpus.npz"))
    rej = np.nonzero(z["verdict"] == 0)[0]
    msgs = [z["arena"][z["off"][i]:z["off"][i] + z["len"][i]].tobytes() for i in rej]
    keep = [j for j, m in enumerate(msgs) if len(m) == 32]        # tx-id-shaped messages
    rej = rej[keep]
    return z["pk"][rej], z["sig"][rej], [msgs[j] for j in keep]


def build(eng, n, key_pool, adv):
    b = workload.make_batch(eng, 0, n, 32, seed=4096 + n, key_pool=key_pool)
    pk, sig, arena, off, ln = b.to_host()
    arena = arena.copy()
    expect = np.ones(n, bool)
    apk, asig, amsg = adv
    for j, i in enumerate(range(0, n, 16)):
        a = j % len(apk)
        pk[i], sig[i] = apk[a], asig[a]
        arena[i * 32:(i + 1) * 32] = np.frombuffer(amsg[a], np.uint8)
        expect[i] = False
    return pk, sig, np.concatenate([arena, np.zeros(16, np.uint8)]), off, ln, expect


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--cpu-reps", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import cv_oracle  # test-infrastructure checker / CPU baseline
    eng = native.Engine(1)
    adv = adversarial_pool()
    threads = int(os.environ.get("CV_CPU_THREADS", "16"))
    rows = []
    for k in range(8, 17):
        n = 1 << k
        row = {"batch": n, "txs": n // 8}
        for label, pool in (("distinct", None), ("pool64", 64)):
            pk, sig, arena, off, ln, expect = build(eng, n, pool, adv)
            tx_begin = np.arange(0, n + 1, 8, dtype=np.uint32)
            lat = []
            for r in range(args.reps + 5):
                t = time.perf_counter()
                bitmap, _ = eng.verify_batch(pk, sig, arena, off, ln, want_status=False)
                txok = native.tx_verdicts(bitmap, tx_begin)
                dt = time.perf_counter() - t
                if r >= 5:
                    lat.append(dt)
            got = native.bitmap_to_bools(bitmap, n)
            ref, _ = cv_oracle.verify_batch(pk, sig, arena, off, ln, nthreads=threads)
            assert np.array_equal(got, ref.astype(bool)), f"verdicts differ from the oracle at n={n} ({label})"
            assert np.array_equal(got, expect)
            row[label] = {"p50_ms": float(np.percentile(lat, 50) * 1e3), "p99_ms": float(np.percentile(lat, 99) * 1e3),
                          "tx_ok": int(txok.sum())}
            if label == "distinct":
                cl = []
                for _ in range(args.cpu_reps):
                    t = time.perf_counter()
                    cv_oracle.verify_batch(pk, sig, arena, off, ln, nthreads=threads)
                    cl.append(time.perf_counter() - t)
                row["cpu_p50_ms"] = float(np.median(cl) * 1e3)
        rows.append(row)
        print(json.dumps(row), flush=True)
    out = {"config": "C4 notary batch sweep, 32-byte tx ids, 8 signers/tx, 1/16 adversarial (golden corpus)",
           "reps": args.reps, "cpu_threads": threads, "rows": rows}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    eng.close()


if __name__ == "__main__":
    main()
