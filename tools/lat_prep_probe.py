#!/usr/bin/env python3
"""Latency-prep time (fused scalars + points launch of the tri form) of a notary-sized batch, honest vs
with the C4 adversarial mix, and with the adversarial records all in ONE wave vs spread (every 16th):
shows whether the prep's critical path is the point lanes or the slowest scalar wave.

    python tools/lat_prep_probe.py [--n 4096] [--reps 30]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from corda_amd import native, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    eng = native.Engine(1)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    adv = workload.adversarial_records(os.path.join(REPO, "tests", "golden", "ed25519_corpus.npz"))
    n = a.n
    b = workload.make_batch(eng, 0, n, 32, seed=99)
    honest = b.to_host()
    spread = workload.notary_batch(eng, 0, n, adv)[:5]
    pk, sig, arena, off, ln = (x.copy() for x in honest)
    apk, asig, amsg = adv
    k = min(64, len(apk))                         # adversarial records packed into the first wave
    pk[:k], sig[:k] = apk[:k], asig[:k]
    arena = arena.copy()
    for i in range(k):
        arena[int(off[i]):int(off[i]) + 32] = amsg[i]
    packed = (pk, sig, arena, off, ln)
    for name, arrs in (("honest", honest), ("adv_spread", spread), ("adv_one_wave", packed)):
        d = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in
             (arrs[0], arrs[1], arrs[2], arrs[3].view(np.int64), arrs[4].view(np.int32))]
        bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
        ph = np.median(np.array([eng.verify_device_timed(0, n, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                                         d[3].data_ptr(), d[4].data_ptr(), bm.data_ptr(),
                                                         s.cuda_stream) for _ in range(a.reps)]), axis=0)
        print(json.dumps({"batch": name, "n": n, "prep_us": float(ph[0] * 1e3), "straus_us": float(ph[2] * 1e3)}),
              flush=True)
    eng.close()


if __name__ == "__main__":
    main()
