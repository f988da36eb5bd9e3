#!/usr/bin/env python3
"""Small-batch scaling of the latency launch group (diagnostic): device-timed phases for n = 256 ..
16384 with and without the 1/16 golden adversarial items (tools/notary_sweep.py mix)."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from corda_amd import native, workload  # noqa: E402
from notary_sweep import adversarial_pool, build  # noqa: E402

eng = native.Engine(1)
lib = native.load()
import ctypes  # noqa: E402
for kv in filter(None, os.environ.get("CV_KNOBS", "").split(",")):   # e.g. cvk_set_prep_lat_fused=0
    k, v = kv.split("=")
    getattr(lib, k).argtypes = [ctypes.c_int]
    getattr(lib, k)(int(v))
adv = adversarial_pool()
dev = torch.device("cuda", 0)
# python tools/lat_scaling.py [SIZES [MIXES]]   e.g. 4096 1  (one size, adversarial only)
sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else (256, 1024, 4096, 16384)
mixes = [bool(int(x)) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else (False, True)
for n in sizes:
    for mix in mixes:
        if mix:
            pk, sig, arena, off, ln, _ = build(eng, n, None, adv)
        else:
            b = workload.make_batch(eng, 0, n, 32, seed=77 + n)
            pk, sig, arena, off, ln = b.to_host()
            arena = np.concatenate([arena, np.zeros(16, np.uint8)])
        d = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in
             (pk, sig, arena, off.view(np.int64), ln.view(np.int32))]
        bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
        ph = np.median(np.array([eng.verify_device_timed(0, n, *[t.data_ptr() for t in d], bm.data_ptr())
                                 for _ in range(30)]), axis=0)
        print(json.dumps({"n": n, "adversarial": mix, "phase_ms": [round(float(x), 4) for x in ph]}), flush=True)
