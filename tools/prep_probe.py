#!/usr/bin/env python3
"""Phase cycles of the fused prep kernel and the cycle-basis MAC peak, on the C2 workload.

    python tools/prep_probe.py [--n 1000000] [--msg 300]

Prints one JSON line: cv_diag_prep_phases (mean shader cycles per wave of hash | lattice | digits |
decode A+R | tables) and cv_calibrate_cycles.  Diagnostic only (DESIGN.md "Measurement").
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--msg", type=int, default=300)
    args = ap.parse_args()
    eng = native.Engine(1)
    stream = torch.cuda.Stream(0)
    torch.cuda.set_stream(stream)
    b = workload.make_batch(eng, 0, args.n, args.msg, seed=1, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    ptrs = (b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(), b.len.data_ptr())
    out = {"n": args.n, "msg": args.msg}
    eng.diag_prep_phases(0, args.n, *ptrs)
    ph = eng.diag_prep_phases(0, args.n, *ptrs)
    tot = ph["total"]
    ph["share"] = {k: round(ph[k] / tot, 4) for k in ("hash", "lattice", "digits", "decode", "tables")}
    out["prep_phase_cycles_per_wave"] = ph
    out["mad_clock"] = eng.calibrate_cycles(0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
