#!/usr/bin/env python3
"""Order effect between bench.py's two host C3 steps (separate calls vs cv_verify_transactions_async): both run
in one process with a torch stream current (as bench.py runs them), in the order given, several times.

    python tools/c3_order_probe.py [--order sep,fused,fused,sep,sep,fused] [--steps 4]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from corda_amd import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", default="sep,fused,fused,sep,sep,fused")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--opts", default="", help="name=value,...: set before every step whose name ends in '+'")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    eng = native.Engine(1)
    pcie = bench.pcie_h2d_probe(dev)
    opts = [(k, int(v)) for k, v in (kv.split("=") for kv in filter(None, a.opts.split(",")))]
    defaults = {k: eng.get_option(k) for k, _ in opts}
    for w in a.order.split(","):
        for k, v in opts:
            eng.set_option(k, v if w.endswith("+") else defaults[k])
        fn = bench.host_c3_rate if w.rstrip("+") == "sep" else bench.host_c3_fused_rate
        r = fn(eng, 0, sh, 1_000_000, a.steps, 1.0, pcie)
        print(json.dumps({"what": w, "ms_per_step": round(r["ms_per_step"], 2)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
