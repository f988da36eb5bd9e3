import sys, os, time, json
sys.path.insert(0, os.getcwd())
import torch, numpy as np
import bench
from corda_amd import native, workload
eng = native.Engine(1)
b = workload.make_batch(eng, 0, 8_000_000, 32, seed=5)
r = bench.host_api_rate(eng, b, 3, 1.0, "c5", async_steps=8)
print(json.dumps({"first": [r["ms_per_step"], r["sync_pinned"]["ms_per_step"], r["async_pageable"]["ms_per_step"], r["pageable"]["ms_per_step"]]}), flush=True)
r = bench.host_api_rate(eng, b, 3, 1.0, "c5", async_steps=8)
print(json.dumps({"second": [r["ms_per_step"], r["sync_pinned"]["ms_per_step"], r["async_pageable"]["ms_per_step"], r["pageable"]["ms_per_step"]]}), flush=True)
