#!/usr/bin/env python3
"""Mean duration per kernel name from rocprofv3 kernel-trace CSV output (diagnostic).

    python tools/trace_summary.py DIR     (searches DIR for *kernel_trace.csv)
"""
import csv
import glob
import os
import sys
from collections import defaultdict

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    with open(f) as fh:
        rows += list(csv.DictReader(fh))
acc = defaultdict(list)
for r in rows:
    acc[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{len(v):6d}  mean {sum(v) / len(v):9.2f} us  median {v[len(v) // 2]:9.2f} us  {k}")
