#!/usr/bin/env python3
"""Mean duration per kernel from rocprofv3 kernel-trace CSV output, per launch shape (grid size), so
the whole-chunk 1M launches of the bench's timed phases can be compared with its HIP-event times.

    python tools/trace_summary.py DIR [name-substring ...]   (searches DIR for *kernel_trace.csv)
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
want = sys.argv[2:]
acc = defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0]
    if want and not any(w in name for w in want):
        continue
    acc[(name, int(r["Grid_Size_X"]), r.get("VGPR_Count", ""), r.get("Scratch_Size", ""))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{'launches':>8}  {'mean us':>10}  {'median us':>10}  {'grid':>9}  vgpr scratch  kernel")
for (name, grid, vgpr, scr), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{len(v):8d}  {sum(v) / len(v):10.1f}  {v[len(v) // 2]:10.1f}  {grid:9d}  {vgpr:>4} {scr:>7}  {name}")
