#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV by (kernel, grid size): launches, mean / median duration,
VGPRs and scratch bytes, sorted by total time.  Host-side tool (reads the CSV only).

    python tools/trace_by_shape.py gpurun_out/TAG/prof/prof_kernel_trace.csv > profiles/TAG_trace_by_shape.txt
"""
import csv
import statistics
import sys
from collections import defaultdict


def main(path):
    groups = defaultdict(list)
    meta = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0]
            key = (name, int(r["Grid_Size_X"]))
            groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            meta[key] = (int(r["VGPR_Count"]), int(r["Scratch_Size"]))
    rows = sorted(groups.items(), key=lambda kv: -sum(kv[1]))
    print(f"{'launches':>8} {'mean us':>11} {'median us':>11} {'grid':>10} {'vgpr':>5} {'scratch':>7}  kernel")
    for (name, grid), ts in rows:
        v, s = meta[(name, grid)]
        print(f"{len(ts):8d} {statistics.mean(ts):11.1f} {statistics.median(ts):11.1f} {grid:10d} {v:5d} {s:7d}  {name}")


if __name__ == "__main__":
    main(sys.argv[1])
