#!/usr/bin/env python3
"""Where a pipelined call's GPU time goes, from a rocprofv3 --kernel-trace CSV (host-side tool, reads the CSV only):
inside a window of the trace, the union of kernel intervals (busy), the time each kernel class runs ALONE (no other
class on the GPU), the time two or more classes overlap, and the idle gaps.  A class running alone for long is a
stretch where the chip holds only that kernel's waves (e.g. a Merkle tree kernel or a part-round Straus tail).

    python tools/trace_concurrency.py TRACE.csv [--marker cv_tx_verdict_kernel --first 4 --last 8]

The window runs from the end of the `first`-th to the end of the `last`-th launch of `marker` (1-based; defaults: the
whole trace).  For the fused transaction call the marker is its one per-call verdict kernel.
"""
import argparse
import csv
from collections import defaultdict

CLASSES = (("hs_straus", "straus"), ("points", "points"), ("scalars", "scalars"), ("leaf_hash", "merkle_leaf"),
           ("merkle_tree", "merkle_tree"), ("tx_sig_refs", "sig_refs"), ("tx_verdict", "verdict"))


def klass(name: str) -> str:
    for pat, k in CLASSES:
        if pat in name:
            return k
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default=None)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    lo, hi = rows[0][0], max(r[1] for r in rows)
    if a.marker:
        ends = sorted(e for s, e, n in rows if a.marker in n)
        lo = ends[a.first - 1] if a.first else lo
        hi = ends[a.last - 1] if a.last else hi
    ev = []
    dur = defaultdict(float)
    launches = defaultdict(int)
    for s, e, n in rows:
        s, e = max(s, lo), min(e, hi)
        if e <= s:
            continue
        k = klass(n)
        ev.append((s, 1, k))
        ev.append((e, -1, k))
        dur[k] += (e - s) / 1e6
        launches[k] += 1
    ev.sort(key=lambda x: (x[0], x[1]))
    active = defaultdict(int)
    alone = defaultdict(float)
    multi = idle = 0.0
    gaps = []
    t_prev = lo
    for t, d, k in ev:
        dt = (t - t_prev) / 1e6
        if dt > 0:
            ks = [c for c, v in active.items() if v > 0]
            if not ks:
                idle += dt
                gaps.append(dt)
            elif len(ks) == 1:
                alone[ks[0]] += dt
            else:
                multi += dt
        active[k] += d
        t_prev = t
    span = (hi - lo) / 1e6
    print(f"window {span:.3f} ms: busy {span - idle:.3f}, idle {idle:.3f} ({len(gaps)} gaps, "
          f"{sum(g for g in gaps if g > 0.05):.3f} ms in gaps > 50 us), two or more classes {multi:.3f} ms")
    print(f"{'class':>12} {'launches':>8} {'sum of durations ms':>20} {'alone ms':>9}")
    for k in sorted(dur, key=lambda k: -dur[k]):
        print(f"{k:>12} {launches[k]:8d} {dur[k]:20.3f} {alone[k]:9.3f}")


if __name__ == "__main__":
    main()
