#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (scripts/pmc.sh) per kernel, and write the HBM-traffic record of
the dominant kernel that bench.py reports as roofline.traffic.

    python tools/pmc_summary.py gpurun_out/<tag>/pmc N_SIGNATURES [--kernel cv_hs_straus_kernel]
                                [--out profiles/pmc_hs_straus.json]

Counter values are averaged over the dispatches of each kernel.  HBM bytes follow
MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half
the bytes of 16-B-per-lane reads (every load of the verify kernels is a 16-B-per-lane global_load),
so the read bytes are 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B-per-lane stores.
"""
import collections
import csv
import glob
import json
import os
import sys


def load(pmc_dir):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in per.items()}


def main():
    pmc_dir, n = sys.argv[1], int(sys.argv[2])
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    data = load(pmc_dir)
    for k, d in sorted(data.items()):
        print(k)
        for c, v in sorted(d.items()):
            print(f"    {c:28s} {v:.6g}")
    want = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "cv_straus_kernel"
    key = next((k for k in data if want in k), None)
    if key is None:
        print(f"no {want} dispatches found")
        return
    d = data[key]
    rec = {"kernel": key, "n": n, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (scripts/pmc.sh)",
           "fetch_kib_raw": d.get("FETCH_SIZE"), "write_kib": d.get("WRITE_SIZE")}
    if rec["fetch_kib_raw"] is not None and rec["write_kib"] is not None:
        rd = 2 * rec["fetch_kib_raw"] * 1024
        wr = rec["write_kib"] * 1024
        rec.update(read_bytes=rd, write_bytes=wr, hbm_bytes_per_launch=rd + wr,
                   bytes_per_verify=(rd + wr) / n)
    for c in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVES",
              "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "SQ_WAIT_INST_ANY", "GRBM_GUI_ACTIVE"):
        if c in d:
            rec[c] = d[c]
    print(json.dumps(rec, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
