#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (scripts/pmc.sh) per kernel, and write the HBM-traffic record of
the dominant kernel that bench.py reports as roofline.traffic.

    python tools/pmc_summary.py gpurun_out/<tag>/pmc N_SIGNATURES [--kernel cv_hs_straus_kernel]
                                [--out profiles/pmc_hs_straus.json] [--mac 130460]

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


SIMDS = 1024          # 256 CUs x 4 SIMDs
XCDS = 8              # GRBM_GUI_ACTIVE is summed over the XCDs (MI355X_MICROARCH.md "DVFS give-back")


def derived(d: dict, n: int, mac: float) -> dict:
    """Issue model of one kernel from its counters (means over its dispatches; the counters of one pass each):
    kernel cycles = GRBM_GUI_ACTIVE / 8; SQ_WAVE_CYCLES / SQ_ACTIVE_INST_ANY / SQ_WAIT_* count quad-cycles
    (MI355X_MICROARCH.md, "s_memtime tick vs SQ PMC units"), so x 4 gives cycles.
      occupancy            mean resident waves per SIMD = 4 SQ_WAVE_CYCLES / (kernel cycles x 1,024)
      simd_cycles_per_valu SIMD cycles per VALU wave-instruction = kernel cycles x 1,024 / SQ_INSTS_VALU
      issue_active         share of SIMD cycles in which a wave issued = 4 SQ_ACTIVE_INST_ANY / (cycles x 1,024)
      valu_per_verify      VALU instructions per lane (= per verify, one signature per lane) = SQ_INSTS_VALU / (n/64)
      valu_per_mac         valu_per_verify / the kernel's MAC count per verify"""
    out = {}
    ga = d.get("GRBM_GUI_ACTIVE")
    if not ga:
        return out
    cyc = ga / XCDS
    out["kernel_cycles"] = cyc
    if d.get("SQ_WAVE_CYCLES"):
        out["occupancy_waves_per_simd"] = 4 * d["SQ_WAVE_CYCLES"] / (cyc * SIMDS)
        for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
            if c in d:
                out[f"share_of_wave_cycles_{c}"] = d[c] / d["SQ_WAVE_CYCLES"]
    if d.get("SQ_ACTIVE_INST_ANY"):
        out["issue_active"] = 4 * d["SQ_ACTIVE_INST_ANY"] / (cyc * SIMDS)
    if d.get("SQ_INSTS_VALU"):
        out["simd_cycles_per_valu"] = cyc * SIMDS / d["SQ_INSTS_VALU"]
        out["valu_per_verify"] = d["SQ_INSTS_VALU"] / (n / 64)
        if mac:
            out["valu_per_mac"] = out["valu_per_verify"] / mac
        if d.get("SQ_INSTS_VALU_INT64"):
            out["int64_share_of_valu"] = d["SQ_INSTS_VALU_INT64"] / d["SQ_INSTS_VALU"]
    return out


def main():
    pmc_dir, n = sys.argv[1], int(sys.argv[2])
    mac = float(sys.argv[sys.argv.index("--mac") + 1]) if "--mac" in sys.argv else 130460.0
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
              "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "SQ_WAIT_INST_ANY", "GRBM_GUI_ACTIVE", "SQ_INSTS_VALU_INT64",
              "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY"):
        if c in d:
            rec[c] = d[c]
    rec["derived"] = derived(d, n, mac)
    print(json.dumps(rec["derived"], indent=1))
    print(json.dumps(rec, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
