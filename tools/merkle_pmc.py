#!/usr/bin/env python3
"""Merkle-kernel PMC record for bench.py's c3.merkle_roofline (MERKLE_PMC_FILE).

    python tools/merkle_pmc.py gpurun_out/<tag>/pmc_merkle PROBE_JSON --out profiles/r03_pmc_merkle.json

PMC_DIR holds rocprofv3 --pmc passes over tools/merkle_probe.py (SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU,
SQ_ACTIVE_INST_VALU ...); PROBE_JSON is that probe's JSON line (its "compressions" field counts the
leaf blocks and internal nodes of the same batch).  Derived per SHA-256 compression:
  valu_lane_slots_per_compression       64 x wave-instructions / compressions (idle lanes included)
  valu_active_lane_instr_per_compression SQ_THREAD_CYCLES_VALU-weighted: lane-instructions that did work
  lane_utilisation                      active lanes per issued wave-instruction / 64
  instr_efficiency_vs_floor             bench.SHA256_FLOOR_INSTR / active lane-instructions
Leaf and tree kernels are summed (the unit spans both)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tools.pmc_summary import load  # noqa: E402


def main():
    pmc_dir, probe = sys.argv[1], sys.argv[2]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    with open(probe) as f:
        line = [json.loads(x) for x in f if x.startswith("{")][-1]
    comp = line["compressions"]
    data = load(pmc_dir)
    rec = {"source": "rocprofv3 --pmc over tools/merkle_probe.py (scripts/pmc_merkle.sh)", "ntx": line["ntx"],
           "compressions": comp, "median_ms": line["median_ms"], "kernels": {}}
    tot_v = tot_t = 0.0
    for k, d in data.items():
        if "leaf_hash" in k or "merkle_tree" in k:
            rec["kernels"][k] = d
            tot_v += d.get("SQ_INSTS_VALU", 0.0)
            tot_t += d.get("SQ_THREAD_CYCLES_VALU", 0.0)
    c = comp["total"]
    rec["SQ_INSTS_VALU"] = tot_v
    rec["valu_lane_slots_per_compression"] = 64 * tot_v / c
    if tot_t:
        # SQ_THREAD_CYCLES_VALU sums the active lanes of every VALU wave-instruction on this chip
        # (round-2 reading: 6.48e10 / (64 x 1.25e9) = 0.81 lane utilisation of the unsorted-by-length
        # kernel agreed with the leaf-length mix), so it is the count of lane-instructions that did work
        act = sum(d.get("SQ_ACTIVE_INST_VALU", 0.0) for d in rec["kernels"].values())
        rec["lane_utilisation"] = tot_t / (64 * act) if act else None
        rec["valu_active_lane_instr_per_compression"] = tot_t / c
        rec["instr_efficiency_vs_floor"] = bench.SHA256_FLOOR_INSTR / (tot_t / c)
        rec["lane_utilisation_per_kernel"] = {
            k: d["SQ_THREAD_CYCLES_VALU"] / (64 * d["SQ_ACTIVE_INST_VALU"])
            for k, d in rec["kernels"].items() if d.get("SQ_ACTIVE_INST_VALU")}
    rec["leaf_mode"] = line.get("leaf_mode")
    print(json.dumps(rec, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
