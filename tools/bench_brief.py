#!/usr/bin/env python3
"""Print the headline numbers of a bench.py JSON line (last line of the given log)."""
import json
import sys

d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(f"C2 {d['value'] / 1e6:.1f} M/s  {d['ms_per_step']:.3f} ms/step  hs frac {r['frac']:.3f}  phases {r['phase_ms']}")
print(f"group frac {r['group']['frac']:.3f}  cycle basis {r.get('cycle_basis', {}).get('frac_vs_measured_clock')}")
for k in ("c3", "c5_shard", "keyed"):
    if k in d:
        print(f"{k} {d[k]['value'] / 1e6:.1f} M/s {d[k]['ms_per_step']:.2f} ms phases {d[k].get('phase_ms')}")
n = d.get("notary", {})
print(f"notary 4096 p50 {n.get('p50_ms')} p99 {n.get('p99_ms')}  sweep " +
      " ".join(f"{s['batch']}:{s['p50_ms']:.3f}" for s in d.get("notary_sweep", [])))
if "cpu_baseline" in d:
    print(f"cpu_baseline {d['cpu_baseline']['value']:.0f} {d['cpu_baseline']['unit']} cores {d['cpu_baseline']['cores']}")
