#!/usr/bin/env python3
"""Static instruction mix of the gfx950 kernels (what the VALU will have to issue).

    python tools/isa_stats.py [kernel-substring ...]

Compiles the kernel translation units corda_amd/csrc/cv_k_*.hip to assembly (device only) and prints, per kernel, the
instruction counts by opcode, the scratch (spill) instructions, and the weighted issue cost using
the per-wave-instruction cycle costs measured on the box (tools/microbench/instr_rates.hip).
Static counts: loop bodies count once — use it to compare variants of the same kernel.
"""
import collections
import glob
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = sorted(glob.glob(os.path.join(REPO, "corda_amd", "csrc", "cv_k_*.hip")))

# measured clk per wave64 instruction on MI355X (profiles/README.md, round 2; round 6: profiles/r06a_issue_cost.txt), default 2.4
COST = {"v_mad_u64_u32": 5.0, "v_mad_i64_i32": 5.7, "v_lshrrev_b64": 4.2, "v_lshlrev_b64": 4.2,
        "v_lshl_add_u64": 4.2, "v_ashrrev_i64": 4.2, "v_mul_lo_u32": 4.15, "v_mul_hi_u32": 4.15,
        "v_alignbit_b32": 4.15, "v_lshl_add_u32": 4.15, "v_add3_u32": 4.15, "v_mad_u32_u24": 4.15,
        "v_bitop3_b32": 4.15, "v_lshl_or_b32": 4.15, "v_and_or_b32": 4.15, "v_or3_b32": 4.15,
        "v_perm_b32": 4.15, "v_bfe_u32": 4.15}


def asm(flags=()):
    text = []
    for src in SRCS:
        out = "/tmp/" + os.path.basename(src) + ".s"
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only",
                        "-mllvm", "-amdgpu-sched-strategy=max-ilp", "-S", src, "-o", out, *flags], check=True,
                       stderr=subprocess.DEVNULL)
        text.append(open(out).read())
    return "\n".join(text)


def kernels(s):
    cur, body = None, []
    for line in s.split("\n"):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur and line.startswith("\t") and not line.strip().startswith((".", ";")):
            body.append(line.strip())
        if cur and line.startswith("\t.size"):
            yield cur, body
            cur = None
    if cur:
        yield cur, body


def main():
    want = sys.argv[1:] or ["straus", "prep", "finish"]
    s = asm()
    for name, body in kernels(s):
        if not any(w in name for w in want):
            continue
        ops = collections.Counter(l.split()[0] for l in body)
        valu = {o: c for o, c in ops.items() if o.startswith("v_")}
        cost = sum(c * COST.get(o.split("_e32")[0].split("_e64")[0], 2.4) for o, c in valu.items())
        scratch = sum(c for o, c in ops.items() if o.startswith("scratch_") or o.startswith("buffer_"))
        print(f"{name}: {len(body)} instrs, VALU {sum(valu.values())}, weighted VALU clk {cost:.0f}, "
              f"scratch/buffer {scratch}, s_waitcnt {ops.get('s_waitcnt', 0)}")
        for o, c in ops.most_common(24):
            print(f"    {o:28s} {c}")


if __name__ == "__main__":
    main()
