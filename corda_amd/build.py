"""Builds the in-tree native library corda_amd/libcordaverify.so for gfx950.

    python -m corda_amd.build          # or __graft_entry__.build()

hipcc cross-compiles here without a GPU; the .so is git-ignored but travels to the GPU box with the
gpurun snapshot.  Objects are rebuilt only when a source or header is newer than the library.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libcordaverify.so")
OBJDIR = os.path.join(HERE, "_obj")
ARCH = os.environ.get("CV_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = ["cv_kernels.hip", "cv_api.cpp"]
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
          "-Wno-unused-variable"]
# kernels: LLVM's max-ILP machine scheduler (A/B on one MI355X, 3 alternating rounds: C2 1M verify
# 11.34 -> 11.15 ms median; the iterative-ILP strategy was 5 % slower) — DESIGN.md "Kernels"
KERNEL_FLAGS = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]


def _deps():
    return (glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(REPO, "include", "*.h")) +
            [os.path.abspath(__file__)])


def _stale(target: str, inputs) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(p) > t for p in inputs)


def build(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    tables = os.path.join(CSRC, "cv_tables.h")
    gen = os.path.join(CSRC, "gen_tables.py")
    if force or _stale(tables, [gen]):
        subprocess.run([sys.executable, gen], check=True)
    madc, gen_m = os.path.join(CSRC, "cv_madc.h"), os.path.join(CSRC, "gen_madc.py")
    if force or _stale(madc, [gen_m]):
        subprocess.run([sys.executable, gen_m], check=True)
    objs = []
    deps = _deps()
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        op = os.path.join(OBJDIR, os.path.splitext(src)[0] + ".o")
        objs.append(op)
        if force or _stale(op, [sp] + deps):
            cmd = [HIPCC] + CFLAGS + KERNEL_FLAGS + ["-c", sp, "-o", op]
            if src.endswith(".cpp"):
                cmd = [HIPCC, "-x", "hip"] + CFLAGS + ["-c", sp, "-o", op]
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
    if force or _stale(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs + ["-lpthread"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
