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
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libcordaverify.so")
OBJDIR = os.path.join(HERE, "_obj")
MAPFILE = os.path.join(CSRC, "cordaverify.map")   # export list: the header's cv_* entry points only
ARCH = os.environ.get("CV_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# kernel translation units (cv_kcommon.h) compile in parallel; cv_kernels.hip holds the launchers
SOURCES = ["cv_k_hs.hip", "cv_k_hss.hip", "cv_k_lat.hip", "cv_k_keyed.hip", "cv_k_misc.hip", "cv_kernels.hip",
           "cv_api.cpp"]
# host symbols hidden: the library exports only the cv_* entry points include/cordaverify.h declares
# (cv_api.cpp gives the header's declarations default visibility); the cvk_* launchers stay internal
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
          "-Wno-unused-variable", "-Xarch_host", "-fvisibility=hidden"]
# kernels: LLVM's max-ILP machine scheduler (A/B on one MI355X, 3 alternating rounds: C2 1M verify
# 11.34 -> 11.15 ms median; the iterative-ILP strategy was 5 % slower) — profiles/README.md, round 2
KERNEL_FLAGS = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
# per-translation-unit extra flags (CV_HSS_FLAGS overrides the Straus kernel's, for A/Bs)
SRC_FLAGS = {"cv_k_hss.hip": os.environ["CV_HSS_FLAGS"].split() if os.environ.get("CV_HSS_FLAGS") else []}


def _deps():
    return (glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(REPO, "include", "*.h")) +
            [os.path.abspath(__file__), MAPFILE])


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
    objs, cmds = [], []
    deps = _deps()
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        op = os.path.join(OBJDIR, os.path.splitext(src)[0] + ".o")
        objs.append(op)
        if force or _stale(op, [sp] + deps):
            cmd = [HIPCC] + CFLAGS + KERNEL_FLAGS + SRC_FLAGS.get(src, []) + ["-c", sp, "-o", op]
            if src.endswith(".cpp"):
                # host code only (no kernels): no device pass, so host-only attributes such as target_clones work
                cmd = [HIPCC, "-x", "hip", "--offload-host-only"] + CFLAGS + ["-c", sp, "-o", op]
            cmds.append(cmd)
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    if verbose:
        for cmd in cmds:
            print(" ".join(cmd), flush=True)
    with ThreadPoolExecutor(jobs) as pool:
        for r in pool.map(lambda c: subprocess.run(c, capture_output=True, text=True), cmds):
            if r.returncode:
                sys.stderr.write(r.stderr)
                raise subprocess.CalledProcessError(r.returncode, r.args)
            if verbose and r.stderr.strip():
                sys.stderr.write(r.stderr)
    if force or _stale(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs + ["-lpthread",
                                                                                 f"-Wl,--version-script={MAPFILE}"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
