#!/usr/bin/env python3
"""Where the host-buffer calls spend host CPU (the two host-runtime effects).

For each scenario — C2 (1M x 300 B, pinned) two async calls in flight with the caller waiting right after
submitting or sleeping first, the synchronous C2 call, and the keyed C2 call (1,024-key pool) async and
sync — prints wall time per call, the process's CPU time per call (user + system), the busiest threads' CPU
per call (psutil), and the cgroup's CPU-throttling counters over the scenario (cpu.stat nr_throttled /
throttled_usec, with cpu.max), so a spinning wait or a CPU quota shows up as numbers.

    python tools/host_cpu_probe.py [--calls 8] [--scenarios c2_async_wait,c2_async_sleep,...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import psutil

# CV_PKG_ROOT: import the corda_amd package (Python mirror + its library) from another tree, e.g. an earlier
# round's build, to compare host behaviour on one box
sys.path.insert(0, os.environ.get("CV_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402


PRE_STREAMS = [0]


def cgroup_stat():
    out = {}
    for p in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat", "/sys/fs/cgroup/cpu,cpuacct/cpu.stat"):
        try:
            for ln in open(p):
                k, v = ln.split()
                out[k] = int(v)
            out["_path"] = p
            break
        except (OSError, ValueError):
            continue
    return out


def cgroup_quota():
    for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            return open(p).read().strip()
        except OSError:
            continue
    return None


def thread_times(proc):
    return {t.id: t.user_time + t.system_time for t in proc.threads()}


def measure(eng, name, fn, calls, proc):
    fn()                                          # warm (pool tables, ring blocks)
    c0, t0, th0 = cgroup_stat(), os.times(), thread_times(proc)
    eng.stats("pipe", reset=True)
    w = time.perf_counter()
    fn(calls)
    wall = time.perf_counter() - w
    st = eng.stats("pipe", reset=True)
    c1, t1, th1 = cgroup_stat(), os.times(), thread_times(proc)
    cpu = (t1.user - t0.user) + (t1.system - t0.system)
    per_thread = sorted(((th1[k] - th0.get(k, 0.0)) / calls * 1e3 for k in th1), reverse=True)[:6]
    d = {k: c1[k] - c0[k] for k in c1 if k in c0 and not k.startswith("_")}
    return {"scenario": name, "wall_ms_per_call": wall / calls * 1e3, "cpu_ms_per_call": cpu / calls * 1e3,
            "cpu_cores_busy": cpu / wall, "top_threads_cpu_ms_per_call": [round(x, 2) for x in per_thread],
            "threads": len(th1), "cgroup_delta": d, "lib": os.environ.get("CV_LIB_PATH") or os.environ.get("CV_PKG_ROOT") or "in-tree",
            "host_ms_per_call": {k[:-2]: round(v / calls * 1e3, 3) for k, v in st.items() if k.endswith("_s")},
            "pre_streams": PRE_STREAMS[0], "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=8)
    ap.add_argument("--scenarios", default="c2_async_wait,c2_async_sleep,c2_sync,keyed_async,keyed_sync")
    ap.add_argument("--sleep-ms", type=float, default=8.0)
    ap.add_argument("--pre-streams", type=int, default=0,
                    help="create and use this many torch streams before the engine (shifts which hardware queues "
                         "the engine's streams land on when there are more streams than GPU_MAX_HW_QUEUES)")
    a = ap.parse_args()
    PRE_STREAMS[0] = a.pre_streams
    import torch
    pre = [torch.cuda.Stream() for _ in range(a.pre_streams)]
    for st in pre:
        with torch.cuda.stream(st):
            torch.ones(16, device="cuda").add_(1)
    torch.cuda.synchronize()
    proc = psutil.Process()
    print(json.dumps({"cpu_max": cgroup_quota(), "affinity": len(os.sched_getaffinity(0)), "nproc": os.cpu_count(),
                      "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cgroup_stat": cgroup_stat(),
                      "pre_streams": a.pre_streams, "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}),
          flush=True)
    eng = native.Engine(1)
    batches = {}

    def get(kind):
        if kind not in batches:
            b = workload.make_batch(eng, 0, 1_000_000, 300, seed=7 if kind == "c2" else 9,
                                    key_pool=1024 if kind == "keyed" else None)
            batches[kind] = tuple(eng.host_copy(x) for x in b.to_host())
            del b
        return batches[kind]

    def async2(kind, sleep_s):
        arrs = get(kind)

        def run(calls=2):
            pend = []
            for _ in range(calls):
                pend.append(eng.verify_batch_async(*arrs, want_status=False))
                if len(pend) == 2:
                    if sleep_s:
                        time.sleep(sleep_s)
                    bm, _ = eng.wait(pend.pop(0))
            for t in pend:
                bm, _ = eng.wait(t)
            assert native.bitmap_to_bools(bm, 1_000_000).all()
        return run

    def sync(kind):
        arrs = get(kind)

        def run(calls=1):
            for _ in range(calls):
                bm, _ = eng.verify_batch(*arrs, want_status=False)
            assert native.bitmap_to_bools(bm, 1_000_000).all()
        return run

    scen = {"c2_async_wait": lambda: async2("c2", 0.0), "c2_async_sleep": lambda: async2("c2", a.sleep_ms / 1e3),
            "c2_sync": lambda: sync("c2"), "keyed_async": lambda: async2("keyed", 0.0),
            "keyed_async_sleep": lambda: async2("keyed", a.sleep_ms / 1e3), "keyed_sync": lambda: sync("keyed")}
    for name in a.scenarios.split(","):
        print(json.dumps(measure(eng, name, scen[name](), a.calls, proc)), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
