#!/usr/bin/env python3
"""Throughput bench of the MI355X Ed25519 verify engine (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W] [--config c2|c5] [--n PER_GPU]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`--gpus N` with N > 1 and no launcher environment (WORLD_SIZE unset): the process starts N fresh ranks of
itself (corda_amd/launch.py: RANK / LOCAL_RANK / WORLD_SIZE set, before any GPU call, no exec) and exits
with their status; with fewer than N visible GPUs it exits 2 and names the count.  A WORLD_SIZE that
differs from --gpus is an error too, so a line never reports a GPU count other than the one asked for.

A "step" = one verify pass over the whole per-GPU batch (inputs resident in HBM; the engine's
production launch plan), plus — for N > 1 —
the RCCL all-gather of the verdict bitmaps that feeds the notary commit step.  Weak scaling: every
rank verifies its own N_PER_GPU signatures.  value = all signatures verified by all ranks / the max
over ranks of the timed region.  N > 1 adds two sub-lines (BASELINE.json configs[4]):
  c5           8M signatures over 32-byte ids per rank (64M at N = 8), RCCL all-gather of the bitmaps
               inside every timed step, the gathered bitmap checked all-ones
  c_abi_multi  the JVM node's form: ONE process, cv_open(0) over every visible GPU, the N x 8M C5 batch
               from pinned host buffers through cv_ed25519_verify_batch (routed over the devices by the
               engine, no collective), against the same call on one device

Default workload (N=1): BASELINE config C2 — 1,000,000 single-signer Ed25519 signatures over
300-byte messages, distinct key per signature, generated on the GPU by the engine's signer.

Extra fields on the JSON line:
  roofline      VALU-issue roofline of the dominant kernel (cv_hs_straus_kernel: 130,460 32x32->64
                MACs per verify) against the measured v_mad_u64_u32
                peak of this GPU, kernel time from HIP events on whole-chunk launches of the same
                batch; "group" = the whole launch group against its own MAC count
  roofline.cycle_basis  the same peak priced per shader cycle (SIMDs x 64 / cycles per wave-level
                v_mad_u64_u32 x the clock measured over the calibration launch), and against 2.4 GHz
  cpu_baseline  oracle/ C restatement of eddsa-0.1.0 verify (rank 0, N=1 only, bounded sample) on the
                host cores this process may use (capped by the box's OMP_NUM_THREADS share)
  c3, c5_shard  BASELINE configs C3 (1M txs x 8 signers: Merkle tx-id recompute + 8M verifies) and
                C5 (8M-signature shard) on the same GPU: value, tx_ids_per_s, phases, roofline
  host_api      the drop-in (host-buffer) path at C2, C5, C3 and keyed C2 (1,024-key pool), against the
                device-resident rates of the same run
  notary        C4: p50/p99 end-to-end latency of a 4096-signature notary batch (host buffers in and
                out, 1/16 adversarial records from the golden corpus's rejected classes), with the
                p50 breakdown (transfers + host, launch + sync, per kernel) and the CPU restatement on
                the same batch; notary_sweep = the same at 2^k, k = 8..16 (k != 12), pageable p50/p99, with
                notary_sweep_pinned the p50 from cv_host_alloc inputs; notary_keyed = 64 signers
  resolve_chain p50/p99 latency of a 5,000-tx dependency chain (2 signers/tx, 6 leaves/tx): one
                Merkle call + one verify call + per-tx AND with the id check
The printed line keeps every headline value and stays under ~4 KB; per-kernel breakdowns and the full
sub-line dicts go to gpurun_out/bench_detail.json (--detail PATH).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# Hardware queues per device (HIP reads GPU_MAX_HW_QUEUES when it starts): recorded in the line, not set
# here.  Round 4 same-box A/B of this line at 4 (HIP's default, what the GPU box exports) vs 8 queues:
# 9.22 vs 9.30 ms per C2 call, medians of 3 alternating fresh-process runs (profiles/r04_queue_ab.log).
HW_QUEUES = os.environ.get("GPU_MAX_HW_QUEUES")

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from corda_amd import distributed as D, native, workload  # noqa: E402

W_MAC_PER_VERIFY = 2.28e5       # algorithmic 32x32->64 MACs per verify (32-byte msg)
# Straus phase alone (cv_straus_kernel, the dominant kernel): 63 windows x (16 S + 13 M) + 64 -A adds x 7 M
# + 32 B madds x 7 M = 1008 S + 1491 M, at S = 55 and M = 100 limb products (profiles/README.md, round 1)
W_MAC_STRAUS = 1008 * 55 + 1491 * 100
# Half-size schedule, cv_hs_straus_kernel at the typical 33 windows:
# 32 x 4 doublings (16 S + 13 M) + 33 x (R add + A add: 15 M) + 8 x 2 B madds from the radix-2^16
# rows (14 M per B window) = 512 S + 1023 M  (round 2 start: 16 B windows from radix-256 rows, 1135 M)
HS_NW = 33
HS_BWIN = 8
W_MAC_HS_STRAUS = (HS_NW - 1) * (16 * 55 + 13 * 100) + HS_NW * 15 * 100 + HS_BWIN * 14 * 100
# whole half-size group: + 2 point decodes (254 S + 19 M each) + 2 odd-multiple tables (4 S + 59 M each)
W_MAC_HS_GROUP = W_MAC_HS_STRAUS + 2 * (258 * 55 + 78 * 100)
# keyed comb (cv_comb_kernel): 7 x 8 = 56 doublings (4 S + 3 M each, the last of a window
# 4 S + 4 M) + 32 key-row and 16 basepoint mixed additions (7 M each with their conversion) = 224 S + 535 M per verify
W_MAC_COMB = 224 * 55 + 535 * 100
MSG_BYTES = {"c2": 300, "c5": 32, "c3": 32}
CONFIG_NAME = {
    "c2": "C2: 1M single-signer Ed25519 txs, 300-byte msg, distinct keys, SoA batch",
    "c5": "C5 shard: 8M single-signer sigs per GPU over 32-byte tx ids",
    "c3": "C3: IRS-shaped 1M txs x 8 signers per GPU, SHA-256 Merkle tx-id recompute + 8M verifies",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# The PMC record of the dominant kernel on the current kernel code: scripts/pmc.sh + tools/pmc_summary.py, named
# with the commit it was measured on (the round-3 file described an older build)
PMC_HS_FILE = "profiles/pmc_hs_straus_r06.json"


def pmc_traffic(n: int):
    """HBM bytes per launch of the dominant kernel from the committed PMC pass (PMC_HS_FILE), scaled to n.
    Returns (bytes, provenance, VALU wave-instructions per verify, derived issue model): the figures are a committed
    measurement, not one taken in this run (PMC counters need their own rocprofv3 pass)."""
    p = os.path.join(REPO, PMC_HS_FILE)
    if not os.path.exists(p):
        return None, None, None, {}
    with open(p) as f:
        d = json.load(f)
    src = (f"{PMC_HS_FILE}: FETCH_SIZE+WRITE_SIZE of one {d['n']}-signature launch "
           f"({d.get('build', 'build of that commit')}), scaled to n; not measured in this run")
    der = dict(d.get("derived", {}))
    der["lds_bank_conflict_cycles"] = d.get("SQ_LDS_BANK_CONFLICT")
    return d["hbm_bytes_per_launch"] * n / d["n"], src, d.get("SQ_INSTS_VALU", 0) / d["n"], der


def pcie_h2d_probe(dev, mb: int = 256, reps: int = 5) -> float:
    """Host-to-device copy rate from pinned memory (GB/s, best of reps): the ceiling of the host-buffer
    path's input DMA."""
    h = torch.empty(mb << 20, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(mb << 20, dtype=torch.uint8, device=dev)
    best = 0.0
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        d.copy_(h, non_blocking=True)
        e1.record()
        e1.synchronize()
        best = max(best, (mb << 20) / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    return best


def host_api_rate(eng, batch, steps: int, device_value: float, name: str, async_steps: int = 0):
    """The drop-in path: the same batch handed over as host numpy buffers to
    cv_ed25519_verify_batch — what the JVM shim calls for SignedTransaction.checkSignaturesAreValid
    (SignedTransaction.kt:82-87) and the resolve loop (ResolveTransactionsFlow.kt:105-111).  Each step =
    one synchronous call, pipelined over sub-chunks inside the call.  value = signatures / wall time of
    the K calls.  Two forms of the same call:
      pinned    the inputs live in pinned host memory (cv_host_alloc — how the JVM shim builds its
                batches): every sub-chunk is DMAed straight out of them (no packing copy)
      pageable  ordinary numpy buffers: host threads pack each sub-chunk into pinned staging first
    `value` is the pinned form (the shim's production layout); the pageable form is reported beside it.
    async_steps (default: steps) = calls of the two async forms, timed in the loop's steady state (the first
    call's ramp outside the clock; cold_ms_per_step, with it, beside)."""
    pk, sig, arena, off, ln = batch.to_host()
    n = batch.n
    in_bytes = pk.nbytes + sig.nbytes + off.nbytes + ln.nbytes + int(ln.astype(np.int64).sum())

    def timed(a):
        for _ in range(2):                                   # warm: staging / device blocks allocated
            bm, _ = eng.verify_batch(*a, want_status=False)
        t = time.perf_counter()
        for _ in range(steps):
            bm, _ = eng.verify_batch(*a, want_status=False)
        dt = time.perf_counter() - t
        assert native.bitmap_to_bools(bm, n).all(), "host API rejected an honest signature"
        return dt

    asteps = async_steps or steps

    def timed_async(a):
        """K calls with two in flight (cv_ed25519_verify_batch_async / cv_wait): submit k+1, then wait k.
        Warm-up: five calls, so every input-ring block has carried an async-sized sub-chunk (see host_keyed_rate)."""
        pend = []
        for _ in range(5):
            pend.append(eng.verify_batch_async(*a, want_status=False))
            if len(pend) == 2:
                eng.wait(pend.pop(0))
        for tk in pend:
            eng.wait(tk)

        def loop(k):
            t = time.perf_counter()
            pend = []
            for _ in range(k):
                pend.append(eng.verify_batch_async(*a, want_status=False))
                if len(pend) == 2:
                    bm, _ = eng.wait(pend.pop(0))
            for tk in pend:
                bm, _ = eng.wait(tk)
            assert native.bitmap_to_bools(bm, n).all(), "async host API rejected an honest signature"
            return time.perf_counter() - t

        dt_cold = loop(asteps)
        # the loop's steady state (as host_c3_fused_rate's): T(K + 2 calls) - T(2 calls), the first call's ramp and
        # the last one's drain cancelling
        t2 = loop(2)
        dt = loop(asteps + 2) - t2
        return dt, dt_cold

    eng.stats("pipe", reset=True)
    dt_page = timed((pk, sig, arena, off, ln))
    pp = eng.stats("pipe")
    # the pageable call's host phases per call (its packing of the records into pinned staging is the part the pinned
    # form does not have: bound by the box's host memory bandwidth)
    page_phases = {k[:-2] + "_ms": pp[k] / max(1.0, pp["calls"]) * 1e3 for k in ("plan_s", "pack_s", "wait_s", "enqueue_s",
                                                                                 "sync_s")}
    pinned = tuple(eng.host_copy(x) for x in (pk, sig, arena, off, ln))
    eng.stats("pipe", reset=True)
    dt_pin = timed(pinned)
    ps = eng.stats("pipe")
    direct = int(ps["direct_subchunks"])
    calls = max(1.0, ps["calls"])
    # where a synchronous call's time goes: the host phases of the calls above, per call, and
    # the GPU timeline of 3 more calls (CV_OPT_TIMELINE: HIP events per sub-chunk, outside the timed loop)
    breakdown = {k[:-2] + "_ms": ps[k] / calls * 1e3 for k in ("plan_s", "pack_s", "wait_s", "enqueue_s", "sync_s")}
    breakdown["subchunks"] = ps["subchunks"] / calls
    eng.set_option("timeline", 1)
    eng.stats("timeline", reset=True)
    for _ in range(3):
        eng.verify_batch(*pinned, want_status=False)
    tl = eng.stats("timeline", reset=True)
    eng.set_option("timeline", 0)
    tc = max(1.0, tl["calls"])
    breakdown.update({k: tl[k] / tc for k in ("host_pre_ms", "ramp_ms", "dma_end_ms", "span_ms", "busy_ms", "idle_ms",
                                              "tail_ms", "result_copy_ms", "host_post_ms", "first_subchunk")})
    breakdown["timeline_calls"] = tl["calls"]
    dt_async, dt_async_cold = timed_async(pinned)
    dt_async_page, _ = timed_async((pk, sig, arena, off, ln))
    del pinned
    v, vp, vs = n * asteps / dt_async, n * steps / dt_page, n * steps / dt_pin
    va = n * asteps / dt_async_page
    return {"workload": name, "value": v, "unit": "verifies/s", "ms_per_step": dt_async / asteps * 1e3, "steps": asteps,
            "cold_ms_per_step": dt_async_cold / asteps * 1e3,
            "timing": "steady state: T(K + 2 calls) - T(2 calls), two in flight (ramp and drain cancel)",
            "sigs": n, "ratio_to_device_value": v / device_value, "device_value": device_value,
            "input_bytes_per_call": in_bytes, "input_gb_per_s": in_bytes * asteps / dt_async / 1e9,
            "path": "cv_ed25519_verify_batch_async from pinned host buffers (cv_host_alloc), two calls in flight "
                    "(a batching node submits batch k+1 before waiting for batch k); sub-chunks DMAed in place",
            "sync_pinned": {"value": vs, "ms_per_step": dt_pin / steps * 1e3, "ratio_to_device_value": vs / device_value,
                            "direct_dma_subchunks": direct, "breakdown": breakdown,
                            "path": "cv_ed25519_verify_batch (synchronous, one call at a time) from pinned buffers"},
            "async_pageable": {"value": va, "ms_per_step": dt_async_page / asteps * 1e3,
                               "ratio_to_device_value": va / device_value,
                               "path": "cv_ed25519_verify_batch_async from pageable numpy buffers, two in flight"},
            "pageable": {"value": vp, "ms_per_step": dt_page / steps * 1e3, "ratio_to_device_value": vp / device_value,
                         "input_gb_per_s": in_bytes * steps / dt_page / 1e9, "host_phases": page_phases,
                         "path": "cv_ed25519_verify_batch (synchronous) from pageable numpy buffers (host threads "
                                 "pack pinned staging per sub-chunk)"}}


def host_c3_rate(eng, local, sh, ntx: int, steps: int, device_value: float, pcie_gbs: float):
    """C3 through the drop-in boundary: per step, the Merkle ids of 1M transactions from
    host leaf buffers (cv_merkle_tx_ids_async), the verify of their 8M signatures over those ids
    (cv_ed25519_verify_batch_async: the messages are the ids the Merkle call returned), and per transaction
    id == claimed AND all signature bits (cv_tx_verdicts).  Inputs in pinned host memory (cv_host_alloc, how
    the JVM shim builds its batches).  Pipelined like a node's loop: the Merkle call of step k+1 is submitted
    behind the verify of step k, so its leaf copies overlap that verify's kernels; three id buffers rotate
    (the verify of step k-1 may still read its ids while step k+1's are written)."""
    signers = 8
    tb = workload.make_tx_batch(eng, local, ntx, signers, seed=20261016, stream=sh)
    n = ntx * signers
    pin = lambda t: eng.host_copy(t.cpu().numpy())  # noqa: E731
    arena, leaf_off = pin(tb.leaf_arena), eng.host_copy(tb.leaf_off.cpu().numpy().astype(np.uint64))
    leaf_len, tx_begin = eng.host_copy(tb.leaf_len.cpu().numpy().astype(np.uint32)), \
        eng.host_copy(tb.tx_begin.cpu().numpy().astype(np.uint32))
    claimed = tb.ids.cpu().numpy().view(np.uint64).reshape(ntx, 4)
    pk, sig = pin(tb.sigs.pk), pin(tb.sigs.sig)
    leaf_bytes = int(tb.leaf_len.to(torch.int64).sum())
    del tb
    torch.cuda.empty_cache()
    msg_off = eng.host_copy((np.arange(n, dtype=np.uint64) // signers) * 32)
    msg_len = eng.host_copy(np.full(n, 32, np.uint32))
    sig_begin = np.arange(0, n + 1, signers, dtype=np.uint32)
    bufs = [eng.host_empty(ntx * 32 + 16) for _ in range(3)]      # id arenas (the verify's messages)
    for b in bufs:
        b[-16:] = 0

    blocked = {"merkle_ms": 0.0, "verify_ms": 0.0}

    def run(k_steps):
        ok_all = True
        tm = eng.merkle_tx_ids_async(arena, leaf_off, leaf_len, tx_begin, ids=bufs[0][:ntx * 32].reshape(ntx, 32))
        tv_prev = None
        for k in range(k_steps):
            t0 = time.perf_counter()
            ids, st = eng.wait(tm)
            blocked["merkle_ms"] += (time.perf_counter() - t0) * 1e3
            tv = eng.verify_batch_async(pk, sig, bufs[k % 3], msg_off, msg_len, want_status=False)
            if k + 1 < k_steps:
                nb = bufs[(k + 1) % 3]
                tm = eng.merkle_tx_ids_async(arena, leaf_off, leaf_len, tx_begin, ids=nb[:ntx * 32].reshape(ntx, 32))
            id_ok = (ids.view(np.uint64).reshape(ntx, 4) == claimed).all(axis=1) & (st == 0)
            if tv_prev is not None:
                t0 = time.perf_counter()
                bm, _ = eng.wait(tv_prev[0])
                blocked["verify_ms"] += (time.perf_counter() - t0) * 1e3
                ok_all &= bool((native.tx_verdicts(bm, sig_begin).astype(bool) & tv_prev[1]).all())
            tv_prev = (tv, id_ok)
        bm, _ = eng.wait(tv_prev[0])
        ok_all &= bool((native.tx_verdicts(bm, sig_begin).astype(bool) & tv_prev[1]).all())
        return ok_all

    assert run(2), "host C3 step rejected an honest transaction"        # warm: staging / device blocks
    blocked.update(merkle_ms=0.0, verify_ms=0.0)
    t = time.perf_counter()
    ok = run(steps)
    dt_cold = time.perf_counter() - t
    assert ok, "host C3 step rejected an honest transaction"
    # the loop's steady state, as host_c3_fused_rate's: T(K + 2 steps) - T(2 steps), K = max(steps, 8)
    ks = max(steps, 8)
    t = time.perf_counter()
    ok = run(2)
    t2 = time.perf_counter() - t
    blocked.update(merkle_ms=0.0, verify_ms=0.0)
    t = time.perf_counter()
    ok &= run(ks + 2)
    dt = time.perf_counter() - t - t2
    assert ok, "host C3 step (steady state) rejected an honest transaction"
    in_bytes = leaf_bytes + ntx * 6 * 12 + (ntx + 1) * 4 + n * (32 + 64 + 8 + 4) + ntx * 32
    v = n * ks / dt
    return {"value": v, "unit": "verifies/s", "tx_ids_per_s": ntx * ks / dt, "ms_per_step": dt / ks * 1e3,
            "cold_ms_per_step": dt_cold / steps * 1e3,
            "timing": f"steady state: T({ks} + 2 steps) - T(2 steps) (fill and drain cancel); cold: {steps} from idle",
            "steps": ks, "ratio_to_device_value": v / device_value, "device_value": device_value,
            "input_bytes_per_step": in_bytes, "pcie_floor_ms_per_step": in_bytes / (pcie_gbs * 1e9) * 1e3,
            "host_blocked_ms_per_step": {k: v / (ks + 2) for k, v in blocked.items()},
            "path": "cv_merkle_tx_ids_async (leaves) + cv_ed25519_verify_batch_async (sigs over the returned ids) "
                    "+ cv_tx_verdicts and the id check, pinned host buffers, Merkle k+1 submitted behind verify k"}


def host_c3_fused_rate(eng, local, sh, ntx: int, steps: int, device_value: float, pcie_gbs: float, sync: bool = False):
    """C3 through the fused drop-in entry point (cv_verify_transactions_async: SignedTransaction.verifySignatures'
    id + signature checks for the batch in one call): per step the leaves, keys and signatures of 1M transactions
    from pinned host buffers; the ids stay on the device as the verify's messages; per transaction tx_ok AND id ==
    claimed.  Two calls in flight (a node's loop submits batch k+1 before it takes the verdicts of batch k).
    sync: the synchronous call, one step at a time."""
    signers = 8
    tb = workload.make_tx_batch(eng, local, ntx, signers, seed=20261016, stream=sh)
    n = ntx * signers
    pin = lambda t: eng.host_copy(t.cpu().numpy())  # noqa: E731
    arena, leaf_off = pin(tb.leaf_arena), eng.host_copy(tb.leaf_off.cpu().numpy().astype(np.uint64))
    leaf_len, tx_begin = eng.host_copy(tb.leaf_len.cpu().numpy().astype(np.uint32)), \
        eng.host_copy(tb.tx_begin.cpu().numpy().astype(np.uint32))
    claimed = tb.ids.cpu().numpy().view(np.uint64).reshape(ntx, 4)
    pk, sig = pin(tb.sigs.pk), pin(tb.sigs.sig)
    leaf_bytes = int(tb.leaf_len.to(torch.int64).sum())
    del tb
    torch.cuda.empty_cache()
    sig_begin = eng.host_copy(np.arange(0, n + 1, signers, dtype=np.uint32))
    bufs = [eng.host_empty((ntx, 32)) for _ in range(3)]
    args = (arena, leaf_off, leaf_len, tx_begin, pk, sig, sig_begin)
    blocked = {"wait_ms": 0.0}

    fails = []

    def check(ok, ids):
        idok = (ids.view(np.uint64).reshape(ntx, 4) == claimed).all(axis=1)
        good = bool(ok.all() and idok.all())
        if not good:
            bad = np.nonzero(ok == 0)[0]
            # the same host arrays through the separate verify over the claimed ids: bad inputs or a bad call?
            bm, _ = eng.verify_batch(pk, sig, np.concatenate([claimed.view(np.uint8).reshape(-1), np.zeros(16, np.uint8)]),
                                     (np.arange(n, dtype=np.uint64) // signers) * 32, np.full(n, 32, np.uint32),
                                     want_status=False)
            sep = np.nonzero(~native.bitmap_to_bools(bm, n))[0]
            fails.append({"rejected": int(bad.size), "ids_wrong": int((~idok).sum()), "first": bad[:8].tolist(),
                          "last": bad[-3:].tolist(), "separate_bad_sigs": int(sep.size), "separate_first": sep[:4].tolist(),
                          "separate_last": sep[-3:].tolist()})
        return good

    def run(k_steps):
        ok_all = True
        if sync:
            for k in range(k_steps):
                ok, ids, _, _ = eng.verify_transactions(*args, ids=bufs[k % 3], want_status=False)
                ok_all &= check(ok, ids)
            return ok_all
        prev = None
        for k in range(k_steps):
            t = eng.verify_transactions_async(*args, ids=bufs[k % 3], want_status=False)
            if prev is not None:
                t0 = time.perf_counter()
                ok, rest = eng.wait(prev)
                blocked["wait_ms"] += (time.perf_counter() - t0) * 1e3
                ok_all &= check(ok, rest[0])
            prev = t
        ok, rest = eng.wait(prev)
        return ok_all & check(ok, rest[0])

    # warm: staging, device blocks, and every one of the device's four call outputs (one per fused call, where
    # the separate form uses two per step; an output sized by smaller calls grows — a device-wide free — on
    # first use: 93 ms for the first timed fused steps after the separate ones against 87 ms once warm,
    # tools/c3_order_probe.py)
    assert run(4), f"fused C3 step rejected an honest transaction: {fails}"
    blocked["wait_ms"] = 0.0
    t = time.perf_counter()
    ok = run(steps)
    dt_cold = dt = time.perf_counter() - t
    assert ok, f"fused C3 step rejected an honest transaction: {fails}"
    if not sync:
        # the value: the loop's steady state.  The K calls above include the first call's fill and the last one's
        # drain (in the kernel trace of such a loop the GPU idles ~25 ms before and inside the first call, then not
        # at all, profiles/r06o_fused_trace_concurrency.txt); both are the same for a loop of 2 calls and one of
        # K + 2, so the difference of the two loops' times is K calls of a loop that runs continuously
        ks = max(steps, 8)
        t = time.perf_counter()
        ok = run(2)
        t2 = time.perf_counter() - t
        blocked["wait_ms"] = 0.0
        t = time.perf_counter()
        ok &= run(ks + 2)
        dt = time.perf_counter() - t - t2
        assert ok, f"fused C3 step (steady state) rejected an honest transaction: {fails}"
    else:
        ks = steps
    # where a fused call's time goes: two synchronous calls timed on the GPU (CV_OPT_TIMELINE:
    # per launch group, Merkle and verify groups apart), outside the timed loop
    eng.set_option("timeline", 1)
    eng.stats("timeline", reset=True)
    sync_ms = 0.0
    for k in range(2):
        ts = time.perf_counter()
        okk, idk, _, _ = eng.verify_transactions(*args, ids=bufs[k % 3], want_status=False)
        sync_ms += (time.perf_counter() - ts) / 2 * 1e3            # the call alone (not the check below)
        assert check(okk, idk), f"fused C3 (timed call) rejected an honest transaction: {fails}"
    tl = eng.stats("timeline", reset=True)
    eng.set_option("timeline", 0)
    tc = max(1.0, tl["calls"])
    breakdown = {k: tl[k] / tc for k in ("host_pre_ms", "ramp_ms", "merkle_dma_end_ms", "dma_end_ms", "merkle_busy_ms",
                                         "verify_busy_ms", "busy_ms", "idle_ms", "span_ms", "tail_ms",
                                         "result_copy_ms", "host_post_ms", "groups")}
    breakdown["sync_call_ms"] = sync_ms
    in_bytes = leaf_bytes + ntx * 6 * 12 + 2 * (ntx + 1) * 4 + n * (32 + 64)
    v = n * ks / dt
    return {"value": v, "unit": "verifies/s", "tx_ids_per_s": ntx * ks / dt, "ms_per_step": dt / ks * 1e3,
            "cold_ms_per_step": dt_cold / steps * 1e3,
            "timing": "synchronous calls" if sync else
                      f"steady state: T({ks} + 2 calls) - T(2 calls), two in flight (fill and drain cancel); "
                      f"cold: {steps} calls from idle",
            "steps": ks, "ratio_to_device_value": v / device_value, "device_value": device_value,
            "input_bytes_per_step": in_bytes, "pcie_floor_ms_per_step": in_bytes / (pcie_gbs * 1e9) * 1e3,
            "host_blocked_ms_per_step": {k: v / (steps if sync else ks + 2) for k, v in blocked.items()},
            "breakdown": breakdown,
            "path": ("cv_verify_transactions (synchronous)" if sync else
                     "cv_verify_transactions_async, two in flight") +
                    ": leaves + keys + signatures from pinned host buffers, ids kept on the device as the messages, "
                    "tx_ok AND id == claimed"}


def host_keyed_rate(eng, local, sh, n: int, msg_len: int, steps: int, device_value: float, pcie_gbs: float):
    """The keyed path through host buffers: C2 with a 1,024-key pool handed to
    cv_ed25519_verify_batch(_async) as plain records — the engine dedupes the keys itself (host threads,
    per device shard) and runs the keyed pipeline (key indices instead of keys staged per sub-chunk).  value =
    async form from pinned buffers, two calls in flight.  PCIe carries ~376 B per signature at C2 (300-B
    message + signature + offset/length + key index), so the host form is bounded by the H2D rate, not by the
    comb kernel's 250 M/s."""
    b = workload.make_batch(eng, local, n, msg_len, seed=4243, key_pool=1024, stream=sh)
    pk, sig, arena, off, ln = (eng.host_copy(x) for x in b.to_host())
    del b
    torch.cuda.empty_cache()

    def loop(k_steps, sync):
        pend, bm = [], None
        for _ in range(k_steps):
            if sync:
                bm, _ = eng.verify_batch(pk, sig, arena, off, ln, want_status=False)
                continue
            pend.append(eng.verify_batch_async(pk, sig, arena, off, ln, want_status=False))
            if len(pend) == 2:
                bm, _ = eng.wait(pend.pop(0))
        for tk in pend:
            bm, _ = eng.wait(tk)
        return bm

    eng.stats("route", reset=True)
    # warm until every block of the device's 16-block input ring has carried a keyed sub-chunk (4 per call): a
    # block first grows to the call's sub-chunk size at its next use, and growing frees device memory, which
    # synchronises the device — inside the timed calls that cost ~2 ms per call (9.1-9.3 vs 7.3 ms per call
    # with a 2-call warm-up after the C2 host calls had sized the blocks for their smaller sub-chunks; r05s)
    loop(6, False)
    assert eng.stats("route")["keyed_shards"] >= 1, "the host keyed path was not taken"
    eng.stats("pipe", reset=True)
    t = time.perf_counter()
    bm = loop(steps, False)
    dt = time.perf_counter() - t
    st = eng.stats("pipe", reset=True)
    assert native.bitmap_to_bools(bm, n).all(), "host keyed path rejected an honest signature"
    t = time.perf_counter()
    loop(max(2, steps // 2), True)
    dts = (time.perf_counter() - t) / max(2, steps // 2)
    per_sig = msg_len + 64 + 8 + 4 + 4
    v = n * steps / dt
    return {"value": v, "unit": "verifies/s", "ms_per_step": dt / steps * 1e3, "steps": steps,
            "ratio_to_device_value": v / device_value, "device_value": device_value,
            "sync_pinned_value": n / dts, "pcie_bound_value": pcie_gbs * 1e9 / per_sig,
            "ratio_to_pcie_bound": v / (pcie_gbs * 1e9 / per_sig),
            "host_ms_per_call": {k[:-2]: st[k] / steps * 1e3 for k in st if k.endswith("_s")},
            "path": "cv_ed25519_verify_batch_async on plain records with a 1,024-key pool from pinned buffers, two "
                    "in flight; host dedupe + keyed pipeline"}


def affinity_cores() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def host_threads() -> int:
    """Host cores the CPU baseline uses, read on the box at run time: the cores this process may run
    on (sched_getaffinity), capped by the box's declared CPU share when it sets one (OMP_NUM_THREADS:
    a shared box's affinity mask can list every core of the machine).  CV_CPU_THREADS overrides."""
    if os.environ.get("CV_CPU_THREADS"):
        return int(os.environ["CV_CPU_THREADS"])
    n = affinity_cores()
    share = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(share)) if share.isdigit() and int(share) > 0 else n


def jvm_probe() -> str:
    """the reference's own verify path (JVM + eddsa-0.1.0) is timed when a JDK and
    the jar exist on the box; report what the probe found."""
    import shutil
    import subprocess
    java = shutil.which("java")
    if not java:
        return "java absent (no JDK on the box): the C restatement of eddsa-0.1.0 stands in"
    try:
        r = subprocess.run([java, "-version"], capture_output=True, text=True, timeout=10)
        return "java present (" + (r.stderr or r.stdout).strip().splitlines()[0] + "), eddsa-0.1.0 jar absent"
    except Exception as e:  # noqa: BLE001
        return f"java probe failed: {e}"


def cpu_baseline(batch, rank_device: int, seconds: float):
    """Times the C restatement (oracle/, test infrastructure) on a bounded sample of the same batch."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import cv_oracle  # noqa: E402

    threads = host_threads()
    # 1-thread probe sizes the sample so the multi-thread leg runs ~`seconds`
    n1 = 1024
    pk, sig, arena, off, ln = batch.to_host(0, n1)
    t = time.perf_counter()
    v1, _ = cv_oracle.verify_batch(pk, sig, arena, off, ln, 1)
    rate1 = n1 / (time.perf_counter() - t)
    ns = int(min(batch.n, max(4096, rate1 * threads * seconds)))
    pk, sig, arena, off, ln = batch.to_host(0, ns)
    t = time.perf_counter()
    vm, _ = cv_oracle.verify_batch(pk, sig, arena, off, ln, threads)
    ratem = ns / (time.perf_counter() - t)
    return {"value": ratem, "unit": "verifies/s", "cores": threads, "kind": "port",
            "single_thread_value": rate1, "jvm_probe": jvm_probe(), "affinity_cores": affinity_cores(),
            "extrapolated_all_cores": rate1 * affinity_cores(),
            "extrapolated_all_cores_note": "EXTRAPOLATION, not measured: single_thread_value x affinity_cores "
                                           "(BASELINE.md: nproc threads, extrapolated per core); the box grants "
                                           "this process an OMP_NUM_THREADS share, which `value` is measured on",
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "sample": f"first {ns} signatures of the same batch ({batch.msg_len}-byte msgs) on {threads} host "
                      f"threads; single-thread rate from the first {n1}",
            "accepted_fraction": float(vm.mean())}


def notary_latency(eng, device: int, n: int, reps: int, cpu: bool, key_pool=None, adv=None):
    """C4 (BASELINE.json configs[3]): one notary batch of n signatures over 32-byte tx ids, 8 signers
    per transaction, 1/16 adversarial records cycling through the golden corpus's rejected classes.
    p50/p99 of the notary's end-to-end step through the host-buffer C-ABI (H2D + kernels + D2H + the
    per-tx AND), and where it goes: the same batch through the device API on resident inputs
    (kernels + launch overhead) and the per-kernel HIP-event phases.  With key_pool the signers come
    from that many parties (the engine's host dedupe takes the keyed path; the key pool is warm after
    the first repetition, as on a running notary)."""
    pk, sig, arena, off, ln, expect = workload.notary_batch(eng, device, n, adv, key_pool=key_pool)
    tx_begin = np.arange(0, n + 1, 8, dtype=np.uint32)
    lat = []
    for r in range(reps + 5):
        t = time.perf_counter()
        bitmap, _ = eng.verify_batch(pk, sig, arena, off, ln, want_status=False)
        txok = native.tx_verdicts(bitmap, tx_begin)
        dt = time.perf_counter() - t
        if r >= 5:
            lat.append(dt)
    assert np.array_equal(native.bitmap_to_bools(bitmap, n), expect), "notary batch verdicts wrong"
    out = {"batch": n, "p50_ms": float(np.percentile(lat, 50) * 1e3), "p99_ms": float(np.percentile(lat, 99) * 1e3),
           "reps": reps, "txs": n // 8, "tx_ok": int(txok.sum()), "signer_keys": key_pool or "distinct",
           "adversarial": "1/16, golden corpus rejected classes", "inputs": "pageable numpy buffers"}
    # the same batch from pinned host buffers (cv_host_alloc: how the JVM shim builds its batches),
    # DMAed in place without the packing copy
    pin = [eng.host_copy(x) for x in (pk, sig, arena, off, ln)]
    lat_p = []
    for r in range(reps + 5):
        t = time.perf_counter()
        bitmap, _ = eng.verify_batch(*pin, want_status=False)
        txok = native.tx_verdicts(bitmap, tx_begin)
        dt = time.perf_counter() - t
        if r >= 5:
            lat_p.append(dt)
    assert np.array_equal(native.bitmap_to_bools(bitmap, n), expect), "notary batch verdicts wrong (pinned)"
    out["pinned_inputs"] = {"p50_ms": float(np.percentile(lat_p, 50) * 1e3),
                            "p99_ms": float(np.percentile(lat_p, 99) * 1e3)}
    del pin
    if key_pool is None:
        dev = torch.device("cuda", device)
        d = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in
             (pk, sig, arena, off.view(np.int64), ln.view(np.int32))]
        bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
        s = torch.cuda.Stream(dev)
        dl = []
        for r in range(reps + 5):
            t = time.perf_counter()
            eng.verify_device(device, n, *[x.data_ptr() for x in d], bm.data_ptr(), 0, s.cuda_stream)
            s.synchronize()
            if r >= 5:
                dl.append(time.perf_counter() - t)
        ph = np.median(np.array([eng.verify_device_timed(device, n, *[x.data_ptr() for x in d], bm.data_ptr(),
                                                         s.cuda_stream) for _ in range(10)]), axis=0)
        dev_p50 = float(np.percentile(dl, 50) * 1e3)
        names = (("scalars_and_point_pairs", "bitmap_clear", "hs_straus_tri" if n <= 4096 else "hs_straus_quad")
                 if n <= 32768 else ("scalars", "points", "hs_straus"))
        out["breakdown_p50_ms"] = {"host_api_total": out["p50_ms"], "device_api_total": dev_p50,
                                   "transfers_and_host": out["p50_ms"] - dev_p50,
                                   "kernels": {k: float(v) for k, v in zip(names, ph)},
                                   "launch_and_sync": dev_p50 - float(ph.sum())}
    if cpu:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import cv_oracle  # noqa: E402
        threads = host_threads()
        cl = []
        for r in range(3):
            t = time.perf_counter()
            v, _ = cv_oracle.verify_batch(pk, sig, arena, off, ln, threads)
            cl.append(time.perf_counter() - t)
        assert np.array_equal(v.astype(bool), expect)
        out["cpu_p50_ms"] = float(np.median(cl) * 1e3)
        out["cpu_threads"] = threads
        t = time.perf_counter()
        cv_oracle.verify_batch(pk[:512], sig[:512], arena, off[:512], ln[:512], 1)
        per_sig = (time.perf_counter() - t) / 512
        out["cpu_extrapolated_all_cores_ms"] = per_sig * n / affinity_cores() * 1e3
        out["cpu_extrapolated_note"] = (f"EXTRAPOLATION: 1-thread time per signature x {n} / {affinity_cores()} "
                                        "affinity cores (perfect scaling assumed)")
    return out


def resolve_chain_latency(eng, device: int, reps: int, cpu: bool, ntx: int = 5000, signers: int = 2):
    """ResolveTransactionsFlow (core/src/main/kotlin/net/corda/flows/
    ResolveTransactionsFlow.kt:105-111,119) checks a whole dependency chain; the reference loops
    `stx.verifySignatures()` per transaction (id recompute + sequential EdDSAEngine verifies).  Here
    the chain is ONE Merkle call (every WireTransaction.id) + ONE verify call (every signature over its
    claimed id) + the per-tx AND with the id check, host buffers in and out; p50/p99 over reps.
    Synthetic chain: C3-shaped leaves (6 per tx), `signers` signatures per tx, one in 16 txs with a
    mutated signature and one in 64 with a mutated leaf (id mismatch)."""
    tb = workload.make_tx_batch(eng, device, ntx, signers=signers, seed=5000)
    arena = tb.leaf_arena.cpu().numpy().copy()
    leaf_off = tb.leaf_off.cpu().numpy().astype(np.uint64)
    leaf_len = tb.leaf_len.cpu().numpy().astype(np.uint32)
    tx_begin = tb.tx_begin.cpu().numpy().astype(np.uint32)
    claimed = tb.ids.cpu().numpy()
    pk, sig, _, _, _ = tb.sigs.to_host()
    sig = sig.copy()
    bad_sig_tx = np.arange(0, ntx, 16)
    sig[bad_sig_tx * signers, 40] ^= 1                         # S bit flip: reject
    bad_leaf_tx = np.arange(3, ntx, 64)
    arena[leaf_off[tx_begin[bad_leaf_tx]].astype(np.int64)] ^= 0x5a      # first leaf byte: id mismatch
    msg_arena = np.concatenate([claimed.reshape(-1), np.zeros(16, np.uint8)])
    msg_off = (np.arange(ntx * signers, dtype=np.uint64) // signers) * 32
    msg_len = np.full(ntx * signers, 32, np.uint32)
    sig_tx_begin = np.arange(0, ntx * signers + 1, signers, dtype=np.uint32)
    expect = np.ones(ntx, bool)
    expect[bad_sig_tx] = False
    expect[bad_leaf_tx] = False

    def chain_gpu():
        ids, st = eng.merkle_tx_ids(arena, leaf_off, leaf_len, tx_begin)
        bitmap, _ = eng.verify_batch(pk, sig, msg_arena, msg_off, msg_len, want_status=False)
        return native.tx_verdicts(bitmap, sig_tx_begin).astype(bool) & (ids == claimed).all(axis=1) & (st == 0)

    lat = []
    for r in range(reps + 5):
        t = time.perf_counter()
        ok = chain_gpu()
        dt = time.perf_counter() - t
        if r >= 5:
            lat.append(dt)
    assert np.array_equal(ok, expect), "resolve chain verdicts wrong"
    out = {"txs": ntx, "signers_per_tx": signers, "sigs": ntx * signers, "leaves_per_tx": 6,
           "p50_ms": float(np.percentile(lat, 50) * 1e3), "p99_ms": float(np.percentile(lat, 99) * 1e3),
           "reps": reps, "tx_ok": int(ok.sum())}
    if cpu:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import cv_oracle  # noqa: E402
        threads = host_threads()
        cl = []
        for r in range(3):
            t = time.perf_counter()
            ids_c = cv_oracle.merkle_tx_ids(arena, leaf_off, leaf_len, tx_begin)
            v, _ = cv_oracle.verify_batch(pk, sig, msg_arena, msg_off, msg_len, threads)
            cl.append(time.perf_counter() - t)
        ids_c = ids_c[0] if isinstance(ids_c, tuple) else ids_c
        okc = (v.astype(bool).reshape(ntx, signers).all(axis=1) & (ids_c == claimed).all(axis=1))
        assert np.array_equal(okc, expect), "CPU restatement disagrees on the resolve chain"
        out["cpu_p50_ms"] = float(np.median(cl) * 1e3)
        out["cpu_threads"] = threads
    return out


def keyed_rate(eng, device: int, n: int, msg_len: int, steps: int, sh: int, pool: int = 1024):
    """Keyed path (per-key comb tables) on the same C2 shape with a `pool`-key
    pool: each step resolves the keys against the device key pool and verifies all n signatures."""
    b = workload.make_batch(eng, device, n, msg_len, seed=4242, key_pool=pool, stream=sh)
    bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=torch.device("cuda", device))
    args = (device, n, b.nkeys, b.pk.data_ptr(), b.key_index.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(),
            b.off.data_ptr(), b.len.data_ptr(), bm.data_ptr(), 0, sh)
    cold = eng.verify_device_keyed(*args, timed=True)            # first call computes the key tables
    ph = []
    t = time.perf_counter()
    for _ in range(steps):
        ph.append(eng.verify_device_keyed(*args, timed=True))
    dt = time.perf_counter() - t
    assert bool((bm == -1).all()) or n % 64, "keyed path rejected an honest signature"
    m = np.mean(np.array(ph), axis=0)
    return {"workload": f"C2 shape, {pool}-key pool, keyed device path", "value": n * steps / dt,
            "unit": "verifies/s", "ms_per_step": dt / steps * 1e3,
            "phase_ms": {"key_tables": float(m[0]), "hash": float(m[1]), "comb": float(m[2]), "finish": float(m[3])},
            "cold_key_tables_ms": float(cold[0]), "comb_work_per_unit": "224 S + 535 M per verify (56 doublings, 32 radix-256 key-row + 16 radix-2^16 basepoint madds)"}


def straus_roofline(eng, local: int, n: int, straus_ms: float, kern_ms: float, mad_rate: float):
    """Roofline fields of the dominant kernel from its HIP-event time (half-size schedule counts)."""
    achieved = n * W_MAC_HS_STRAUS / (straus_ms * 1e-3)
    group = n * W_MAC_HS_GROUP / (kern_ms * 1e-3)
    return {"bound": "valu", "achieved": achieved / 1e12, "peak": mad_rate / 1e12, "unit": "Tmac/s",
            "frac": achieved / mad_rate, "kernel": "cv_hs_straus_kernel", "kernel_ms": straus_ms,
            "group": {"kernel_ms": kern_ms, "achieved": group / 1e12, "frac": group / mad_rate}}


def run_c3(eng, local, rank, world, sh, dev, ntx: int, steps: int, warmup: int):
    """C3 step (BASELINE.json configs[2]): recompute every tx id (leaf SHA-256 + Merkle tree), verify
    all signatures over the claimed ids, then per transaction: id matches AND all its signature bits
    set.  Returns the timing dict (rank 0's view after the max over ranks)."""
    t0 = time.perf_counter()
    tb = workload.make_tx_batch(eng, local, ntx, 8, seed=20261015 + 7919 * rank, stream=sh)
    log(f"[rank {rank}] generated {ntx} txs / {tb.sigs.n} signatures on GPU in {time.perf_counter() - t0:.2f}s")
    n = tb.sigs.n
    nleaves = int(tb.leaf_len.numel())
    ids = torch.empty_like(tb.ids)
    ws = torch.empty(nleaves * 32, dtype=torch.uint8, device=dev)
    bitmap = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    sig_args = (tb.sigs.pk.data_ptr(), tb.sigs.sig.data_ptr(), tb.sigs.arena.data_ptr(), tb.sigs.off.data_ptr(),
                tb.sigs.len.data_ptr(), bitmap.data_ptr())

    def merkle():
        eng.merkle_device(local, ntx, nleaves, tb.leaf_arena.data_ptr(), tb.leaf_off.data_ptr(),
                          tb.leaf_len.data_ptr(), tb.tx_begin.data_ptr(), ws.data_ptr(), ids.data_ptr(), 0, sh)

    def step():
        merkle()
        eng.verify_device(local, n, *sig_args[:5], sig_args[5], 0, sh)
        return D.tx_verdicts_torch(bitmap, tb.sig_tx_begin) & (ids == tb.ids).all(dim=1)

    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        ok = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    assert bool(ok.all()), "an honest transaction was rejected"
    # phases: the Merkle call (torch events on the same stream) and the verify kernels (HIP events)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    mk = []
    for _ in range(max(2, steps)):
        e0.record()
        merkle()
        e1.record()
        e1.synchronize()
        mk.append(e0.elapsed_time(e1))
    ph = np.mean(np.array([eng.verify_device_timed(local, n, *sig_args, sh) for _ in range(max(2, steps))]), axis=0)
    merkle_ms = float(np.mean(mk))
    comp = merkle_compressions(tb.leaf_len, tb.tx_begin)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt[0])
    tb = None
    return {"n": n, "ntx": ntx, "elapsed": elapsed, "merkle_ms": merkle_ms, "phases": ph,
            "leaves": nleaves, "compressions": comp}


# SHA-256 instruction floor per compression on gfx950 (VALU lane-instructions, every one a VOP3 at the
# v_mad_u64_u32 issue rate): per round Sigma1 and Sigma0 as 3 v_alignbit + 1 v_bitop3 xor3 each, Ch and
# Maj one v_bitop3 each, T1 two v_add3, a' one v_add3, e' one v_add = 14; per schedule word (48)
# sigma0 / sigma1 as 2 v_alignbit + 1 shift + 1 v_bitop3 each, W two adds = 10; 16 v_perm byte swaps
# of the message words; 8 state adds:  64*14 + 48*10 + 16 + 8 = 1,400.
SHA256_FLOOR_INSTR = 64 * 14 + 48 * 10 + 16 + 8
# PMC of the leaf kernel (tools/merkle_probe.py under rocprofv3 --pmc; file below): VALU
# wave-instructions and the compressions of that run, for the instruction-efficiency figure
MERKLE_PMC_FILE = "profiles/r03_pmc_merkle.json"


def merkle_compressions(leaf_len: torch.Tensor, tx_begin: torch.Tensor) -> dict:
    """SURVEY.md §8(d) Merkle unit, one SHA-256 compression: per leaf ceil((len + 9) / 64) blocks, per
    internal node (odd levels duplicate the last node: cv_merkle_root_inplace) sha256(l || r) = 2
    blocks.  Counted from the actual leaf lengths of the batch."""
    leaf = int(((leaf_len.to(torch.int64) + 9 + 63) // 64).sum())
    cnt = (tx_begin[1:] - tx_begin[:-1]).to(torch.int64)
    nodes = torch.zeros_like(cnt)
    while bool((cnt > 1).any()):
        m = torch.where(cnt > 1, (cnt + 1) // 2, torch.zeros_like(cnt))
        nodes += m
        cnt = torch.where(cnt > 1, m, cnt)
    internal = int(nodes.sum())
    return {"leaf": leaf, "internal_nodes": internal, "total": leaf + 2 * internal}


def merkle_roofline(comp: dict, ntx: int, merkle_ms: float, mad_rate: float) -> dict:
    """VALU-issue roofline of the Merkle tx-id recompute (cv_leaf_hash_kernel + cv_merkle_tree_kernel):
    compressions/s against the chip's VOP3 issue rate (measured v_mad_u64_u32 rate, lane-instr/s)
    over the 1,400-instruction SHA-256 floor."""
    rate = comp["total"] / (merkle_ms * 1e-3)
    peak = mad_rate / SHA256_FLOOR_INSTR
    out = {"bound": "valu", "unit": "compressions/s", "achieved": rate, "peak": peak, "frac": rate / peak,
           "compressions_per_tx": comp["total"] / ntx, "leaf_compressions": comp["leaf"],
           "internal_nodes": comp["internal_nodes"], "kernel_ms": merkle_ms,
           "floor_instr_per_compression": SHA256_FLOOR_INSTR,
           "peak_note": "measured v_mad_u64_u32 lane rate / SHA-256 VOP3 instruction floor (bench.py)"}
    try:
        with open(os.path.join(REPO, MERKLE_PMC_FILE)) as f:
            pmc = json.load(f)
        out["pmc"] = {"source": MERKLE_PMC_FILE, **{k: pmc[k] for k in
                      ("valu_lane_slots_per_compression", "valu_active_lane_instr_per_compression",
                       "lane_utilisation", "instr_efficiency_vs_floor") if k in pmc}}
    except (OSError, ValueError, KeyError):
        pass
    return out


def c3_line(eng, local, rank, world, sh, dev, ntx, steps, warmup, mad_rate):
    r = run_c3(eng, local, rank, world, sh, dev, ntx, steps, warmup)
    ph = r["phases"]
    return {"workload": CONFIG_NAME["c3"], "value": world * r["n"] * steps / r["elapsed"], "unit": "verifies/s",
            "tx_ids_per_s": world * ntx * steps / r["elapsed"], "ms_per_step": r["elapsed"] / steps * 1e3,
            "steps": steps, "txs_per_gpu": ntx, "sigs_per_gpu": r["n"], "leaves_per_gpu": r["leaves"],
            "phase_ms": {"merkle": r["merkle_ms"], "scalars": float(ph[0]), "points": float(ph[1]),
                         "hs_straus": float(ph[2])},
            "roofline": straus_roofline(eng, local, r["n"], float(ph[2]), float(ph.sum()), mad_rate),
            "merkle_roofline": merkle_roofline(r["compressions"], ntx, r["merkle_ms"], mad_rate)}


def c5_line(eng, local, rank, sh, dev, n, steps, mad_rate, host_api: bool = True):
    """C5 (BASELINE.json configs[4]) single-GPU shard: n single-signer signatures over 32-byte tx ids,
    verified in the engine's 2M-signature workspace chunks."""
    t0 = time.perf_counter()
    b = workload.make_batch(eng, local, n, 32, seed=5 + 7919 * rank, stream=sh)
    log(f"[rank {rank}] generated {n} C5 signatures in {time.perf_counter() - t0:.2f}s")
    bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    a = (b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(), b.len.data_ptr(), bm.data_ptr())
    eng.verify_device(local, n, *a, 0, sh)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.verify_device(local, n, *a, 0, sh)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    assert bool((bm == -1).all()) or n % 64, "C5: verify rejected an honest signature"
    ph = np.mean(np.array([eng.verify_device_timed(local, n, *a, sh) for _ in range(2)]), axis=0)
    host = host_api_rate(eng, b, 3, n * steps / el, CONFIG_NAME["c5"] + " (host buffers)",
                         async_steps=8) if host_api else None
    del b
    return {"workload": CONFIG_NAME["c5"], "value": n * steps / el, "unit": "verifies/s", "host_api": host,
            "ms_per_step": el / steps * 1e3, "steps": steps, "sigs_per_gpu": n,
            "tx_ids_per_s": n * steps / el, "tx_ids_note": "single-signer: one tx id per signature",
            "phase_ms": {"scalars": float(ph[0]), "points": float(ph[1]), "hs_straus": float(ph[2])},
            "roofline": straus_roofline(eng, local, n, float(ph[2]), float(ph.sum()), mad_rate)}


def timed_steps(step, steps: int, world: int, sync):
    """The contract's timed region: barrier + sync, K steps, sync + barrier; returns (seconds, last step's
    result).  sync() waits for this rank's device (a no-op in the CPU plumbing mode)."""
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    out = None
    for k in range(steps):
        out = step(k)
    sync()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0, out


def written_all_ones(bitmaps, n: int) -> bool:
    """Every verdict word of every bitmap all ones (bits past n clear).  The bitmaps are zeroed before each
    timed region, so this proves the timed launches wrote every word (an honest batch) — a skipped or no-op
    launch leaves zeros."""
    words = (n + 63) // 64
    full = torch.full((words,), -1, dtype=torch.int64, device=bitmaps[0].device)
    if n % 64:
        full[-1] = (1 << (n % 64)) - 1
    return all(torch.equal(bm, full) for bm in bitmaps)


def max_over_ranks(vals, device) -> list:
    """Element-wise max of per-rank floats (the slowest rank's timed region is the job's)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [float(v) for v in vals]
    tt = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=device)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return [float(x) for x in tt.cpu()]


def c5_multi_line(eng, local, rank, world, sh, dev, n: int, steps: int) -> dict:
    """C5 over the ranks (BASELINE.json configs[4]): each rank verifies its own n signatures over 32-byte ids
    (device-resident) and every timed step ends with the RCCL all-gather of the verdict bitmaps into the
    replicated global bitmap the commit step reads; weak scaling, value = world * n * steps / max time."""
    assert n % 64 == 0, "per-rank shard must be whole bitmap words"
    b = workload.make_batch(eng, local, n, 32, seed=5 + 7919 * rank, stream=sh)
    bm = torch.zeros(n // 64, dtype=torch.int64, device=dev)
    a = (b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(), b.len.data_ptr(), bm.data_ptr())

    def step(k):
        eng.verify_device(local, n, *a, 0, sh)
        return D.gather_bitmap(bm, world * n)             # on the current (= sh) stream, behind the verify

    step(0)                                               # warm: workspace chunks, RCCL channels
    torch.cuda.synchronize(dev)
    bm.zero_()                                            # so the all-ones check below proves the TIMED steps wrote it
    el, gathered = timed_steps(step, steps, world, lambda: torch.cuda.synchronize(dev))
    ok = bool((gathered == -1).all()) and torch.equal(gathered.view(world, -1)[rank], bm)
    (el, bad) = max_over_ranks([el, 0.0 if ok else 1.0], dev)
    assert bad == 0.0, "C5 multi-GPU: a gathered verdict bitmap is not all-ones"
    del b
    torch.cuda.empty_cache()
    return {"workload": f"C5: {n} sigs per GPU x {world} GPUs = {world * n} over 32-byte tx ids, RCCL all-gather "
                        "of the verdict bitmaps in every step",
            "value": world * n * steps / el, "unit": "verifies/s", "ms_per_step": el / steps * 1e3, "steps": steps,
            "sigs_total": world * n, "gathered_bitmap_words": world * n // 64, "gathered_all_ones": True}


def c_abi_multi_line(eng, local, sh, dev, n_per_dev: int, steps: int) -> dict:
    """The JVM node's multi-GPU form: ONE process, one context over every visible GPU
    (cv_open(0)), the whole C5 batch of n_per_dev x devices signatures from pinned host buffers through the
    synchronous cv_ed25519_verify_batch — the engine cuts it into 64-aligned ranges over the devices, each
    shard's bitmap words copied straight into the caller's bitmap, no collective (cv_api.cpp dispatch) — and
    the same call with two in flight (the async form a batching node uses).  Baseline beside it: the first
    n_per_dev records through a one-device context (this rank's GPU), so value / (devices x single) is the
    C-ABI path's scaling efficiency."""
    multi = native.Engine(0)
    ndev = multi.device_count
    N = ndev * n_per_dev
    pk, sig = multi.host_empty((N, 32)), multi.host_empty((N, 64))
    arena = multi.host_empty(N * 32 + 16)
    arena[-16:] = 0
    for j in range(ndev):                                 # generated on this rank's GPU, DMAed into pinned memory
        b = workload.make_batch(eng, local, n_per_dev, 32, seed=900 + j, stream=sh)
        lo, hi = j * n_per_dev, (j + 1) * n_per_dev
        torch.from_numpy(pk[lo:hi]).copy_(b.pk)
        torch.from_numpy(sig[lo:hi]).copy_(b.sig)
        torch.from_numpy(arena[lo * 32:hi * 32]).copy_(b.arena[:n_per_dev * 32])
        del b
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    off = multi.host_copy(np.arange(N, dtype=np.uint64) * 32)
    ln = multi.host_copy(np.full(N, 32, np.uint32))
    full = native.bitmap_to_bools

    def sync_calls(e, n, k):
        bm = None
        t = time.perf_counter()
        for _ in range(k):
            bm, _ = e.verify_batch(pk[:n], sig[:n], arena, off[:n], ln[:n], want_status=False)
        dt = time.perf_counter() - t
        assert full(bm, n).all(), "C-ABI multi-device call rejected an honest signature"
        return dt

    def async_calls(e, n, k):
        pend, bm = [], None
        t = time.perf_counter()
        for _ in range(k):
            pend.append(e.verify_batch_async(pk[:n], sig[:n], arena, off[:n], ln[:n], want_status=False))
            if len(pend) == 2:
                bm, _ = e.wait(pend.pop(0))
        for tk in pend:
            bm, _ = e.wait(tk)
        dt = time.perf_counter() - t
        assert full(bm, n).all(), "C-ABI multi-device async call rejected an honest signature"
        return dt

    multi.stats("route", reset=True)
    sync_calls(multi, N, 1)                               # warm: every device's workspace and input ring
    route = multi.stats("route")
    dt = sync_calls(multi, N, steps)
    dta = async_calls(multi, N, steps + 1)
    sync_calls(eng, n_per_dev, 1)
    dt1 = sync_calls(eng, n_per_dev, steps)
    dta1 = async_calls(eng, n_per_dev, steps + 1)
    multi.close()
    del pk, sig, arena, off, ln
    v, va = N * steps / dt, N * (steps + 1) / dta
    v1, va1 = n_per_dev * steps / dt1, n_per_dev * (steps + 1) / dta1
    return {"workload": f"C5 through the C-ABI: {N} sigs ({n_per_dev} x {ndev} devices) over 32-byte ids, pinned "
                        "host buffers, one process, cv_open(0)",
            "devices": ndev, "value": v, "unit": "verifies/s", "ms_per_call": dt / steps * 1e3, "steps": steps,
            "async_value": va, "async_ms_per_call": dta / (steps + 1) * 1e3,
            "single_device_value": v1, "single_device_async_value": va1,
            "efficiency_vs_devices_x_single": v / (ndev * v1), "async_efficiency_vs_devices_x_single": va / (ndev * va1),
            "shards_per_call": route["shards"], "path": "cv_ed25519_verify_batch (sync) and _async two in flight, "
                                                        "engine-routed over the context's devices"}


def plumbing_main(args, world: int, rank: int):
    """CPU check of the N > 1 machinery (tests/test_bench_launch.py): the self-launch, the gloo process group,
    the timed region's barriers, the bitmap all-gather and the max over ranks, with NO verification — each
    rank's "verify" fills its shard bitmap with ones.  The printed line says so and is never a measurement."""
    dist.init_process_group("gloo")
    n = args.n or 64 * 1000
    assert n % 64 == 0
    bm = torch.zeros(n // 64, dtype=torch.int64)

    def step(k):
        if not args.plumbing_noop:
            bm.fill_(-1)                                  # stand-in for this rank's verify kernel
        return D.gather_bitmap(bm, world * n)

    step(0)
    bm.zero_()                                            # as the GPU form: the timed steps must write every word
    el, gathered = timed_steps(step, args.steps, world, lambda: None)
    ok = written_all_ones([bm], n) and bool((gathered == -1).all())
    (el, bad) = max_over_ranks([el, 0.0 if ok else 1.0], "cpu")
    assert bad == 0.0, "plumbing: a verdict bitmap was not written by the timed steps"

    if rank == 0:
        print(json.dumps({"metric": "PLUMBING CHECK (launcher + gloo all-gather + timing; no verification)",
                          "value": None, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": el / args.steps * 1e3, "gathered_words": int(gathered.numel()),
                          "gathered_all_ones": bool((gathered == -1).all()),
                          "rank_env": {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE",
                                                                       "MASTER_ADDR")}}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(MSG_BYTES))
    ap.add_argument("--n", type=int, default=0, help="signatures per GPU (default 1M for c2, 8M for c5)")
    ap.add_argument("--key-pool", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-notary", action="store_true")
    ap.add_argument("--no-keyed", action="store_true")
    ap.add_argument("--no-sub", action="store_true", help="skip the C3 / C5-shard sub-lines")
    ap.add_argument("--no-host", action="store_true", help="skip the host-buffer (drop-in) sub-lines")
    ap.add_argument("--detail", default="", help="where the full measurement dict goes (default "
                                                     "gpurun_out/bench_detail.json)")
    ap.add_argument("--streams", type=int, default=2,
                    help="device streams the K timed steps are dealt over (each its own workspace slot); the "
                         "line also reports the other form (1 <-> 2 streams) beside it")
    ap.add_argument("--c5-per-gpu", type=int, default=8_000_000,
                    help="N > 1: signatures per GPU of the c5 and c_abi_multi sub-lines (BASELINE configs[4]: 8M)")
    ap.add_argument("--c-abi-multi", action="store_true",
                    help="also run the c_abi_multi sub-line at N = 1 (it always runs at N > 1)")
    ap.add_argument("--plumbing-noop", action="store_true",
                    help="test hook of --plumbing: the stand-in verify writes nothing, so the timed steps' all-ones "
                         "check must fail (tests/test_bench_launch.py)")
    ap.add_argument("--plumbing", action="store_true",
                    help="CPU check of the N > 1 launcher / gloo all-gather / timing, no GPU and NO verification "
                         "(tests/test_bench_launch.py); its line is never a measurement")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start the ranks ourselves (no GPU call has been made in this process)
        from corda_amd import launch
        sys.exit(launch.spawn(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                              require_gpus=not args.plumbing))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but the launcher's WORLD_SIZE is {world}; refusing to report a line "
            f"for a GPU count other than the one asked for")
        sys.exit(2)
    if args.plumbing:
        plumbing_main(args, world, rank)
        return
    if world > 1 and torch.cuda.device_count() < world:
        log(f"bench.py: {world} ranks but only {torch.cuda.device_count()} GPU(s) visible")
        sys.exit(2)
    cpu_group = None
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        # ranks that wait for rank 0's one-rank legs (c_abi_multi, notary, ...) block on the CPU, not in an
        # RCCL kernel on their GPU (the c_abi_multi leg uses every GPU of the node)
        cpu_group = dist.new_group(backend="gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    n = args.n or (1_000_000 if args.config == "c2" else 8_000_000)
    msg_len = MSG_BYTES[args.config]

    eng = native.Engine(1 << local)
    # a dedicated (non-null) stream: the verify kernels, the HIP events that time them and the RCCL
    # all-gather are all ordered on it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    assert sh != 0
    if args.config == "c3":
        ntx = args.n or 1_000_000
        r = run_c3(eng, local, rank, world, sh, dev, ntx, args.steps, args.warmup)
        if rank == 0:
            mad_rate, _ = eng.calibrate(local)
            ph = r["phases"]
            print(json.dumps({
                "metric": "Ed25519 verifies/sec (node)", "value": world * r["n"] * args.steps / r["elapsed"],
                "unit": "verifies/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": r["elapsed"] / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": "uint32/uint64 (GF(2^255-19) radix 2^25.5 limbs), SHA-256",
                "data": "synthetic (leaf blobs, keys, signatures generated on-GPU from seeded RNG)",
                "config": {"workload": CONFIG_NAME["c3"], "txs_per_gpu": ntx, "signers_per_tx": 8,
                           "leaves_per_tx": 6, "sigs_per_gpu": r["n"], "parallelism": f"shard-by-transaction x{world}"},
                "tx_ids_per_s": world * ntx * args.steps / r["elapsed"],
                "phase_ms": {"merkle": r["merkle_ms"], "scalars": float(ph[0]), "points": float(ph[1]),
                             "hs_straus": float(ph[2])},
                "roofline": straus_roofline(eng, local, r["n"], float(ph[2]), float(ph.sum()), mad_rate),
                "merkle_roofline": merkle_roofline(r["compressions"], ntx, r["merkle_ms"], mad_rate)}), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        eng.close()
        return
    t0 = time.perf_counter()
    batch = workload.make_batch(eng, local, n, msg_len, seed=20261015 + 7919 * rank,
                                key_pool=args.key_pool or None, stream=sh)
    log(f"[rank {rank}] generated {n} signatures on GPU in {time.perf_counter() - t0:.2f}s")
    words = (n + 63) // 64
    if world > 1:
        assert n % 64 == 0, "per-GPU shard must be whole bitmap words"
    # Steps are independent batches (a node's concurrent verify calls): step k goes on streams[k % S],
    # each stream with its own bitmap; the engine gives each stream its own workspace slot, so step k+1's
    # prep runs while step k's last Straus round drains.  Every step is a full verify of all n signatures.
    # (round 3: with HIP's default four hardware queues one vs two streams flipped from box to box with the
    # queues the streams landed on, profiles/r03n_stream_ab.log, r03o_stream_ab_q4.log; round 4: two streams
    # at four vs eight queues within 2 %, profiles/r04_queue_ab.log, so the bench keeps HIP's default and
    # records it.  The other form is reported beside the value.)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(max(2, args.streams) - 1)]
    nstreams = max(1, args.streams)
    bitmaps = [torch.zeros(words, dtype=torch.int64, device=dev) for _ in streams]
    bitmap = bitmaps[0]

    def step(k, ns=len(streams)):
        st, bm = streams[k % ns], bitmaps[k % ns]
        eng.verify_device(local, n, batch.pk.data_ptr(), batch.sig.data_ptr(), batch.arena.data_ptr(),
                          batch.off.data_ptr(), batch.len.data_ptr(), bm.data_ptr(), 0, st.cuda_stream)
        if world > 1:
            with torch.cuda.stream(st):                       # the gather waits for this step's verify only
                return D.gather_bitmap(bm, world * n)
        return bm

    def timed(ns):
        # N>1: every step ends with the RCCL all-gather into the commit step
        return timed_steps(lambda k: step(k, ns), args.steps, world, lambda: torch.cuda.synchronize(dev))

    def zero_bitmaps():
        torch.cuda.synchronize(dev)
        for bm in bitmaps:
            bm.zero_()
        torch.cuda.synchronize(dev)

    for k in range(args.warmup):
        step(k)
    # the bitmaps are zeroed outside every timed region, so each all-ones check below proves that the timed
    # launches themselves wrote every verdict word
    zero_bitmaps()

    # Timed region: K production verify calls dealt over the streams (the engine's own launch plan,
    # incl. the drain-overlap sub-chunks it picks for near-empty last rounds), one sync at the end.
    elapsed, gathered = timed(nstreams)
    assert written_all_ones(bitmaps[:min(nstreams, args.steps)], n), \
        "timed verify calls did not write an all-ones verdict bitmap (honest batch)"
    prod_bitmap = bitmap.clone()
    zero_bitmaps()
    other_streams = 2 if nstreams == 1 else 1
    other_elapsed, _ = timed(other_streams)
    assert written_all_ones(bitmaps[:min(other_streams, args.steps)], n), \
        "timed verify calls (other stream form) did not write an all-ones verdict bitmap"
    zero_bitmaps()
    # Roofline: K more calls of the same batch as whole-chunk launches, timed kernel by kernel with HIP
    # events recorded on `stream` between the launches (cv_ed25519_verify_device_timed waits for the last).
    phases = []
    for k in range(args.steps):
        phases.append(eng.verify_device_timed(local, n, batch.pk.data_ptr(), batch.sig.data_ptr(),
                                              batch.arena.data_ptr(), batch.off.data_ptr(), batch.len.data_ptr(),
                                              bitmap.data_ptr(), sh))
    torch.cuda.synchronize(dev)
    assert torch.equal(prod_bitmap, bitmap), "production and timed launch plans disagree"
    # correctness of the timed configuration: every generated signature is honest
    assert written_all_ones([bitmap], n), "verify rejected an honest signature"
    ph = np.mean(np.array(phases), axis=0)
    kern_ms, straus_ms = float(ph.sum()), float(ph[2])
    # the dominant kernel over whole rounds of resident waves (3 per SIMD x 4 SIMDs per CU x 64 lanes) of the same
    # batch: its steady-state rate, without the 1M launch's partly filled last round (roofline.frac_whole_rounds)
    per_round = torch.cuda.get_device_properties(dev).multi_processor_count * 4 * 3 * 64
    n_whole = (n // per_round) * per_round
    whole_rounds = {}
    if n_whole and n_whole != n:
        # median of K launches (the mean of the K 1M launches is the headline: it must match rocprof's mean; this
        # side figure takes the median, as tools/round_tail_probe.py, so one slow launch does not decide it)
        wph = [eng.verify_device_timed(local, n_whole, batch.pk.data_ptr(), batch.sig.data_ptr(), batch.arena.data_ptr(),
                                       batch.off.data_ptr(), batch.len.data_ptr(), bitmap.data_ptr(), sh)
               for _ in range(max(5, args.steps))]
        whole_rounds = {"n": n_whole, "rounds": n_whole // per_round,
                        "hs_straus_ms": float(np.median([w[2] for w in wph])),
                        "hs_straus_ms_all": [float(w[2]) for w in wph]}
        torch.cuda.synchronize(dev)
        bitmap.copy_(prod_bitmap)
    multi = {}
    if world > 1:
        elapsed, kern_ms, straus_ms, other_elapsed = max_over_ranks([elapsed, kern_ms, straus_ms, other_elapsed], dev)
        assert torch.equal(gathered.view(world, words)[rank], bitmap)
        assert bool((gathered == -1).all()), "a rank rejected an honest signature"
    value = world * n * args.steps / elapsed
    if world > 1 and not args.no_sub:
        del batch
        torch.cuda.empty_cache()
        multi["c5"] = c5_multi_line(eng, local, rank, world, sh, dev, args.c5_per_gpu, 3)
    if (world > 1 or args.c_abi_multi) and not args.no_host:
        if rank == 0:
            multi["c_abi_multi"] = c_abi_multi_line(eng, local, sh, dev, args.c5_per_gpu, 3)
        if world > 1:
            dist.barrier(group=cpu_group)

    if rank == 0:
        mad_rate, femul_rate = eng.calibrate(local)
        achieved = n * W_MAC_HS_STRAUS / (straus_ms * 1e-3)
        if whole_rounds:
            whole_rounds["frac"] = whole_rounds["n"] * W_MAC_HS_STRAUS / (whole_rounds["hs_straus_ms"] * 1e-3) / mad_rate
        group = n * W_MAC_HS_GROUP / (kern_ms * 1e-3)
        traffic, traffic_src, valu_per_verify, pmc = pmc_traffic(n)
        cyc = eng.calibrate_cycles(local)
        other_key = f"{'two' if other_streams == 2 else 'single'}_stream"
        # everything measured, in full: written to the detail file; the printed line is a digest of it
        D_ = {"roofline": {
            "bound": "valu", "achieved": achieved / 1e12, "peak": mad_rate / 1e12, "unit": "Tmac/s",
            "frac": achieved / mad_rate, "traffic": traffic, "traffic_source": traffic_src,
            "pmc_valu_wave_instr_per_verify": valu_per_verify, "pmc_issue_model": pmc,
            "whole_rounds": whole_rounds,
            "kernel": "cv_hs_straus_kernel", "kernel_ms": straus_ms,
            "work_per_unit": (f"{W_MAC_HS_STRAUS} 32x32->64 MAC per verify in the half-size Straus phase at {HS_NW} "
                              f"windows (512 S + 1023 M: 16 basepoint madds from the radix-2^16 rows)"),
            "phase_ms": {"scalars": float(ph[0]), "points": float(ph[1]), "hs_straus": float(ph[2])},
            "group": {"kernels": "scalars + points + hs_straus", "kernel_ms": kern_ms, "achieved": group / 1e12,
                      "frac": group / mad_rate,
                      "work_per_unit": f"{W_MAC_HS_GROUP} MAC per verify (half-size schedule: Straus + 2 decodes + 2 tables)"},
            "fe_mul_per_s": femul_rate,
            "cycle_basis": {
                "clock_ghz": cyc["clock_ghz"], "cycles_per_wave_mad": cyc["cycles_per_wave_instr"],
                "peak_at_measured_clock": cyc["mac_per_s"] / 1e12, "peak_at_2p4ghz": cyc["mac_per_s_at_2p4ghz"] / 1e12,
                "frac_vs_measured_clock": achieved / cyc["mac_per_s"],
                "frac_vs_2p4ghz": achieved / cyc["mac_per_s_at_2p4ghz"],
                "note": "peak = SIMDs x 64 lanes / cycles-per-wave-mad x clock; clock from s_memtime/s_memrealtime "
                        "over the same calibration launch"}}}
        if world == 1 and not args.no_cpu:
            D_["cpu_baseline"] = cpu_baseline(batch, local, args.cpu_seconds)
        pcie = pcie_h2d_probe(dev)
        if world == 1 and not args.no_host:
            D_["host_api"] = {"c2": host_api_rate(eng, batch, max(6, args.steps), value,
                                                  CONFIG_NAME[args.config] + " (host buffers)"),
                              "pcie_h2d_gb_per_s_pinned": pcie}
        if world == 1 and not args.no_sub:
            del batch
            torch.cuda.empty_cache()
            D_["c3"] = c3_line(eng, local, rank, world, sh, dev, 1_000_000, 3, 1, mad_rate)
            if not args.no_host:
                D_["host_api"]["c3"] = host_c3_rate(eng, local, sh, 1_000_000, 4, D_["c3"]["value"], pcie)
                D_["host_api"]["c3_fused"] = host_c3_fused_rate(eng, local, sh, 1_000_000, 4, D_["c3"]["value"], pcie)
            D_["c5_shard"] = c5_line(eng, local, rank, sh, dev, 8_000_000, 3, mad_rate, host_api=not args.no_host)
            if D_["c5_shard"].get("host_api") and "host_api" in D_:
                D_["host_api"]["c5"] = D_["c5_shard"].pop("host_api")
        if not args.no_keyed and world == 1:
            D_["keyed"] = keyed_rate(eng, local, n, msg_len, max(3, args.steps // 2), sh)
            if not args.no_host:
                D_["host_api"]["keyed"] = host_keyed_rate(eng, local, sh, n, msg_len, 8, D_["keyed"]["value"], pcie)
        if not args.no_notary:
            adv = workload.adversarial_records(os.path.join(REPO, "tests", "golden", "ed25519_corpus.npz"))
            cpu4 = world == 1 and not args.no_cpu
            # batches of 2^k signatures, k = 8..16, >= 200 timed repetitions per size
            D_["notary"] = notary_latency(eng, local, 4096, 200, cpu=cpu4, adv=adv)
            D_["notary_sweep"] = [notary_latency(eng, local, 1 << k, 200, cpu=False, adv=adv)
                                  for k in range(8, 17) if k != 12]
            D_["notary_keyed"] = notary_latency(eng, local, 4096, 200, cpu=False, key_pool=64, adv=adv)
            D_["resolve_chain"] = resolve_chain_latency(eng, local, 30, cpu=(world == 1 and not args.no_cpu))
        r3 = lambda x: None if x is None else float(f"{x:.4g}")  # noqa: E731
        R = D_["roofline"]
        result = {
            "metric": "Ed25519 verifies/sec (node)",
            "value": value,
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint32/uint64 (GF(2^255-19) radix 2^25.5 limbs, v_mad_u64_u32)",
            "data": "synthetic (keys, messages, signatures generated on-GPU from seeded RNG, RFC 8032 signing)",
            "config": {"workload": CONFIG_NAME[args.config], "sigs_per_gpu": n, "msg_bytes": msg_len,
                       "key_pool": args.key_pool or "distinct", "parallelism": f"shard-by-signature x{world}",
                       "device_streams": nstreams, "gpu_max_hw_queues": HW_QUEUES or "unset (HIP default 4)",
                       "collective": "RCCL all_gather of verdict bitmaps" if world > 1 else "none"},
            f"{other_key}_ms_per_step": r3(other_elapsed / args.steps * 1e3),
            f"{other_key}_value": r3(world * n * args.steps / other_elapsed),
            "roofline": {"bound": "valu", "achieved": r3(R["achieved"]), "peak": r3(R["peak"]), "unit": "Tmac/s",
                         "frac": r3(R["frac"]), "traffic": r3(traffic), "kernel": R["kernel"], "kernel_ms": r3(straus_ms),
                         "frac_vs_2p4ghz": r3(R["cycle_basis"]["frac_vs_2p4ghz"]),
                         "clock_ghz": r3(cyc["clock_ghz"]), "group_frac": r3(R["group"]["frac"]),
                         "phase_ms": {k: r3(v) for k, v in R["phase_ms"].items()},
                         "work_per_unit": f"{W_MAC_HS_STRAUS} MAC/verify", "traffic_source": PMC_HS_FILE,
                         # north_star's counters (committed PMC pass, PMC_HS_FILE): resident waves per SIMD, VALU
                         # instructions per MAC, SIMD cycles per VALU instruction, share of SIMD cycles issuing, LDS
                         # bank-conflict cycles
                         "occupancy": r3(pmc.get("occupancy_waves_per_simd")),
                         "valu_instr_per_mac": r3(pmc.get("valu_per_mac")),
                         "simd_cycles_per_valu_instr": r3(pmc.get("simd_cycles_per_valu")),
                         "valu_busy": r3(pmc.get("issue_active")),
                         "lds_bank_conflicts": pmc.get("lds_bank_conflict_cycles"),
                         # the same kernel over the largest whole number of resident-wave rounds <= n (HIP events):
                         # the 1M launch's partly filled last round is what separates frac from this
                         "frac_whole_rounds": r3(whole_rounds.get("frac")),
                         "whole_rounds_n": whole_rounds.get("n")},
        }
        if "cpu_baseline" in D_:
            c = D_["cpu_baseline"]
            result["cpu_baseline"] = {"value": r3(c["value"]), "unit": c["unit"], "cores": c["cores"], "kind": c["kind"],
                                      "sample": c["sample"], "single_thread_value": r3(c["single_thread_value"])}
        if "host_api" in D_:
            H = D_["host_api"]
            h = {"pcie_h2d_gb_per_s": r3(pcie)}
            for k in ("c2", "c5", "c3", "c3_fused", "keyed"):
                if k in H:
                    h[k] = {"value": r3(H[k]["value"]), "ratio": r3(H[k]["ratio_to_device_value"]),
                            "ms_per_step": r3(H[k]["ms_per_step"])}
            for k in ("c2", "c5"):
                if k in H:
                    h[k]["cold_ms_per_step"] = r3(H[k]["cold_ms_per_step"])
                    h[k]["sync_pinned_ratio"] = r3(H[k]["sync_pinned"]["ratio_to_device_value"])
                    h[k]["sync_pinned_ms"] = r3(H[k]["sync_pinned"]["ms_per_step"])
                    h[k]["pageable_ratio"] = r3(H[k]["pageable"]["ratio_to_device_value"])
                    h[k]["pageable_pack_ms"] = r3(H[k]["pageable"]["host_phases"]["pack_ms"])
            if "c2" in H:
                h["c2"]["sync_breakdown"] = {k: r3(v) for k, v in H["c2"]["sync_pinned"]["breakdown"].items()}
            if "c3_fused" in H:
                h["c3_fused"]["breakdown"] = {k: r3(v) for k, v in H["c3_fused"]["breakdown"].items()
                                              if k in ("merkle_dma_end_ms", "dma_end_ms", "merkle_busy_ms",
                                                       "verify_busy_ms", "idle_ms", "span_ms", "tail_ms",
                                                       "sync_call_ms")}
                h["c3_fused"]["pcie_floor_ms_per_step"] = r3(H["c3_fused"]["pcie_floor_ms_per_step"])
                h["c3_fused"]["cold_ms_per_step"] = r3(H["c3_fused"]["cold_ms_per_step"])
                h["c3_fused"]["timing"] = "steady state, T(K+2 calls) - T(2 calls); cold_ms_per_step: K calls from idle"
            if "keyed" in H:
                h["keyed"]["pcie_bound_value"] = r3(H["keyed"]["pcie_bound_value"])
                h["keyed"]["ratio_to_pcie_bound"] = r3(H["keyed"]["ratio_to_pcie_bound"])
            if "c3" in H:
                h["c3"]["pcie_floor_ms_per_step"] = r3(H["c3"]["pcie_floor_ms_per_step"])
                h["c3"]["cold_ms_per_step"] = r3(H["c3"]["cold_ms_per_step"])
            result["host_api"] = h
        if "c3" in D_:
            c = D_["c3"]
            result["c3"] = {"value": r3(c["value"]), "tx_ids_per_s": r3(c["tx_ids_per_s"]), "ms_per_step": r3(c["ms_per_step"]),
                            "merkle_ms": r3(c["phase_ms"]["merkle"]), "merkle_frac": r3(c["merkle_roofline"]["frac"]),
                            "hs_straus_frac": r3(c["roofline"]["frac"])}
        if "c5_shard" in D_:
            result["c5_shard"] = {"value": r3(D_["c5_shard"]["value"]), "hs_straus_frac": r3(D_["c5_shard"]["roofline"]["frac"])}
        D_.update(multi)
        if "c5" in multi:
            m = multi["c5"]
            result["c5"] = {"value": r3(m["value"]), "ms_per_step": r3(m["ms_per_step"]), "sigs_total": m["sigs_total"],
                            "gathered_all_ones": m["gathered_all_ones"]}
        if "c_abi_multi" in multi:
            m = multi["c_abi_multi"]
            result["c_abi_multi"] = {k: (r3(m[k]) if isinstance(m[k], float) else m[k]) for k in
                                     ("devices", "value", "ms_per_call", "async_value", "single_device_value",
                                      "efficiency_vs_devices_x_single", "async_efficiency_vs_devices_x_single")}
        if "keyed" in D_:
            K = D_["keyed"]
            comb_rate = n * W_MAC_COMB / (K["phase_ms"]["comb"] * 1e-3)
            K["roofline"] = {"bound": "valu", "kernel": "cv_comb_kernel", "achieved": comb_rate / 1e12,
                             "peak": mad_rate / 1e12, "unit": "Tmac/s", "frac": comb_rate / mad_rate,
                             "work_per_unit": f"{W_MAC_COMB} MAC/verify (224 S + 535 M)"}
            result["keyed"] = {"value": r3(K["value"]), "comb_ms": r3(K["phase_ms"]["comb"]),
                               "roofline": {"achieved": r3(comb_rate / 1e12), "peak": r3(mad_rate / 1e12),
                                            "unit": "Tmac/s", "frac": r3(comb_rate / mad_rate),
                                            "work_per_unit": f"{W_MAC_COMB} MAC/verify"}}
        if "notary" in D_:
            N = D_["notary"]
            result["notary"] = {"batch": 4096, "p50_ms": r3(N["p50_ms"]), "p99_ms": r3(N["p99_ms"]),
                                "pinned_p50_ms": r3(N["pinned_inputs"]["p50_ms"]), "cpu_p50_ms": r3(N.get("cpu_p50_ms")),
                                "cpu_threads": N.get("cpu_threads"),
                                "kernels_ms": {k: r3(v) for k, v in N.get("breakdown_p50_ms", {}).get("kernels", {}).items()}}
            result["notary_sweep_p50_p99_ms"] = {str(x["batch"]): [r3(x["p50_ms"]), r3(x["p99_ms"])] for x in D_["notary_sweep"]}
            result["notary_sweep_pinned_p50_ms"] = {str(x["batch"]): r3(x["pinned_inputs"]["p50_ms"])
                                                    for x in D_["notary_sweep"]}
            result["notary_keyed_p50_ms"] = r3(D_["notary_keyed"]["p50_ms"])
            result["resolve_chain"] = {"p50_ms": r3(D_["resolve_chain"]["p50_ms"]),
                                       "cpu_p50_ms": r3(D_["resolve_chain"].get("cpu_p50_ms"))}
        detail = args.detail or os.path.join(REPO, "gpurun_out", "bench_detail.json")
        try:
            os.makedirs(os.path.dirname(detail), exist_ok=True)
            with open(detail, "w") as f:
                json.dump({"line": result, "detail": D_}, f, indent=1)
            result["detail_file"] = os.path.relpath(detail, REPO)
        except OSError as ex:
            log(f"could not write {detail}: {ex}")
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier(group=cpu_group)
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
