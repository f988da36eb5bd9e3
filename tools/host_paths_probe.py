"""Where the round-4 host-buffer paths spend their time (diagnostic, one JSON line per measurement):

  resolve   the resolve-chain step of bench.py (5,000 txs x 2 signers): the Merkle call, the verify call and the
            per-tx AND, each p50 over reps
  keyed     C2 with a 1,024-key pool through cv_ed25519_verify_batch(_async): wall time per call and the
            engine's host phases (cv_diag_stats CV_STATS_PIPE: plan incl. key dedupe, pack, wait, enqueue, sync)
  c3        the host C3 step of bench.py (1M txs x 8 signers): per-step wall time, time blocked on the Merkle
            ids and on the verdicts
  c3f       the same step through the fused cv_verify_transactions(_async), async then synchronous
            (MERKLE_STREAMS=0,1,2 C3F_ROUNDS=2: an interleaved A/B of CV_OPT_TXS_MERKLE_STREAM, async form)
  c3dev     the device C3 step (HBM-resident inputs), the host C3 ratios' denominator
  txsmall   notary-sized transaction batches (32 and 512 txs x 8 signers): fused call vs the separate calls, p50

    python tools/host_paths_probe.py [--what resolve,keyed,c3] [--reps N]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from corda_amd import native, workload  # noqa: E402


def p50(fn, reps):
    ts = []
    for r in range(reps + 3):
        t = time.perf_counter()
        fn()
        if r >= 3:
            ts.append(time.perf_counter() - t)
    return float(np.median(ts) * 1e3)


def resolve(eng, reps):
    ntx, signers = 5000, 2
    tb = workload.make_tx_batch(eng, 0, ntx, signers=signers, seed=5000)
    arena = tb.leaf_arena.cpu().numpy().copy()
    leaf_off = tb.leaf_off.cpu().numpy().astype(np.uint64)
    leaf_len = tb.leaf_len.cpu().numpy().astype(np.uint32)
    tx_begin = tb.tx_begin.cpu().numpy().astype(np.uint32)
    claimed = tb.ids.cpu().numpy()
    pk, sig, _, _, _ = tb.sigs.to_host()
    n = ntx * signers
    msg_arena = np.concatenate([claimed.reshape(-1), np.zeros(16, np.uint8)])
    msg_off = (np.arange(n, dtype=np.uint64) // signers) * 32
    msg_len = np.full(n, 32, np.uint32)
    sig_begin = np.arange(0, n + 1, signers, dtype=np.uint32)
    bm, _ = eng.verify_batch(pk, sig, msg_arena, msg_off, msg_len, want_status=False)
    out = {"what": "resolve", "txs": ntx,
           "merkle_ms": p50(lambda: eng.merkle_tx_ids(arena, leaf_off, leaf_len, tx_begin), reps),
           "verify_ms": p50(lambda: eng.verify_batch(pk, sig, msg_arena, msg_off, msg_len, want_status=False), reps),
           "and_ms": p50(lambda: native.tx_verdicts(bm, sig_begin), reps)}
    for k in ("auto_keyed",):
        eng.set_option(k, 0)
        out["verify_no_keyed_gate_ms"] = p50(lambda: eng.verify_batch(pk, sig, msg_arena, msg_off, msg_len,
                                                                      want_status=False), reps)
        eng.set_option(k, 1)
    print(json.dumps(out), flush=True)


def keyed(eng, reps):
    n = 1_000_000
    b = workload.make_batch(eng, 0, n, 300, seed=4243, key_pool=1024)
    arrs = tuple(eng.host_copy(x) for x in b.to_host())
    del b
    torch.cuda.empty_cache()
    eng.verify_batch(*arrs, want_status=False)
    for form in ("sync", "async2"):
        eng.stats("pipe", reset=True)
        t = time.perf_counter()
        pend = []
        for _ in range(reps):
            if form == "sync":
                eng.verify_batch(*arrs, want_status=False)
                continue
            pend.append(eng.verify_batch_async(*arrs, want_status=False))
            if len(pend) == 2:
                eng.wait(pend.pop(0))
        for tk in pend:
            eng.wait(tk)
        dt = (time.perf_counter() - t) / reps
        st = eng.stats("pipe", reset=True)
        calls = max(st["calls"], 1)
        print(json.dumps({"what": "keyed", "form": form, "ms_per_call": dt * 1e3,
                          "host_ms_per_call": {k: st[k] / calls * 1e3 for k in st if k.endswith("_s")},
                          "subchunks_per_call": st["subchunks"] / calls}), flush=True)
    pk = np.ascontiguousarray(arrs[0])
    t = time.perf_counter()
    native.dedupe_keys(pk)
    print(json.dumps({"what": "keyed", "dedupe_ms_diag_call": (time.perf_counter() - t) * 1e3}), flush=True)


def c3(eng, reps):
    import bench  # noqa: E402
    pcie = bench.pcie_h2d_probe(torch.device("cuda", 0))
    r = bench.host_c3_rate(eng, 0, 0, 1_000_000, reps, 1.0, pcie)
    r.pop("ratio_to_device_value", None)
    st = eng.stats("pipe")
    print(json.dumps({"what": "c3", **r, "pipe_stats": st}), flush=True)


def c3dev(eng, reps):
    """The device C3 step of bench.py (HBM-resident inputs): the denominator of the host C3 ratios, same box."""
    import bench  # noqa: E402
    st = torch.cuda.Stream(0)
    torch.cuda.set_stream(st)
    r = bench.run_c3(eng, 0, 0, 1, st.cuda_stream, torch.device("cuda", 0), 1_000_000, 4, 1)
    torch.cuda.set_stream(torch.cuda.default_stream(0))
    print(json.dumps({"what": "c3_device", "ms_per_step": r["elapsed"] / 4 * 1e3, "merkle_ms": r["merkle_ms"],
                      "phase_ms": [float(x) for x in r["phases"]]}), flush=True)


def txsmall(eng, reps):
    """A notary-sized batch of transactions (512 x 8 signers = 4,096 signatures, C3-shaped leaves) through the
    fused call against the separate Merkle + verify + cv_tx_verdicts calls: p50 per batch."""
    for ntx in (32, 512):
        signers = 8
        tb = workload.make_tx_batch(eng, 0, ntx, signers, seed=777 + ntx)
        arena = tb.leaf_arena.cpu().numpy().copy()
        leaf_off = tb.leaf_off.cpu().numpy().astype(np.uint64)
        leaf_len = tb.leaf_len.cpu().numpy().astype(np.uint32)
        tx_begin = tb.tx_begin.cpu().numpy().astype(np.uint32)
        claimed = tb.ids.cpu().numpy()
        pk, sig, _, _, _ = tb.sigs.to_host()
        n = ntx * signers
        sig_begin = np.arange(0, n + 1, signers, dtype=np.uint32)
        msg_off = (np.arange(n, dtype=np.uint64) // signers) * 32
        msg_len = np.full(n, 32, np.uint32)

        def separate():
            ids, st = eng.merkle_tx_ids(arena, leaf_off, leaf_len, tx_begin)
            bm, _ = eng.verify_batch(pk, sig, np.concatenate([ids.reshape(-1), np.zeros(16, np.uint8)]), msg_off,
                                     msg_len, want_status=False)
            return native.tx_verdicts(bm, sig_begin).astype(bool) & (st == 0)

        def fused():
            ok, ids, _, _ = eng.verify_transactions(arena, leaf_off, leaf_len, tx_begin, pk, sig, sig_begin,
                                                    want_status=False)
            return ok.astype(bool)

        assert separate().all() and fused().all() and (eng.merkle_tx_ids(arena, leaf_off, leaf_len, tx_begin)[0]
                                                        == claimed).all()
        print(json.dumps({"what": "txsmall", "txs": ntx, "sigs": n, "separate_p50_ms": p50(separate, reps),
                          "fused_p50_ms": p50(fused, reps)}), flush=True)


def c3f(eng, reps):
    import bench  # noqa: E402
    pcie = bench.pcie_h2d_probe(torch.device("cuda", 0))
    if os.environ.get("ASYNC_CHUNK"):                 # the async sub-chunk (CV_OPT_ASYNC_CHUNK) under test
        eng.set_option("async_chunk", int(os.environ["ASYNC_CHUNK"]))
    # C3F_CONFIGS="txs_merkle_stream=0;txs_merkle_stream=2,async_chunk=589824": an A/B of option sets (each config
    # k=v,... over the defaults), interleaved over C3F_ROUNDS (async form only unless C3F_SYNC=1);
    # MERKLE_STREAMS="0,1,2" is short for the configs txs_merkle_stream=0;...;txs_merkle_stream=2
    if os.environ.get("C3F_CONFIGS"):
        configs = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in c.split(",") if kv)
                   for c in os.environ["C3F_CONFIGS"].split(";")]
    elif os.environ.get("MERKLE_STREAMS"):
        configs = [{"txs_merkle_stream": int(x)} for x in os.environ["MERKLE_STREAMS"].split(",")]
    else:
        configs = [{}]
    defaults = {k: eng.get_option(k) for c in configs for k in c}
    forms = (False, True) if os.environ.get("C3F_SYNC", "1" if len(configs) == 1 else "0") == "1" else (False,)
    for _ in range(int(os.environ.get("C3F_ROUNDS", "1"))):
        for cfg in configs:
            for k, v in {**defaults, **cfg}.items():
                eng.set_option(k, v)
            mode = eng.get_option("txs_merkle_stream")
            for sync in forms:
                eng.stats("pipe", reset=True)
                try:
                    r = bench.host_c3_fused_rate(eng, 0, 0, 1_000_000, reps, 1.0, pcie, sync=sync)
                except AssertionError as e:
                    print(json.dumps({"what": "c3_fused", "sync": sync, "merkle_stream": mode, "config": cfg, "error": str(e)}),
                          flush=True)
                    continue
                r.pop("ratio_to_device_value", None)
                print(json.dumps({"what": "c3_fused", "sync": sync, "merkle_stream": mode, "config": cfg,
                                  "async_chunk": eng.get_option("async_chunk"), **r, "pipe_stats": eng.stats("pipe")}),
                      flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="resolve,keyed,c3")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    eng = native.Engine(1)
    for w in a.what.split(","):
        {"resolve": resolve, "keyed": keyed, "c3": c3, "c3f": c3f, "c3dev": c3dev,
         "txsmall": txsmall}[w](eng, a.reps if w not in ("c3", "c3f") else 4)
    eng.close()


if __name__ == "__main__":
    main()
