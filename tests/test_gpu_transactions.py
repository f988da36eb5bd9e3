"""cv_verify_transactions / _async — SignedTransaction.verifySignatures' id and signature checks for a batch in one
call (core/src/main/kotlin/net/corda/core/transactions/SignedTransaction.kt:59-71 with checkSignaturesAreValid
83-87 and WireTransaction.id, WireTransaction.kt:45-52): the Merkle ids are computed on the device and read there
as the signatures' messages.  Checked on the GPU against the C oracle (oracle/cv_oracle.py: the ids, and every
signature verified over its transaction's id) and against the separate entry points it fuses
(cv_merkle_tx_ids_ex + cv_ed25519_verify_batch + cv_tx_verdicts), result for result."""
import numpy as np
import pytest

from corda_amd import native, workload

pytestmark = pytest.mark.gpu


def _tx_case(engine, oracle_c, corpus, seed, ntx):
    """ntx transactions with ragged leaves (0..12, lengths 0..700 plus every 97th of 3,900..9,000 bytes, laid out
    in reverse order 8 MB into the arena) and ragged signature lists (0..19; the first transactions: no leaves
    with 3 signatures, 1 leaf with none, then 1, 64, 65 and 130 signatures), signed over the oracle's ids, then
    corrupted: every 37th signature's S, every 41st signature swapped for a corpus signature, every 53rd key
    replaced by a corpus key that is not a point."""
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, 13, ntx)
    counts[:6] = [0, 1, 2, 3, 1, 5]
    begin = np.zeros(ntx + 1, np.uint32)
    begin[1:] = np.cumsum(counts)
    nl = int(begin[-1])
    lens = rng.integers(0, 701, nl).astype(np.uint32)
    lens[::97] = rng.integers(3900, 9001, lens[::97].size).astype(np.uint32)
    gaps = rng.integers(0, 40, nl)
    total = int(lens.sum() + gaps.sum())
    base = 8 << 20
    arena = rng.integers(0, 256, base + total + 64, dtype=np.uint8)
    ends = base + total - np.cumsum(lens.astype(np.int64) + gaps) + lens
    off = (ends - lens).astype(np.uint64)
    ids_ref, st_ref = oracle_c.merkle_tx_ids(arena, off, lens, begin)

    scount = rng.integers(0, 20, ntx)
    scount[:6] = [3, 0, 1, 64, 65, 130]
    tsb = np.zeros(ntx + 1, np.uint32)
    tsb[1:] = np.cumsum(scount)
    nsig = int(tsb[-1])
    tx_of = np.repeat(np.arange(ntx), scount)
    msg_arena = np.concatenate([ids_ref.reshape(-1), np.zeros(16, np.uint8)])
    msg_off = tx_of.astype(np.uint64) * 32
    msg_len = np.full(nsig, 32, np.uint32)
    seeds = rng.integers(0, 256, (nsig, 32), dtype=np.uint8)
    pk, sig = engine.sign_batch(seeds, msg_arena, msg_off, msg_len)
    sig[::37, 40] ^= 0x10
    swap = np.arange(11, nsig, 41)
    sig[swap] = corpus["sig"][swap % len(corpus["sig"])]
    bad = np.nonzero(corpus["status"] == 1)[0]
    kbad = np.arange(7, nsig, 53)
    pk[kbad] = corpus["pk"][bad[kbad % len(bad)]]
    verdict, sstat = oracle_c.verify_batch(pk, sig, msg_arena, msg_off, msg_len, nthreads=8)
    ok = (st_ref == 0) & (scount > 0)
    all_valid = np.ones(ntx, bool)
    np.logical_and.at(all_valid, tx_of, verdict.astype(bool))
    ok &= all_valid
    assert 0 < ok.sum() < ntx and sstat.sum() > 0
    leaves = (arena, off, lens, begin)
    return leaves, (pk, sig, tsb), (ids_ref, st_ref, sstat, ok.astype(np.uint8)), (msg_arena, msg_off, msg_len)


def _check(out, ref, what):
    ok, ids, st, sst = out
    ids_ref, st_ref, sst_ref, ok_ref = ref
    assert np.array_equal(ids, ids_ref), what
    assert np.array_equal(st, st_ref), what
    assert np.array_equal(sst, sst_ref), what
    assert np.array_equal(ok, ok_ref), f"{what}: {np.nonzero(ok != ok_ref)[0][:10]}"


def test_verify_transactions_vs_oracle(engine, oracle_c, corpus):
    """4,000 ragged transactions (~38,000 signatures) on contexts of 1 and 3 (virtual) devices: synchronous calls
    (the small one-stream form at this size) from pageable and pinned inputs, and two async calls in flight (the
    pipeline, with small Merkle and signature sub-chunks: many launch groups per shard, signature groups that
    start mid-transaction): ids, Merkle statuses, signature statuses and per-transaction verdicts all equal the
    oracle's — and the separate entry points'."""
    leaves, sigs, ref, msgs = _tx_case(engine, oracle_c, corpus, 31, 4000)
    ntx = leaves[3].shape[0] - 1
    # the separate calls give the same results (the fused call's definition)
    ids_s, st_s = engine.merkle_tx_ids(*leaves)
    bm_s, sst_s = engine.verify_batch(sigs[0], sigs[1], *msgs)
    ok_s = native.tx_verdicts(bm_s, sigs[2]) & (st_s == 0)
    _check((ok_s, ids_s, st_s, sst_s), ref, "separate calls")
    pinned_l = [engine.host_copy(x) for x in leaves]
    pinned_s = [engine.host_copy(x) for x in sigs]
    for k in (1, 3):
        e = engine if k == 1 else native.Engine(1, virtual_devices=k)
        saved = {name: e.get_option(name) for name in ("merkle_chunk", "pipe_first", "pipe_chunk", "async_chunk",
                                                        "shard_min")}
        try:
            e.set_option("merkle_chunk", 3000)
            e.set_option("pipe_first", 1024)
            e.set_option("pipe_chunk", 3072)
            e.set_option("async_chunk", 2048)
            e.set_option("shard_min", 64)
            e.stats("route", reset=True)
            out = e.verify_transactions(*leaves, *sigs, want_sig_status=True)     # small shards: one-stream form
            _check(out, ref, f"k={k} pageable")
            r = e.stats("route")
            assert r["shards"] == k and r["merkle_subchunks"] == 0, r
            out = e.verify_transactions(*pinned_l, *pinned_s, ids=e.host_empty((ntx, 32)), want_sig_status=True)
            _check(out, ref, f"k={k} pinned")
            e.stats("route", reset=True)
            t1 = e.verify_transactions_async(*leaves, *sigs, want_sig_status=True)   # async: the pipeline
            t2 = e.verify_transactions_async(*pinned_l, *pinned_s, want_sig_status=True)
            assert e.stats("route")["merkle_subchunks"] >= 4 * k
            for t in (t2, t1):
                ok, rest = e.wait(t)
                _check((ok, *rest), ref, f"k={k} async")
            ok, ids, st, sst = e.verify_transactions(*leaves, *sigs, want_status=False)
            assert st is None and sst is None and np.array_equal(ok, ref[3]) and np.array_equal(ids, ref[0])
        finally:
            for name, v in saved.items():
                e.set_option(name, v)
            if k != 1:
                e.close()


def test_verify_transactions_edges(engine):
    """No transactions; transactions without signatures or leaves only; one transaction with one signature;
    malformed boundaries rejected (CV_E_ARGS) before anything runs."""
    empty = engine.verify_transactions(np.zeros(16, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32),
                                       np.zeros(1, np.uint32), np.zeros((0, 32), np.uint8), np.zeros((0, 64), np.uint8),
                                       np.zeros(1, np.uint32))
    assert empty[0].size == 0
    arena = np.arange(64, dtype=np.uint8)
    off = np.array([0, 10, 20], np.uint64)
    ln = np.array([10, 10, 30], np.uint32)
    lb = np.array([0, 1, 3, 3], np.uint32)                 # tx 2 has no leaves
    ok, ids, st, _ = engine.verify_transactions(arena, off, ln, lb, np.zeros((0, 32), np.uint8),
                                                np.zeros((0, 64), np.uint8), np.zeros(4, np.uint32))
    assert ok.tolist() == [0, 0, 0] and st.tolist() == [0, 0, 1]
    ids2, _ = engine.merkle_tx_ids(arena, off, ln, lb)
    assert np.array_equal(ids, ids2)
    seed = np.full((1, 32), 7, np.uint8)
    pk, sig = engine.sign_batch(seed, ids2[1].copy(), np.zeros(1, np.uint64), np.full(1, 32, np.uint32))
    ok, _, _, sst = engine.verify_transactions(arena, off, ln, lb, pk, sig, np.array([0, 0, 1, 1], np.uint32),
                                               want_sig_status=True)
    assert ok.tolist() == [0, 1, 0] and sst.tolist() == [0]
    sig[0, 5] ^= 1
    ok, _, _, _ = engine.verify_transactions(arena, off, ln, lb, pk, sig, np.array([0, 0, 1, 1], np.uint32))
    assert ok.tolist() == [0, 0, 0]
    with pytest.raises(native.CvError) as ex:               # decreasing signature boundaries
        engine.verify_transactions(arena, off, ln, lb, pk, sig, np.array([0, 1, 0, 1], np.uint32))
    assert ex.value.code == -3


@pytest.mark.parametrize("mstream", [0, 1, 2])
def test_verify_transactions_c3_shaped(engine, oracle_c, mstream):
    """C3-shaped transactions (6 leaves, 8 signers each, workload.make_tx_batch), 200,000 of them (1.6M signatures,
    the default sub-chunk plans: signature groups that start inside the previous Merkle sub-chunk): one in 16
    with a mutated leaf, one in 32 with a bad signature; tx_ok equals the expectation and the ids the claimed
    ids wherever the leaves are intact — synchronous (the last call also timed on the GPU), and three async calls in
    flight; the expectation itself is the C oracle's on the first 3,000 transactions.  mstream: the stream the
    Merkle groups run on (CV_OPT_TXS_MERKLE_STREAM: the compute streams, the copy stream, their own — the default)."""
    saved = engine.get_option("txs_merkle_stream")
    engine.set_option("txs_merkle_stream", mstream)
    try:
        _c3_shaped(engine, oracle_c)
    finally:
        engine.set_option("txs_merkle_stream", saved)


def _c3_shaped(engine, oracle_c):
    ntx, signers = 200_000, 8
    tb = workload.make_tx_batch(engine, 0, ntx, signers, seed=4402)
    arena = tb.leaf_arena.cpu().numpy().copy()
    leaf_off = tb.leaf_off.cpu().numpy().astype(np.uint64)
    leaf_len = tb.leaf_len.cpu().numpy().astype(np.uint32)
    tx_begin = tb.tx_begin.cpu().numpy().astype(np.uint32)
    claimed = tb.ids.cpu().numpy()
    pk, sig, _, _, _ = tb.sigs.to_host()
    sig = sig.copy()
    bad_leaf = np.arange(3, ntx, 16)
    arena[leaf_off[tx_begin[bad_leaf]].astype(np.int64)] ^= 1
    bad_sig = np.arange(5, ntx, 32)
    sig[bad_sig * signers + 2, 33] ^= 4
    expect = np.ones(ntx, bool)
    expect[bad_leaf] = False                                # its id changes: the claimed-id signatures fail
    expect[bad_sig] = False
    sig_begin = np.arange(0, ntx * signers + 1, signers, dtype=np.uint32)
    args = (arena, leaf_off, leaf_len, tx_begin, pk, sig, sig_begin)
    intact = np.isin(np.arange(ntx), bad_leaf, invert=True)
    # the constructed expectation, checked against the C oracle on a slice: the slice's ids
    # recomputed from its leaves, its signatures verified over the CLAIMED ids, tx_ok = ids match AND all valid
    k = 3000
    l_end = int(tx_begin[k])
    o_ids, o_st = oracle_c.merkle_tx_ids(arena, leaf_off[:l_end], leaf_len[:l_end], tx_begin[:k + 1])
    c_arena = np.concatenate([claimed[:k].reshape(-1), np.zeros(16, np.uint8)])
    o_v, _ = oracle_c.verify_batch(pk[:k * signers], sig[:k * signers], c_arena,
                                   (np.arange(k * signers, dtype=np.uint64) // signers) * 32,
                                   np.full(k * signers, 32, np.uint32), nthreads=8)
    o_ok = (o_ids == claimed[:k]).all(axis=1) & (o_st == 0) & o_v.reshape(k, signers).astype(bool).all(axis=1)
    assert np.array_equal(o_ok, expect[:k]) and not o_ok.all() and o_ok.sum() > k // 2
    for rep in range(3):
        if rep == 2:                                        # the last one timed on the GPU (CV_OPT_TIMELINE)
            engine.set_option("timeline", 1)
            engine.stats("timeline", reset=True)
        try:
            ok, ids, st, _ = engine.verify_transactions(*args)
        finally:
            engine.set_option("timeline", 0)
        assert np.array_equal(ok.astype(bool), expect), (rep, np.nonzero(ok.astype(bool) != expect)[0][:10])
        assert np.array_equal((ids == claimed).all(axis=1), intact) and (st == 0).all()
    t = engine.stats("timeline", reset=True)             # Merkle and verify groups timed apart, consistently
    assert t["calls"] == 1 and t["groups"] >= 2 and t["merkle_busy_ms"] > 0 and t["verify_busy_ms"] > 0
    assert t["merkle_dma_end_ms"] <= t["dma_end_ms"] <= t["span_ms"] and t["ramp_ms"] <= t["span_ms"]
    assert max(t["merkle_busy_ms"], t["verify_busy_ms"]) <= t["busy_ms"] + 1e-3
    assert abs(t["busy_ms"] + t["idle_ms"] - (t["span_ms"] - t["ramp_ms"])) < 1e-3
    pinned = [engine.host_copy(x) for x in args]
    tickets = [engine.verify_transactions_async(*(pinned if k % 2 else args)) for k in range(3)]
    for t in tickets:
        ok, (ids, st, _) = engine.wait(t)
        assert np.array_equal(ok.astype(bool), expect)
        assert np.array_equal((ids == claimed).all(axis=1), intact) and (st == 0).all()


@pytest.mark.parametrize("ntx", [40, 30_000])
def test_leaf_arena_bound(engine, oracle_c, corpus, ntx):
    """cv_merkle_tx_ids_bounded / cv_verify_transactions_ex: the engine bounds the leaves by the caller's arena size in
    its own staging scan (the binding no longer scans 12 B per leaf before every call).  At the exact extent the
    results equal the unbounded calls'; one byte short, and with a leaf whose off + len wraps, every form returns
    CV_E_ARGS (small one-DMA shards at 40 transactions, the pipeline at 30,000, synchronous and with a ticket), and the
    binding raises ValueError; the engine stays exact afterwards."""
    import ctypes
    leaves, sigs, ref, _ = _tx_case(engine, oracle_c, corpus, 7100 + ntx, ntx)
    arena, off, lens, begin = leaves
    pk, sig, tsb = sigs
    ids_ref, st_ref, _, ok_ref = ref
    lib, p = native.load(), native._p
    extent = int((off + lens.astype(np.uint64)).max())
    for async_ in (False, True):
        for bound, want in ((extent, 0), (extent - 1, -3)):
            t = ctypes.c_uint64()
            tk = ctypes.byref(t) if async_ else None
            ids = np.zeros((ntx, 32), np.uint8)
            st = np.zeros(ntx, np.uint8)
            ok = np.zeros(ntx, np.uint8)
            rc = lib.cv_merkle_tx_ids_bounded(engine._h, ntx, p(arena), bound, p(off), p(lens), p(begin), p(ids), p(st),
                                              tk)
            assert rc == want, ("merkle", async_, bound, rc)
            if rc == 0 and async_:
                assert lib.cv_wait(engine._h, t.value) == 0
            if rc == 0:
                assert np.array_equal(ids, ids_ref) and np.array_equal(st, st_ref)
            rc = lib.cv_verify_transactions_ex(engine._h, ntx, p(arena), bound, p(off), p(lens), p(begin), p(pk), p(sig),
                                               p(tsb), p(ids), p(st), None, p(ok), tk)
            assert rc == want, ("txs", async_, bound, rc)
            if rc == 0 and async_:
                assert lib.cv_wait(engine._h, t.value) == 0
            if rc == 0:
                assert np.array_equal(ok, ok_ref) and np.array_equal(ids, ids_ref)
    with pytest.raises(ValueError, match="exceeds the arena"):
        engine.verify_transactions(arena[:extent - 1], off, lens, begin, pk, sig, tsb)
    with pytest.raises(ValueError, match="exceeds the arena"):
        engine.merkle_tx_ids(arena[:extent - 1], off, lens, begin)
    wrap_off, wrap_len = off.copy(), lens.copy()
    last = int(begin[-1]) - 1
    wrap_off[last], wrap_len[last] = np.uint64(2 ** 64 - 8), 32
    for bound in (arena.size, 2 ** 64 - 1):
        rc = lib.cv_verify_transactions_ex(engine._h, ntx, p(arena), bound, p(wrap_off), p(wrap_len), p(begin), p(pk),
                                           p(sig), p(tsb), None, None, None, p(np.zeros(ntx, np.uint8)), None)
        assert rc == -3, bound
    with pytest.raises(ValueError, match="exceeds the arena"):
        engine.verify_transactions_async(arena, wrap_off, wrap_len, begin, pk, sig, tsb)
    ok, ids, st, _ = engine.verify_transactions(arena, off, lens, begin, pk, sig, tsb)
    assert np.array_equal(ok, ok_ref) and np.array_equal(ids, ids_ref) and np.array_equal(st, st_ref)
