"""Round-4 host-buffer paths through the drop-in boundary, on the GPU, against the C oracle and the golden corpus:

  - cv_merkle_tx_ids_ex / _async sharded over a context's devices and pipelined in sub-chunks (WireTransaction.id,
    core/src/main/kotlin/net/corda/core/transactions/WireTransaction.kt:45-52, MerkleTransaction.kt:26-38,66-99,
    reached by the resolve loop ResolveTransactionsFlow.kt:105-111);
  - the keyed path at throughput sizes through host buffers (per-key decode Kryo.kt:300-303):
    the plain entry points dedupe keys themselves and take the keyed pipeline;
  - concurrent callers on a multi-device context (NotaryFlow.kt:97-113,133-141: a notary's batches), routed
    whole to devices, every verdict exact.

Multi-device contexts are virtual device slots on the one GPU of the box (Engine(virtual_devices=k): k
independent devices — lock, worker, streams, workspace, key pool — on GPU 0)."""
import threading

import numpy as np
import pytest
import torch

from corda_amd import native, workload

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _bits(bitmap, n):
    return native.bitmap_to_bools(np.asarray(bitmap, dtype=np.uint64), n)


def _ragged_merkle_batch(seed, ntx, scattered=False):
    """ntx transactions with 0..12 leaves (empty ones included), lengths 0..700 bytes plus every 97th leaf
    of 3,900..9,000 bytes (past the leaf kernel's 63-block bucket), laid out in the arena in REVERSE order
    with gaps, starting 40 MB into it (offsets far from 0 and decreasing) — or, scattered, at random
    positions of a 64 MB arena (the staging gathers them: the compact form)."""
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, 13, ntx)
    counts[:4] = [0, 1, 2, 64]
    begin = np.zeros(ntx + 1, np.uint32)
    begin[1:] = np.cumsum(counts)
    nl = int(begin[-1])
    lens = rng.integers(0, 701, nl).astype(np.uint32)
    lens[::97] = rng.integers(3900, 9001, lens[::97].size).astype(np.uint32)
    if scattered:
        arena = rng.integers(0, 256, 64 << 20, dtype=np.uint8)
        off = rng.integers(0, arena.size - 9001, nl).astype(np.uint64)
    else:
        gaps = rng.integers(0, 40, nl)
        total = int(lens.sum() + gaps.sum())
        base = 40 << 20
        arena = rng.integers(0, 256, base + total + 64, dtype=np.uint8)
        ends = base + total - np.cumsum(lens.astype(np.int64) + gaps) + lens    # leaf i ends before leaf i-1 starts
        off = (ends - lens).astype(np.uint64)
    return arena, off, lens, begin


@pytest.mark.parametrize("scattered", [False, True])
def test_merkle_host_sharded_pipelined_vs_oracle(engine, oracle_c, scattered):
    """the host Merkle call on contexts of k = 1, 2, 3, 8 (virtual) devices, with forced
    small sub-chunks (many per shard), pageable and pinned inputs, synchronous and async: every id and status
    equals the C oracle's on a ragged 30,000-transaction batch (empty transactions, > 63-block leaves,
    non-monotone offsets far from 0 or scattered leaves)."""
    arena, off, lens, begin = _ragged_merkle_batch(11 + scattered, 30_000, scattered)
    ref_ids, ref_st = oracle_c.merkle_tx_ids(arena, off, lens, begin)
    assert ref_st.sum() > 0 and (ref_st == 0).sum() > 0
    pinned = [engine.host_copy(x) for x in (arena, off, lens, begin)]
    for k in (1, 2, 3, 8):
        e = engine if k == 1 else native.Engine(1, virtual_devices=k)
        try:
            e.set_option("merkle_chunk", 5000)                     # ~10 sub-chunks per shard
            e.set_option("shard_min", 64)                          # spread even this batch over every device
            e.stats("route", reset=True)
            ids, st = e.merkle_tx_ids(arena, off, lens, begin)
            assert np.array_equal(ids, ref_ids) and np.array_equal(st, ref_st), f"k={k}"
            r = e.stats("route")
            assert r["merkle_calls"] == 1 and r["shards"] == k, r
            if k == 1:                                             # 75 MB of leaves: the pipelined form
                assert r["merkle_subchunks"] >= 6, r
            out = e.host_empty((30_000, 32))
            ids_p, st_p = e.merkle_tx_ids(*pinned, ids=out)           # direct DMA in, ids DMAed into pinned memory
            assert np.array_equal(ids_p, ref_ids) and np.array_equal(st_p, ref_st)
            e.stats("route", reset=True)
            t1 = e.merkle_tx_ids_async(arena, off, lens, begin)      # async calls always pipeline
            t2 = e.merkle_tx_ids_async(*pinned)
            assert e.stats("route")["merkle_subchunks"] >= 12
            a2, s2 = e.wait(t2)
            a1, s1 = e.wait(t1)
            assert np.array_equal(a1, ref_ids) and np.array_equal(s1, ref_st)
            assert np.array_equal(a2, ref_ids) and np.array_equal(s2, ref_st)
        finally:
            e.set_option("merkle_chunk", 262144)
            e.set_option("shard_min", 4096)
            if k != 1:
                e.close()


def test_c3_host_step_async_overlap(engine):
    """The C3 node step through host buffers on the two async entry points: Merkle ids of batch k+1
    submitted while the verify of batch k runs; per transaction id == claimed AND all signatures valid.
    2,000 C3-shaped transactions x 8 signers, one in 16 with a mutated leaf, one in 32 with a bad signature."""
    ntx, signers = 2000, 8
    tb = workload.make_tx_batch(engine, 0, ntx, signers, seed=4401)
    arena = tb.leaf_arena.cpu().numpy().copy()
    leaf_off = tb.leaf_off.cpu().numpy().astype(np.uint64)
    leaf_len = tb.leaf_len.cpu().numpy().astype(np.uint32)
    tx_begin = tb.tx_begin.cpu().numpy().astype(np.uint32)
    claimed = tb.ids.cpu().numpy()
    pk, sig, _, _, _ = tb.sigs.to_host()
    sig = sig.copy()
    n = ntx * signers                                   # signature i signs the claimed id of tx i // signers
    msg_arena = np.concatenate([claimed.reshape(-1), np.zeros(16, np.uint8)])
    msg_off = (np.arange(n, dtype=np.uint64) // signers) * 32
    msg_len = np.full(n, 32, np.uint32)
    bad_leaf = np.arange(3, ntx, 16)
    arena[leaf_off[tx_begin[bad_leaf]].astype(np.int64)] ^= 1
    bad_sig = np.arange(5, ntx, 32)
    sig[bad_sig * signers + 2, 33] ^= 4
    expect = np.ones(ntx, bool)
    expect[bad_leaf] = False
    expect[bad_sig] = False
    sig_begin = np.arange(0, ntx * signers + 1, signers, dtype=np.uint32)
    tm = engine.merkle_tx_ids_async(arena, leaf_off, leaf_len, tx_begin)
    tv = engine.verify_batch_async(pk, sig, msg_arena, msg_off, msg_len, want_status=False)
    ids, st = engine.wait(tm)
    bm, _ = engine.wait(tv)
    ok = native.tx_verdicts(bm, sig_begin).astype(bool) & (ids == claimed).all(axis=1) & (st == 0)
    assert np.array_equal(ok, expect)


def _keyed_batch(engine, corpus, n, seed):
    """n signatures over 300-byte messages from a 1,024-key pool with corruptions: every 16th S bit, every
    97th R byte, every 101st message byte, every 1,009th key replaced by a golden not-a-point key."""
    b = workload.make_batch(engine, 0, n, 300, seed=seed, key_pool=1024)
    workload.corrupt_fraction(b, 16)
    idx = torch.arange(5, n, 97, device=DEV)
    b.sig[idx, 3] ^= 0x40
    pk, sig, arena, off, ln = b.to_host()
    del b
    torch.cuda.empty_cache()
    pk, arena = pk.copy(), arena.copy()
    midx = np.arange(7, n, 101)
    arena[off[midx].astype(np.int64) + 11] ^= 0x20
    bad = np.nonzero(corpus["status"] == 1)[0]
    kidx = np.arange(11, n, 1009)
    pk[kidx] = corpus["pk"][bad[kidx % len(bad)]]
    return pk, sig, arena, off, ln, kidx


def test_keyed_host_throughput_size_vs_oracle(engine, corpus, oracle_c):
    """2^20 + 12,345 signatures over a 1,024-key pool with S / R / message / golden
    bad-key corruptions through cv_ed25519_verify_batch: the engine's own dedupe takes the keyed pipeline
    (no 2^18 cap), and its verdicts and statuses equal the plain path's (auto-keyed off), the async form's,
    the explicit keyed entry point's, 2- and 3-device contexts' and the C oracle's."""
    n = (1 << 20) + 12_345
    pk, sig, arena, off, ln, kidx = _keyed_batch(engine, corpus, n, seed=9090)
    ref, rst = oracle_c.verify_batch(pk, sig, arena, off, ln, nthreads=16)
    assert 0.8 < ref.mean() < 0.95 and int(rst.sum()) == kidx.size
    engine.stats("route", reset=True)
    bm, st = engine.verify_batch(pk, sig, arena, off, ln)
    assert engine.stats("route")["keyed_shards"] >= 1, "the keyed path was not taken"
    assert np.array_equal(_bits(bm, n), ref.astype(bool)) and np.array_equal(st, rst)
    engine.set_option("auto_keyed", 0)
    try:
        bm_p, st_p = engine.verify_batch(pk, sig, arena, off, ln)
    finally:
        engine.set_option("auto_keyed", 1)
    assert np.array_equal(bm_p, bm) and np.array_equal(st_p, st)
    pinned = [engine.host_copy(x) for x in (pk, sig, arena, off, ln)]
    t = engine.verify_batch_async(*pinned)
    bm_a, st_a = engine.wait(t)
    assert np.array_equal(bm_a, bm) and np.array_equal(st_a, st)
    keys, inv = np.unique(pk, axis=0, return_inverse=True)
    bm_k, st_k = engine.verify_batch_keyed(keys, inv.reshape(-1).astype(np.uint32), sig, arena, off, ln)
    assert np.array_equal(bm_k, bm) and np.array_equal(st_k, st)
    for k in (2, 3):
        ve = native.Engine(1, virtual_devices=k)
        try:
            bm_v, st_v = ve.verify_batch(pk, sig, arena, off, ln)
            assert ve.stats("route")["keyed_shards"] == k
            assert np.array_equal(bm_v, bm) and np.array_equal(st_v, st), f"k={k}"
        finally:
            ve.close()


def test_concurrent_notary_batches_routed(corpus):
    """4 threads x 200 interleaved 4,096-signature golden-tiled batches (each thread its
    own random tiling, so each batch has its own verdict pattern) on a 4-device context: every verdict and
    status exact, no deadlock, and each batch routed whole to one device (no 4-way split of a notary batch)."""
    e = native.Engine(1, virtual_devices=4)
    errors = []
    npk = len(corpus["pk"])
    try:
        def worker(t):
            rng = np.random.default_rng(100 + t)
            try:
                for r in range(200):
                    sel = rng.integers(0, npk, 4096)
                    bm, st = e.verify_batch(corpus["pk"][sel], corpus["sig"][sel], corpus["arena"], corpus["off"][sel],
                                            corpus["len"][sel])
                    if not (np.array_equal(_bits(bm, 4096), corpus["verdict"][sel].astype(bool))
                            and np.array_equal(st, corpus["status"][sel])):
                        errors.append((t, r))
            except Exception as ex:  # noqa: BLE001
                errors.append((t, repr(ex)))

        e.stats("route", reset=True)
        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=240)
        assert not any(x.is_alive() for x in th), "a notary thread hung"
        assert not errors, errors[:5]
        r = e.stats("route")
        assert r["calls"] == 800 and r["routed_whole"] == 800, r
    finally:
        e.close()
