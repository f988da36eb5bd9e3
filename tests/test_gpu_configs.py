"""BASELINE configs C3 and C5 at full size on the GPU, the C-ABI's multi-device host path, and the
device API's cross-stream ordering.

C3 (IRS-demo shape, samples/irs-demo/.../NodeInterestRates.kt:189-224): 1M transactions x 8 signers,
6 leaves per transaction (2 x 120, 2 x 600, 2 x 300 bytes, +-25 %).  One step = every
WireTransaction.id recomputed (leaf SHA-256 + Merkle tree, MerkleTransaction.kt:26-38,66-99), every
signature verified over its transaction's claimed id (SignedTransaction.kt:82-87), then per
transaction: id matches AND all signature bits set (SignedTransaction.kt:58-72).
C5 shard: the per-GPU share of the 64M-signature run, 8M signatures over 32-byte tx ids (4
workspace chunks).  Full sizes are checked through size-independent properties (all honest accepted;
an exact corruption pattern rejected); the oracle checks slices.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from corda_amd import distributed as D  # noqa: E402
from corda_amd import native, workload  # noqa: E402

DEV = "cuda:0"


def _bits(bm_tensor, n):
    return native.bitmap_to_bools(bm_tensor.cpu().numpy().view(np.uint64), n)


def _rejected_corpus(corpus):
    """Golden-corpus items the oracle rejects, with their messages (for substitution into batches)."""
    rej = np.nonzero(corpus["verdict"] == 0)[0]
    return rej


def test_c3_irs_shape(engine, corpus, oracle_c):
    ntx, signers = 1_000_000, 8
    tb = workload.make_tx_batch(engine, 0, ntx, signers, seed=303)
    n = tb.sigs.n
    nleaves = int(tb.leaf_len.numel())
    # --- corruption pattern: leaf bytes (id mismatch), S bits, golden adversarial records
    arena = tb.leaf_arena.clone()
    bad_leaf_tx = torch.arange(5, ntx, 64, device=DEV)
    leaf_idx = tb.tx_begin[bad_leaf_tx].to(torch.int64) + 2                    # the third leaf of the tx
    arena[tb.leaf_off[leaf_idx]] ^= 0x5A
    sig = tb.sigs.sig.clone()
    pk = tb.sigs.pk.clone()
    bad_sig_tx = torch.arange(0, ntx, 16, device=DEV)
    sig[bad_sig_tx * signers + 3, 40] ^= 1                                      # signer 3's S
    # golden rejected records (own messages appended to the id arena), every 1000th tx, signer 7
    rej = _rejected_corpus(corpus)
    adv_tx = torch.arange(11, ntx, 1000, device=DEV)
    na = int(adv_tx.numel())
    pick = rej[np.arange(na) % rej.size]
    msgs = [corpus["arena"][corpus["off"][i]:corpus["off"][i] + corpus["len"][i]] for i in pick]
    id_arena = tb.sigs.arena
    base = int(id_arena.numel())
    adv_arena = np.concatenate(msgs + [np.zeros(16, np.uint8)])
    msg_arena = torch.cat([id_arena, torch.from_numpy(adv_arena).to(DEV)])
    off = tb.sigs.off.clone()
    ln = tb.sigs.len.clone()
    adv_sig_idx = adv_tx * signers + 7
    lens = np.array([m.size for m in msgs], np.int64)
    starts = np.zeros(na, np.int64)
    starts[1:] = np.cumsum(lens[:-1])
    off[adv_sig_idx] = torch.from_numpy(base + starts).to(DEV)
    ln[adv_sig_idx] = torch.from_numpy(lens.astype(np.int32)).to(DEV)
    pk[adv_sig_idx] = torch.from_numpy(corpus["pk"][pick]).to(DEV)
    sig[adv_sig_idx] = torch.from_numpy(corpus["sig"][pick]).to(DEV)

    def c3_step(leaf_arena, pk_, sig_, arena_, off_, ln_):
        ids = torch.empty_like(tb.ids)
        ws = torch.empty(nleaves * 32, dtype=torch.uint8, device=DEV)
        st = torch.full((ntx,), 9, dtype=torch.uint8, device=DEV)
        engine.merkle_device(0, ntx, nleaves, leaf_arena.data_ptr(), tb.leaf_off.data_ptr(), tb.leaf_len.data_ptr(),
                             tb.tx_begin.data_ptr(), ws.data_ptr(), ids.data_ptr(), st.data_ptr())
        bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=DEV)
        engine.verify_device(0, n, pk_.data_ptr(), sig_.data_ptr(), arena_.data_ptr(), off_.data_ptr(),
                             ln_.data_ptr(), bm.data_ptr())
        engine.synchronize(0)
        ok = D.tx_verdicts_torch(bm, tb.sig_tx_begin) & (ids == tb.ids).all(dim=1) & (st == 0)
        return ok, ids, bm

    # honest: every transaction valid
    ok, ids, bm = c3_step(tb.leaf_arena, tb.sigs.pk, tb.sigs.sig, tb.sigs.arena, tb.sigs.off, tb.sigs.len)
    assert bool(ok.all()) and bool((ids == tb.ids).all()) and bool((bm == -1).all())
    # corrupted: exactly the pattern
    ok, ids, bm = c3_step(arena, pk, sig, msg_arena, off, ln)
    expect = torch.ones(ntx, dtype=torch.bool, device=DEV)
    expect[bad_leaf_tx] = False
    expect[bad_sig_tx] = False
    expect[adv_tx] = False
    assert torch.equal(ok, expect)
    id_changed = ~(ids == tb.ids).all(dim=1)
    assert torch.equal(torch.nonzero(id_changed).flatten(), bad_leaf_tx)
    # oracle on a 20k-transaction slice (160k signatures + the slice's leaves)
    lo, hi = 0, 20_000
    a0 = int(tb.leaf_off[lo * 6])
    a1 = int(tb.leaf_off[hi * 6 - 1] + tb.leaf_len[hi * 6 - 1])
    h_arena = arena[a0:a1].cpu().numpy()
    h_off = (tb.leaf_off[lo * 6:hi * 6] - a0).cpu().numpy().astype(np.uint64)
    h_len = tb.leaf_len[lo * 6:hi * 6].cpu().numpy().astype(np.uint32)
    h_beg = (tb.tx_begin[lo:hi + 1] - lo * 6).cpu().numpy().astype(np.uint32)
    ref_ids, ref_st = oracle_c.merkle_tx_ids(h_arena, h_off, h_len, h_beg)
    assert np.array_equal(ref_ids, ids[lo:hi].cpu().numpy()) and not ref_st.any()
    s0, s1 = lo * signers, hi * signers
    h_msg = msg_arena.cpu().numpy()
    ref_v, ref_s = oracle_c.verify_batch(pk[s0:s1].cpu().numpy(), sig[s0:s1].cpu().numpy(), h_msg,
                                         off[s0:s1].cpu().numpy().view(np.uint64),
                                         ln[s0:s1].cpu().numpy().view(np.uint32), nthreads=16)
    assert np.array_equal(_bits(bm, n)[s0:s1], ref_v.astype(bool))


def test_c5_shard_8m(engine):
    """C5's per-GPU shard: 8M signatures over 32-byte ids (four 2^21-signature workspace chunks plus a
    tail), honest then with one S bit flipped in every 16th and one R byte in every 1,001st."""
    n = 8_000_000
    b = workload.make_batch(engine, 0, n, 32, seed=505)
    bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device=DEV)
    engine.verify_device(0, n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                         b.len.data_ptr(), bm.data_ptr())
    engine.synchronize(0)
    assert bool((bm == -1).all())
    expect = workload.corrupt_fraction(b, 16)
    r_idx = torch.arange(7, n, 1001, device=DEV)
    b.sig[r_idx, 5] ^= 0x40
    expect[r_idx] = False
    engine.verify_device(0, n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                         b.len.data_ptr(), bm.data_ptr())
    engine.synchronize(0)
    got = torch.from_numpy(_bits(bm, n)).to(DEV)
    assert torch.equal(got, expect)


def _virtual_engine(k):
    return native.Engine(1, virtual_devices=k)


@pytest.mark.parametrize("k", [2, 3, 8])
def test_multi_device_host_path_virtual_shards(engine, corpus, oracle_c, k):
    """VERDICT r1 #7 / ADVICE: the C-ABI's multi-device path (for_each_shard: one host thread, stream
    and workspace per device, 64-aligned contiguous shards) run with k device slots on one GPU.
    Plain path: fresh distinct-key signatures with corruptions at a ragged size; auto-keyed path: the
    golden corpus tiled (its keys repeat, so the host dedupe picks the keyed path per shard); explicit
    keyed entry point.  Every verdict and status byte equals the single-device engine's and the
    golden / oracle verdicts."""
    ve = _virtual_engine(k)
    try:
        assert ve.device_count == k
        # plain: distinct keys, ragged n
        n = 64 * 3 * k + 37
        b = workload.make_batch(engine, 0, n, 32, seed=700 + k)
        expect = workload.corrupt_fraction(b, 5).cpu().numpy()
        pk, sig, arena, off, ln = b.to_host()
        bm_v, st_v = ve.verify_batch(pk, sig, arena, off, ln)
        bm_1, st_1 = engine.verify_batch(pk, sig, arena, off, ln)
        assert np.array_equal(bm_v, bm_1) and np.array_equal(st_v, st_1)
        assert np.array_equal(native.bitmap_to_bools(bm_v, n), expect)
        # auto-keyed: golden corpus tiled to a ragged size (keys repeat)
        m = 6 * len(corpus["pk"]) + 64 * k + 5             # above 4,096: the dedupe runs
        idx = np.arange(m) % len(corpus["pk"])
        args = (corpus["pk"][idx], corpus["sig"][idx], corpus["arena"], corpus["off"][idx], corpus["len"][idx])
        bm_v, st_v = ve.verify_batch(*args)
        bm_1, st_1 = engine.verify_batch(*args)
        assert np.array_equal(bm_v, bm_1) and np.array_equal(st_v, st_1)
        assert np.array_equal(native.bitmap_to_bools(bm_v, m), corpus["verdict"][idx].astype(bool))
        assert np.array_equal(st_v, corpus["status"][idx])
        # explicit keyed entry point over a 16-key pool
        kb = workload.make_batch(engine, 0, 1000 + k, 32, seed=800 + k, key_pool=16)
        kexp = workload.corrupt_fraction(kb, 7).cpu().numpy()
        kpk, ksig, karena, koff, kln = kb.to_host()
        keys = kpk[:16]
        kidx = kb.key_index.cpu().numpy().astype(np.uint32)
        bm_v, st_v = ve.verify_batch_keyed(keys, kidx, ksig, karena, koff, kln)
        assert np.array_equal(native.bitmap_to_bools(bm_v, kb.n), kexp)
        ref, _ = oracle_c.verify_batch(kpk, ksig, karena, koff, kln, nthreads=8)
        assert np.array_equal(ref.astype(bool), kexp)
    finally:
        ve.close()


def test_device_calls_on_two_streams_are_ordered(engine, corpus):
    """two device-API verifies enqueued back to back on different streams share the
    device's workspace; the engine orders them (the second stream waits for the first call's work),
    so each bitmap is right.  Batch A honest, batch B with every 3rd signature corrupted."""
    n = 300_000
    a = workload.make_batch(engine, 0, n, 32, seed=901)
    bb = workload.make_batch(engine, 0, n, 32, seed=902)
    exp_b = workload.corrupt_fraction(bb, 3)
    s1, s2 = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    bm_a = torch.zeros((n + 63) // 64, dtype=torch.int64, device=DEV)
    bm_b = torch.zeros_like(bm_a)
    torch.cuda.synchronize()
    for _ in range(3):
        engine.verify_device(0, n, a.pk.data_ptr(), a.sig.data_ptr(), a.arena.data_ptr(), a.off.data_ptr(),
                             a.len.data_ptr(), bm_a.data_ptr(), 0, s1.cuda_stream)
        engine.verify_device(0, n, bb.pk.data_ptr(), bb.sig.data_ptr(), bb.arena.data_ptr(), bb.off.data_ptr(),
                             bb.len.data_ptr(), bm_b.data_ptr(), 0, s2.cuda_stream)
    torch.cuda.synchronize()
    assert _bits(bm_a, n).all()
    assert torch.equal(torch.from_numpy(_bits(bm_b, n)).to(DEV), exp_b)
