"""The pipelined host-buffer path (cv_ed25519_verify_batch above the pipeline threshold: sub-chunks dealt
over the device's workspace slots, packing / DMA / kernels overlapped), the device API's workspace slots
(calls on different streams run concurrently), and RCCL on the GPU (a 1-rank "nccl" group).

Reference call sites the host path replaces: SignedTransaction.checkSignaturesAreValid
(core/src/main/kotlin/net/corda/core/transactions/SignedTransaction.kt:82-87) and the resolve loop
(core/src/main/kotlin/net/corda/flows/ResolveTransactionsFlow.kt:105-111); the commit-step gather
replaces NotaryFlow.kt:133-141's single-node view."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch

from corda_amd import native, workload

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _bits(bitmap, n):
    return native.bitmap_to_bools(np.asarray(bitmap, dtype=np.uint64), n)


class _opts:
    """Per-context options (cv_set_option) set for the block and restored after it."""

    def __init__(self, engine, **kw):
        self.e, self.kw = engine, kw

    def __enter__(self):
        self.old = {k: self.e.get_option(k) for k in self.kw}
        for k, v in self.kw.items():
            self.e.set_option(k, v)

    def __exit__(self, *a):
        for k, v in self.old.items():
            self.e.set_option(k, v)


def _bad_key_records(corpus):
    """golden records whose key is not a valid point (status CV_SIG_BAD_KEY, verdict 0)"""
    return np.nonzero(corpus["status"] == 1)[0]


def test_host_pipeline_large_exact_pattern(engine, corpus):
    """2^22 + 200,003 distinct-key signatures over 300-byte messages through the
    host-buffer C-ABI — the pipeline's sub-chunks cross the 2^22 workspace-chunk boundary and end ragged.
    Every 16th S bit flipped (rejected), every 97th R byte flipped (rejected), every 1,009th key replaced
    by a golden not-a-point key (rejected, status 1); everything else accepted; bits past n clear."""
    n = (1 << 22) + 200_003
    b = workload.make_batch(engine, 0, n, 300, seed=3101)
    expect = workload.corrupt_fraction(b, 16)
    idx = torch.arange(5, n, 97, device=DEV)
    b.sig[idx, 3] ^= 0x40
    expect[idx] = False
    pk, sig, arena, off, ln = b.to_host()
    del b
    torch.cuda.empty_cache()
    pk = pk.copy()
    bad = _bad_key_records(corpus)
    kidx = np.arange(11, n, 1009)
    pk[kidx] = corpus["pk"][bad[kidx % len(bad)]]
    exp = expect.cpu().numpy()
    exp[kidx] = False
    st_exp = np.zeros(n, np.uint8)
    st_exp[kidx] = 1
    bitmap, status = engine.verify_batch(pk, sig, arena, off, ln)
    got = _bits(bitmap, n)
    assert np.array_equal(got, exp), f"{int((got != exp).sum())} verdicts differ"
    assert np.array_equal(status, st_exp)
    assert int(bitmap[-1]) >> (n % 64) == 0


@pytest.mark.parametrize("n", [131_137, 600_001])
def test_host_pipeline_sync_subchunk_plan_exact(engine, n):
    """Synchronous calls cut their batch in about n / 16 records per sub-chunk after the ramp (at least 2 x
    pipe_first, at most pipe_chunk): sizes just above the pipeline threshold and mid-way to a C2 batch, from
    pinned buffers (direct DMA) and pageable ones (packed), every 13th S corrupted and every 101st R byte:
    every verdict exact, bits past n clear."""
    b = workload.make_batch(engine, 0, n, 300, seed=n)
    expect = workload.corrupt_fraction(b, 13)
    idx = torch.arange(7, n, 101, device=DEV)
    b.sig[idx, 5] ^= 0x08
    expect[idx] = False
    arrs = b.to_host()
    del b
    exp = expect.cpu().numpy()
    for form, a in (("pageable", arrs), ("pinned", tuple(engine.host_copy(x) for x in arrs))):
        bitmap, _ = engine.verify_batch(*a, want_status=False)
        got = _bits(bitmap, n)
        assert np.array_equal(got, exp), f"{form}: {int((got != exp).sum())} verdicts differ"
        assert int(bitmap[-1]) >> (n % 64) == 0


@pytest.mark.parametrize("first,chunk,overlap,slots", [(64, 64 * 17, 1, 2), (64 * 5, 64 * 3, 1, 2), (1024, 4096, 1, 2),
                                                       (1024, 4096, 0, 2), (8192, 8192, 1, 2), (64 * 5, 64 * 3, 1, 3),
                                                       (1024, 4096, 1, 3), (64 * 5, 64 * 3, 1, 4), (1024, 4096, 0, 4)])
def test_host_pipeline_small_subchunks_golden(engine, corpus, first, chunk, overlap, slots):
    """The pipeline forced onto tiny sub-chunks (first / steady sizes, so one batch has hundreds of
    them, in every kernel form from tri-chain to throughput) over the golden corpus tiled to a ragged
    9,001 records in random order: every verdict and status byte equals the pinned corpus values; with and
    without the first sub-chunk's keys-first prep overlap (CV_OPT_PIPE_OVERLAP_FIRST), over two, three and four
    compute streams (CV_OPT_PIPE_SLOTS)."""
    rng = np.random.default_rng(first + chunk)
    n = 9001
    sel = rng.integers(0, len(corpus["pk"]), n)
    with _opts(engine, pipe_min=512, pipe_first=first, pipe_chunk=chunk, host_threads=3, auto_keyed=0,
               pipe_overlap_first=overlap, pipe_slots=slots):
        bitmap, status = engine.verify_batch(corpus["pk"][sel], corpus["sig"][sel], corpus["arena"],
                                             corpus["off"][sel], corpus["len"][sel])
    assert np.array_equal(_bits(bitmap, n), corpus["verdict"][sel].astype(bool))
    assert np.array_equal(status, corpus["status"][sel])
    assert int(bitmap[-1]) >> (n % 64) == 0


def test_host_pipeline_scattered_arena(engine, corpus, oracle_c):
    """Messages scattered over a 96 MB arena in reverse order with gaps (the staging gathers them back
    to back: the "compact" form), mixed lengths 0..700 bytes, corrupted S / R / keys: the pipelined and
    the small host paths both equal the C oracle."""
    rng = np.random.default_rng(77)
    n = 200_000
    lens = rng.integers(0, 701, n).astype(np.uint32)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    arena = np.zeros(96 << 20, np.uint8)
    gap = (arena.size - int(lens.sum()) - 64) // n
    offs = np.zeros(n, np.uint64)
    pos = arena.size - 32
    for i in range(n):                               # last record first: offsets decrease
        pos -= int(lens[i]) + int(rng.integers(0, gap + 1))
        offs[i] = pos
    arena[:] = rng.integers(0, 256, arena.size, dtype=np.uint8)
    pk, sig = engine.sign_batch(seeds, arena, offs, lens)
    sig[1::9, 40] ^= 0x04
    sig[2::13, 7] ^= 0x01
    pk[3::17, 30] ^= 0x20
    ref, rst = oracle_c.verify_batch(pk, sig, arena, offs, lens, nthreads=8)
    bitmap, status = engine.verify_batch(pk, sig, arena, offs, lens)
    assert np.array_equal(_bits(bitmap, n), ref.astype(bool))
    assert np.array_equal(status, rst)
    with _opts(engine, pipe_min=1 << 30):            # the same batch on the small (one-DMA) path
        b2, s2 = engine.verify_batch(pk, sig, arena, offs, lens)
    assert np.array_equal(b2, bitmap) and np.array_equal(s2, status)


def test_device_api_streams_take_separate_slots(engine):
    """Device-API calls on four streams (more streams than workspace slots), several rounds, interleaved
    with a pipelined host-buffer call that uses every slot on its own streams: each bitmap is exact
    (honest batch all ones; the others their corruption patterns)."""
    n = 200_000
    batches = [workload.make_batch(engine, 0, n, 32, seed=1200 + k) for k in range(4)]
    expects = [torch.ones(n, dtype=torch.bool, device=DEV)] + [workload.corrupt_fraction(batches[k], k + 2)
                                                               for k in range(1, 4)]
    streams = [torch.cuda.Stream(DEV) for _ in range(4)]
    bms = [torch.zeros((n + 63) // 64, dtype=torch.int64, device=DEV) for _ in range(4)]
    hb = workload.make_batch(engine, 0, 300_000, 64, seed=1299)
    hexp = workload.corrupt_fraction(hb, 5).cpu().numpy()
    hpk, hsig, harena, hoff, hln = hb.to_host()
    torch.cuda.synchronize()
    for r in range(3):
        for k in range(4):
            b = batches[k]
            engine.verify_device(0, n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                                 b.len.data_ptr(), bms[k].data_ptr(), 0, streams[k].cuda_stream)
            if r == 1 and k == 1:
                hbm, _ = engine.verify_batch(hpk, hsig, harena, hoff, hln, want_status=False)
                assert np.array_equal(_bits(hbm, hb.n), hexp)
    torch.cuda.synchronize()
    for k in range(4):
        assert torch.equal(torch.from_numpy(_bits(bms[k].cpu().numpy().view(np.uint64), n)).to(DEV), expects[k])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_one_rank_gather_and_sharded_notary(engine, corpus):
    """the commit-step collective on the GPU.  A 1-rank "nccl" process group (RCCL) on
    cuda:0: gather_bitmaps of device tensors returns the local bitmaps, and BatchingNotary(group=pg) on a
    mixed batch (golden rejected records, a double spend, missing signers, a bad signature) decides
    exactly what the same notary without a group decides.  librccl must be mapped into the process."""
    import torch.distributed as dist
    from corda_amd import distributed as D
    from corda_amd.notary import BatchingNotary, SignRequest
    from corda_amd.crypto import DigitalSignature, EdDSAPublicKey
    from corda_amd.transactions import SignedTransaction
    import test_gpu_mirror as M

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        pg = dist.group.WORLD
        n = 1000
        rng = np.random.default_rng(5)
        local = torch.from_numpy(rng.integers(-2**62, 2**62, (2, D.shard_words(n, 1)), dtype=np.int64)).to(DEV)
        glob = D.gather_bitmaps(local, n, pg)
        torch.cuda.synchronize()
        assert torch.equal(glob, local[:, : (n + 63) // 64])
        with open("/proc/self/maps") as f:
            assert "rccl" in f.read(), "librccl is not mapped: the collective did not go through RCCL"

        seed = bytes(range(1, 33))
        reqs = []
        for i in range(6):
            reqs.append(SignRequest(M.make_stx(engine, signer_idx=[130 + i], inputs=(b"rccl-state-%d" % i,)),
                                    caller=f"p{i}"))
        reqs.append(SignRequest(M.make_stx(engine, signer_idx=[140], inputs=(b"rccl-state-0",)), caller="double"))
        reqs.append(SignRequest(M.make_stx(engine, signer_idx=[141], must_idx=[141, 142], inputs=(b"r-141",)),
                                caller="missing"))
        bad = M.make_stx(engine, signer_idx=[143], inputs=(b"r-143",))
        reqs.append(SignRequest(SignedTransaction(bad._wtx, [DigitalSignature.WithKey(bad.sigs[0].by, b"\x05" * 64)],
                                                  bad.id), caller="badsig"))
        rej = np.nonzero(corpus["verdict"] == 0)[0][:5]
        for j, i in enumerate(rej):                  # golden rejected records as a transaction's signature
            st = M.make_stx(engine, signer_idx=[150 + j], inputs=(b"r-gold-%d" % j,))
            key = EdDSAPublicKey(corpus["pk"][i].tobytes())
            reqs.append(SignRequest(SignedTransaction(st._wtx, [DigitalSignature.WithKey(key, corpus["sig"][i].tobytes())],
                                                      st.id), caller=f"gold{j}"))
        got = BatchingNotary(seed, validating=True, engine=engine, group=pg).notarise(reqs)
        want = BatchingNotary(seed, validating=True, engine=engine).notarise(reqs)
        assert [r.ok for r in got] == [r.ok for r in want]
        assert sum(r.ok for r in got) == 6
        for g, w in zip(got, want):
            assert type(g.error) is type(w.error) and type(g.failure) is type(w.failure)
            if g.ok:
                assert g.sig.bits == w.sig.bits
    finally:
        dist.destroy_process_group()


def test_host_pipeline_pinned_inputs_direct_dma(engine, corpus):
    """Inputs in pinned host memory (cv_host_alloc): the pipelined path DMAs every sub-chunk straight
    out of the caller's arrays (no packing) — same verdicts and status as the pageable call on a
    ragged 600,037-signature batch with corrupted S / R bytes and golden not-a-point keys, and the
    direct path was really taken (cv_diag_stats CV_STATS_PIPE)."""
    n = 600_037
    b = workload.make_batch(engine, 0, n, 300, seed=4242)
    expect = workload.corrupt_fraction(b, 16)
    idx = torch.arange(7, n, 89, device=DEV)
    b.sig[idx, 5] ^= 0x10
    expect[idx] = False
    pk, sig, arena, off, ln = b.to_host()
    del b
    pk = pk.copy()
    bad = _bad_key_records(corpus)
    kidx = np.arange(3, n, 997)
    pk[kidx] = corpus["pk"][bad[kidx % len(bad)]]
    exp = expect.cpu().numpy()
    exp[kidx] = False
    page_bm, page_st = engine.verify_batch(pk, sig, arena, off, ln)
    pinned = [engine.host_copy(x) for x in (pk, sig, arena, off, ln)]
    engine.stats("pipe", reset=True)
    pin_bm, pin_st = engine.verify_batch(*pinned)
    assert engine.stats("pipe")["direct_subchunks"] > 0, "pinned inputs did not take the direct-DMA path"
    assert np.array_equal(_bits(pin_bm, n), exp)
    assert np.array_equal(pin_bm, page_bm) and np.array_equal(pin_st, page_st)
    assert int(pin_st.sum()) == kidx.size


@pytest.mark.parametrize("n", [1, 63, 4096, 9001])
def test_host_small_pinned_inputs_golden(engine, corpus, n):
    """The small (notary-sized) host path with pinned inputs (DMAed in place): the golden corpus
    tiled to n records in random order gives the pinned corpus verdicts and status bytes."""
    rng = np.random.default_rng(n)
    sel = rng.integers(0, len(corpus["pk"]), n)
    arr = [engine.host_copy(x) for x in (corpus["pk"][sel], corpus["sig"][sel], corpus["arena"],
                                         corpus["off"][sel], corpus["len"][sel])]
    with _opts(engine, small_direct_min=1, small_zero_copy=0):   # the direct DMAs at every size
        bitmap, status = engine.verify_batch(*arr)
    assert np.array_equal(_bits(bitmap, n), corpus["verdict"][sel].astype(bool))
    assert np.array_equal(status, corpus["status"][sel])
    assert int(bitmap[-1]) >> (n % 64) == 0 if n % 64 else True


@pytest.mark.parametrize("n", [1, 3, 4, 63, 64, 65, 1000, 4096])
def test_host_small_zero_copy_golden(engine, corpus, n):
    """The zero-copy notary path (tri-form batches: the prep kernel reads the packed records from pinned
    host memory over PCIe — or a gather kernel moves them to device memory first, form 2 — and the
    kernels store one verdict byte per wave and the status bytes into pinned host memory) against the DMA form and the golden verdicts/status: the golden corpus tiled to n
    records in random order, pageable and pinned inputs, ragged ends (n % 4, n % 64)."""
    rng = np.random.default_rng(1000 + n)
    sel = rng.integers(0, len(corpus["pk"]), n)
    arr = (corpus["pk"][sel], corpus["sig"][sel], corpus["arena"], corpus["off"][sel], corpus["len"][sel])
    out = {}
    for zc in (0, 1, 2):
        with _opts(engine, small_zero_copy=zc):
            out[zc] = engine.verify_batch(*arr)
            out[zc, "pinned"] = engine.verify_batch(*[engine.host_copy(x) for x in arr])
            out[zc, "nostatus"] = engine.verify_batch(*arr, want_status=False)
    exp = corpus["verdict"][sel].astype(bool)
    for k, (bitmap, status) in out.items():
        assert np.array_equal(_bits(bitmap, n), exp), k
        assert int(bitmap[-1]) >> (n % 64) == 0 if n % 64 else True
        if status is not None:
            assert np.array_equal(status, corpus["status"][sel]), k
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][0], out[2][0])


def test_async_calls_in_flight_match_sync(engine, corpus, oracle_c):
    """cv_ed25519_verify_batch_async: three batches in flight (pageable 300,007 with corrupted S bytes,
    pinned 262,145 with corrupted R bytes and golden not-a-point keys, a 4,096 golden tile) — waited
    out of order: each equals its synchronous cv_ed25519_verify_batch (verdicts and status), and the
    pinned and golden ones their expected patterns."""
    n1, n2, n3 = 300_007, 262_145, 4096
    b1 = workload.make_batch(engine, 0, n1, 300, seed=71)
    e1 = workload.corrupt_fraction(b1, 13).cpu().numpy()
    a1 = b1.to_host()
    b2 = workload.make_batch(engine, 0, n2, 32, seed=72)
    idx = torch.arange(1, n2, 37, device=DEV)
    b2.sig[idx, 2] ^= 0x08
    e2 = torch.ones(n2, dtype=torch.bool, device=DEV)
    e2[idx] = False
    e2 = e2.cpu().numpy()
    pk2, sig2, ar2, off2, ln2 = b2.to_host()
    pk2 = pk2.copy()
    bad = _bad_key_records(corpus)
    kidx = np.arange(5, n2, 1013)
    pk2[kidx] = corpus["pk"][bad[kidx % len(bad)]]
    e2[kidx] = False
    a2 = tuple(engine.host_copy(x) for x in (pk2, sig2, ar2, off2, ln2))
    del b1, b2
    rng = np.random.default_rng(9)
    sel = rng.integers(0, len(corpus["pk"]), n3)
    a3 = (corpus["pk"][sel], corpus["sig"][sel], corpus["arena"], corpus["off"][sel], corpus["len"][sel])
    t1 = engine.verify_batch_async(*a1)
    t2 = engine.verify_batch_async(*a2)
    t3 = engine.verify_batch_async(*a3)
    r3 = engine.wait(t3)
    r1 = engine.wait(t1)
    r2 = engine.wait(t2)
    s1, s2, s3 = engine.verify_batch(*a1), engine.verify_batch(*a2), engine.verify_batch(*a3)
    for r, s_ in ((r1, s1), (r2, s2), (r3, s3)):
        assert np.array_equal(r[0], s_[0]) and np.array_equal(r[1], s_[1])
    assert np.array_equal(_bits(r1[0], n1), e1)
    assert np.array_equal(_bits(r2[0], n2), e2) and int(r2[1].sum()) == kidx.size
    assert np.array_equal(_bits(r3[0], n3), corpus["verdict"][sel].astype(bool))
    assert np.array_equal(r3[1], corpus["status"][sel])


@pytest.mark.parametrize("n", [100, 9001, 65536, 200_000])
def test_verify_batch_ex_arena_bound(engine, corpus, n):
    """cv_ed25519_verify_batch_ex: a record reaching past arena_bytes is rejected (CV_E_ARGS) by the engine's
    staging scan, in the small, zero-copy, mid-size (keys and signatures already in DMA when the scan finds it)
    and pipelined forms and in the async form, and nothing is read past the bound; the same batch with the true
    size verifies exactly (golden tiles)."""
    lib = native.load()
    idx = np.arange(n) % len(corpus["pk"])
    pk, sig = np.ascontiguousarray(corpus["pk"][idx]), np.ascontiguousarray(corpus["sig"][idx])
    arena, off, ln = corpus["arena"], np.ascontiguousarray(corpus["off"][idx]), np.ascontiguousarray(corpus["len"][idx])
    extent = int((off + ln.astype(np.uint64)).max())
    p = native._p
    for async_ in (False, True):
        bm = np.zeros((n + 63) // 64, np.uint64)
        t = ctypes.c_uint64()
        rc = lib.cv_ed25519_verify_batch_ex(engine._h, n, p(pk), p(sig), p(arena), extent - 1, p(off), p(ln), p(bm),
                                            None, ctypes.byref(t) if async_ else None)
        assert rc == -3, (async_, rc)
        rc = lib.cv_ed25519_verify_batch_ex(engine._h, n, p(pk), p(sig), p(arena), extent, p(off), p(ln), p(bm),
                                            None, ctypes.byref(t) if async_ else None)
        assert rc == 0
        if async_:
            assert lib.cv_wait(engine._h, t.value) == 0
        assert np.array_equal(_bits(bm, n), corpus["verdict"][idx].astype(bool))
    with pytest.raises(ValueError, match="exceeds the arena"):
        engine.verify_batch(pk, sig, arena[:extent - 1], off, ln)


@pytest.mark.parametrize("n", [100, 9001, 65536, 200_000])
def test_arena_bound_scattered_and_wrapping(engine, corpus, n):
    """the arena bound is checked on the records' true extent, not on the staged range.  A
    scattered batch (the staging compacts it: its byte range is far above twice its bytes) verifies exactly; the
    same batch with its LAST record pointing a long way past the arena — the compacted stage's range is only the
    sum of the lengths, so a check on it would pass and the packing would read past the arena — is rejected with
    CV_E_ARGS, as is a record whose off + len wraps past 2^64, with and without a bound (small, zero-copy, mid-size
    and pipelined forms: n = 100, 9,001, 65,536, 200,000), and the Python binding raises ValueError for both."""
    lib = native.load()
    p = native._p
    idx = np.arange(n) % len(corpus["pk"])
    pk, sig = np.ascontiguousarray(corpus["pk"][idx]), np.ascontiguousarray(corpus["sig"][idx])
    off = np.ascontiguousarray(corpus["off"][idx]).astype(np.uint64)
    ln = np.ascontiguousarray(corpus["len"][idx])
    A = corpus["arena"].size
    gap = (2 * int(ln.astype(np.uint64).sum()) + (4 << 20) + 15) // 16 * 16
    big = np.zeros(A + gap + A, np.uint8)                 # the corpus arena twice, `gap` bytes apart
    big[:A] = corpus["arena"]
    big[A + gap:] = corpus["arena"]
    off_s = off.copy()
    off_s[1::2] += np.uint64(A + gap)                     # odd records read the far copy: a scattered stage
    bm = np.zeros((n + 63) // 64, np.uint64)
    rc = lib.cv_ed25519_verify_batch_ex(engine._h, n, p(pk), p(sig), p(big), big.size, p(off_s), p(ln), p(bm), None,
                                        None)
    assert rc == 0
    assert np.array_equal(_bits(bm, n), corpus["verdict"][idx].astype(bool))
    bad = off_s.copy()
    bad[-1] = np.uint64(big.size + gap)                   # a record far past the arena, in the last (sub-)chunk
    rc = lib.cv_ed25519_verify_batch_ex(engine._h, n, p(pk), p(sig), p(big), big.size, p(bad), p(ln), p(bm), None, None)
    assert rc == -3
    with pytest.raises(ValueError, match="exceeds the arena"):
        engine.verify_batch(pk, sig, big, bad, ln)
    wrap = off_s.copy()
    wrap[-1] = np.uint64(2 ** 64 - 8)
    lw = ln.copy()
    lw[-1] = 32                                           # off + len wraps to 24
    for bound in (big.size, 2 ** 64 - 1):
        rc = lib.cv_ed25519_verify_batch_ex(engine._h, n, p(pk), p(sig), p(big), bound, p(wrap), p(lw), p(bm), None,
                                            None)
        assert rc == -3, bound
    assert lib.cv_ed25519_verify_batch(engine._h, n, p(pk), p(sig), p(big), p(wrap), p(lw), p(bm), None) == -3
    with pytest.raises(ValueError, match="exceeds the arena"):
        engine.verify_batch(pk, sig, big, wrap, lw)
    # the engine is still usable and exact after the rejected calls
    rc = lib.cv_ed25519_verify_batch_ex(engine._h, n, p(pk), p(sig), p(big), big.size, p(off_s), p(ln), p(bm), None,
                                        None)
    assert rc == 0 and np.array_equal(_bits(bm, n), corpus["verdict"][idx].astype(bool))


def test_merkle_wrapping_leaf_rejected(engine, merkle_cases):
    """A leaf whose off + len wraps past 2^64 is rejected by the Merkle entry points (CV_E_ARGS), small and
    pipelined forms, instead of being gathered from a wrapped address."""
    lib = native.load()
    p = native._p
    m = merkle_cases
    arena, off, ln = m["arena"], m["leaf_off"].astype(np.uint64), m["leaf_len"]
    txb = np.ascontiguousarray(m["tx_leaf_begin"], dtype=np.uint32)
    ntx = txb.size - 1
    ids = np.zeros((ntx, 32), np.uint8)
    st = np.zeros(ntx, np.uint8)
    w = off.copy()
    k = int(txb[-1]) - 1
    w[k] = np.uint64(2 ** 64 - 4)
    lw = ln.copy()
    lw[k] = 64
    assert lib.cv_merkle_tx_ids_ex(engine._h, ntx, p(arena), p(w), p(lw), p(txb), p(ids), p(st)) == -3
    t = ctypes.c_uint64()
    assert lib.cv_merkle_tx_ids_async(engine._h, ntx, p(arena), p(w), p(lw), p(txb), p(ids), p(st),
                                      ctypes.byref(t)) == -3
    assert lib.cv_merkle_tx_ids_ex(engine._h, ntx, p(arena), p(off), p(ln), p(txb), p(ids), p(st)) == 0


@pytest.mark.parametrize("n,overlap_min", [(1000, 64), (16384, 16384), (32768, 32768), (65536, 32768)])
def test_notary_midsize_forms_golden_and_oracle(engine, corpus, oracle_c, n, overlap_min):
    """Notary batches from the tri form to the mid sizes (16,384 and 32,768: quad form; 65,536: throughput form),
    unpipelined host path, with the prep overlap (point decodes on the slot's helper stream once keys and
    signatures are resident, beside the rest of the DMA and the scalars: CV_OPT_PREP_OVERLAP_MIN) and without it,
    from pageable and pinned inputs: a golden tile (1/16 of the records drawn from the corpus's rejected classes)
    gives the pinned verdicts and status bytes, and a corrupted random batch the C oracle's; pageable inputs both
    packed and DMAed in pieces (CV_OPT_MID_PIECES, default) and in one DMA per part."""
    rng = np.random.default_rng(n + 101)
    rej = np.where(corpus["verdict"] == 0)[0]
    acc = np.where(corpus["verdict"] == 1)[0]
    sel = rng.choice(acc, n)
    bad = rng.random(n) < 1 / 16
    sel[bad] = rng.choice(rej, int(bad.sum()))
    gold = (corpus["pk"][sel], corpus["sig"][sel], corpus["arena"], corpus["off"][sel], corpus["len"][sel])
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    arena = rng.integers(0, 256, n * 32 + 16, dtype=np.uint8)
    off = np.arange(n, dtype=np.uint64) * 32
    ln = np.full(n, 32, np.uint32)
    pk, sig = engine.sign_batch(seeds, arena, off, ln)
    sig[1::5, 35] ^= 4
    sig[3::11, 63] |= 0x20                      # S >= 2^253 on some records
    pk[2::7, 3] ^= 0x40
    rand = (pk, sig, arena, off, ln)
    ref, rst = oracle_c.verify_batch(pk, sig, arena, off, ln, nthreads=8)
    for om, pieces in ((1 << 40, 4), (overlap_min, 4), (overlap_min, 1)):
        with _opts(engine, prep_overlap_min=om, small_zero_copy=0, mid_pieces=pieces):
            for arrs, ev, es in ((gold, corpus["verdict"][sel], corpus["status"][sel]), (rand, ref, rst)):
                for pinned in (False, True):
                    if pinned and pieces == 1:
                        continue                    # (pieces apply to pageable inputs only)
                    a = [engine.host_copy(x) for x in arrs] if pinned else arrs
                    bitmap, status = engine.verify_batch(*a)
                    assert np.array_equal(_bits(bitmap, n), ev.astype(bool)), (om, pinned, pieces)
                    assert np.array_equal(status, es), (om, pinned, pieces)
                    if n % 64:
                        assert int(bitmap[-1]) >> (n % 64) == 0


def test_sync_call_timeline_diagnostics(engine):
    """CV_OPT_TIMELINE: a synchronous pipelined call timed on the GPU (events per sub-chunk) keeps its verdicts
    exact and reports a consistent timeline: 0 <= ramp <= span, busy + idle = span - ramp, tail = span - last DMA
    end, the first sub-chunk the plan's; off again, nothing more is recorded."""
    n = 300_000
    b = workload.make_batch(engine, 0, n, 300, seed=77)
    expect = workload.corrupt_fraction(b, 11).cpu().numpy()
    a = tuple(engine.host_copy(x) for x in b.to_host())
    del b
    engine.set_option("timeline", 1)
    try:
        engine.stats("timeline", reset=True)
        for _ in range(2):
            bm, _ = engine.verify_batch(*a, want_status=False)
            assert np.array_equal(_bits(bm, n), expect)
        t = engine.stats("timeline", reset=True)
    finally:
        engine.set_option("timeline", 0)
    assert t["calls"] == 2
    c = t["calls"]
    ramp, span, busy, idle = t["ramp_ms"] / c, t["span_ms"] / c, t["busy_ms"] / c, t["idle_ms"] / c
    assert 0 <= ramp <= span and busy > 0 and idle >= -1e-3
    assert abs(busy + idle - (span - ramp)) < 1e-3
    assert abs(t["tail_ms"] / c - (span - t["dma_end_ms"] / c)) < 1e-3
    assert t["result_copy_ms"] >= 0 and t["first_subchunk"] / c == engine.get_option("pipe_first")
    engine.verify_batch(*a, want_status=False)
    assert engine.stats("timeline")["calls"] == 0
