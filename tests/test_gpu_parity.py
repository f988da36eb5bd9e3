"""GPU parity tests: the HIP engine (through the C-ABI) against the oracle and the golden fixtures.

Bit-exact bar: every verdict, every key-status byte, every tx id.  Sizes: the golden corpus and
oracle-checked random batches at sizes the oracle finishes in seconds; BASELINE sizes (1M) through
size-independent properties (all honest accepted, an exact corruption pattern rejected).
"""
import ctypes
import hashlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from corda_amd import native  # noqa: E402


def _bits(bitmap, n):
    return native.bitmap_to_bools(bitmap, n)


def test_golden_corpus_verdicts(engine, corpus, manifest):
    bitmap, status = engine.verify_batch(corpus["pk"], corpus["sig"], corpus["arena"], corpus["off"], corpus["len"])
    got = _bits(bitmap, len(corpus["pk"]))
    exp = corpus["verdict"].astype(bool)
    bad = np.where(got != exp)[0]
    classes = manifest["classes"]
    assert bad.size == 0, f"mismatches in classes {sorted({classes[corpus['cls'][i]] for i in bad})}"
    assert np.array_equal(status, corpus["status"])


def test_golden_corpus_per_class_and_shuffled(engine, corpus, manifest):
    """Same corpus in a shuffled order, tiled 10x: verdicts must follow the records (no cross-lane leaks)."""
    n = len(corpus["pk"])
    rng = np.random.default_rng(1)
    perm = np.concatenate([rng.permutation(n) for _ in range(10)])
    bitmap, status = engine.verify_batch(corpus["pk"][perm], corpus["sig"][perm], corpus["arena"], corpus["off"][perm],
                                         corpus["len"][perm])
    assert np.array_equal(_bits(bitmap, perm.size), corpus["verdict"][perm].astype(bool))
    assert np.array_equal(status, corpus["status"][perm])


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 129, 255, 256, 257, 1000])
def test_ragged_sizes(engine, corpus, n):
    idx = np.arange(n) % len(corpus["pk"])
    bitmap, status = engine.verify_batch(corpus["pk"][idx], corpus["sig"][idx], corpus["arena"], corpus["off"][idx],
                                         corpus["len"][idx])
    assert bitmap.size == (n + 63) // 64
    assert np.array_equal(_bits(bitmap, n), corpus["verdict"][idx].astype(bool))
    # bits past n in the last word stay clear
    if n % 64:
        assert int(bitmap[-1]) >> (n % 64) == 0


def test_empty_batch(engine):
    bitmap, status = engine.verify_batch(np.zeros((0, 32), np.uint8), np.zeros((0, 64), np.uint8), np.zeros(0, np.uint8),
                                         np.zeros(0, np.uint64), np.zeros(0, np.uint32))
    assert bitmap.size == 0 and status.size == 0


def test_gpu_signer_matches_oracle(engine):
    import ed25519_ref as E
    rng = np.random.default_rng(7)
    n = 48
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    lens = rng.integers(0, 400, n).astype(np.uint32)
    lens[:4] = [0, 32, 300, 111]
    msgs = [rng.integers(0, 256, int(l), dtype=np.uint8).tobytes() for l in lens]
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1])
    arena = np.frombuffer(b"".join(msgs) + b"\0" * 16, np.uint8)
    pk, sig = engine.sign_batch(seeds, arena, off, lens)
    for i in range(n):
        s = seeds[i].tobytes()
        assert pk[i].tobytes() == E.public_key_of(s)
        assert sig[i].tobytes() == E.sign(s, msgs[i])
    # entropyToKeyPair seeds of the reference's test keys (DUMMY_NOTARY_KEY = 20, CASH_ISSUER = 10)
    for ent in (20, 10):
        s = np.frombuffer(E.entropy_to_seed(ent), np.uint8)[None]
        m = np.frombuffer(b"\x07" * 32, np.uint8)
        p2, s2 = engine.sign_batch(s, m, np.zeros(1, np.uint64), np.array([32], np.uint32))
        assert s2[0].tobytes() == E.sign(E.entropy_to_seed(ent), b"\x07" * 32)


def test_random_batch_vs_c_oracle(engine, oracle_c):
    rng = np.random.default_rng(11)
    n = 8192
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    lens = rng.integers(0, 320, n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1])
    arena = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
    pk, sig = engine.sign_batch(seeds, arena, off, lens)
    # corruptions of every kind at known positions
    sig[1::7, rng.integers(0, 64)] ^= 0x10
    pk[2::11, 3] ^= 0x01
    sig[3::13, 63] |= 0x80                     # S >= 2^255 (slide carry-loss territory)
    arena[off[5::17].astype(np.int64)] ^= 0xFF  # message byte (where len > 0)
    bitmap, status = engine.verify_batch(pk, sig, arena, off, lens)
    ref, rst = oracle_c.verify_batch(pk, sig, arena, off, lens, nthreads=8)
    assert np.array_equal(_bits(bitmap, n), ref.astype(bool))
    assert np.array_equal(status, rst)
    assert 0.5 < ref.mean() < 0.95


def test_baseline_size_all_honest_and_exact_pattern(engine):
    """C2 at full size (1M, 300-byte messages): every honest signature accepted, and after flipping
    one S bit in every 16th signature exactly those are rejected (size-independent properties)."""
    import torch
    from corda_amd import workload
    n = 1_000_000
    b = workload.make_batch(engine, 0, n, 300, seed=99)
    bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda:0")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    engine.verify_device(0, n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                         b.len.data_ptr(), bm.data_ptr(), st.data_ptr())
    engine.synchronize(0)
    got = native.bitmap_to_bools(bm.cpu().numpy().view(np.uint64), n)
    assert got.all()
    assert int(st.sum()) == 0
    expect = workload.corrupt_fraction(b, 16).cpu().numpy()
    engine.verify_device(0, n, b.pk.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(), b.off.data_ptr(),
                         b.len.data_ptr(), bm.data_ptr(), 0)
    engine.synchronize(0)
    got = native.bitmap_to_bools(bm.cpu().numpy().view(np.uint64), n)
    assert np.array_equal(got, expect)


def test_key_pool_batch(engine, oracle_c):
    """1,024-key pool variant (repeated keys across lanes; above 4,096 signatures the host dedupe
    sends it down the keyed comb path) with S, R, message and key corruptions vs the C oracle."""
    from corda_amd import workload
    for n in (4096, 9000):
        b = workload.make_batch(engine, 0, n, 32, seed=5, key_pool=1024)
        pk, sig, arena, off, ln = b.to_host()
        assert len({bytes(r) for r in pk}) == 1024
        bitmap, _ = engine.verify_batch(pk, sig, arena, off, ln)
        assert _bits(bitmap, n).all()
        sig, arena, pk = sig.copy(), arena.copy(), pk.copy()
        sig[1::17, 50] ^= 0x04                          # S
        sig[2::19, 7] ^= 0x80                           # R
        arena[off[3::23].astype(np.int64) + 5] ^= 0x01  # message
        pk[5::29, 31] ^= 0x40                           # key (sign bit or y bit 254)
        bitmap, status = engine.verify_batch(pk, sig, arena, off, ln)
        ref, rst = oracle_c.verify_batch(pk, sig, arena, off, ln, nthreads=8)
        assert np.array_equal(_bits(bitmap, n), ref.astype(bool))
        assert np.array_equal(status, rst)
        assert 0 < int(ref.sum()) < n


def test_merkle_golden(engine, merkle_cases):
    m = merkle_cases
    ids, st = engine.merkle_tx_ids(m["arena"], m["leaf_off"], m["leaf_len"], m["tx_leaf_begin"])
    assert np.array_equal(st, m["status"])
    assert np.array_equal(ids, m["ids"])
    assert ids[0].tobytes().hex().upper() == "F6D8FB3720114F8D040D64F633B0D9178EB09A55AA7D62FAE1A070D1BF561051"


def test_merkle_sha256_multiblock_kat(engine):
    """One-leaf tx over the 71,644-byte prospectus jar: id = SHA-256(jar) = decd0986... (SellerFlow.kt:23)."""
    here = os.path.dirname(os.path.abspath(__file__))
    data = np.fromfile(os.path.join(here, "golden", "bank-of-london-cp.jar.bin"), np.uint8)
    ids, st = engine.merkle_tx_ids(data, np.zeros(1, np.uint64), np.array([data.size], np.uint32),
                                   np.array([0, 1], np.uint32))
    assert ids[0].tobytes().hex() == "decd098666b9657314870e192ced0c3519c2c9d395507a238338f8d003929de9"


def test_merkle_random_vs_oracle(engine, oracle_c):
    rng = np.random.default_rng(3)
    ntx = 3000
    counts = rng.integers(0, 12, ntx)
    counts[:5] = [0, 1, 2, 3, 64]
    begin = np.zeros(ntx + 1, np.uint32)
    begin[1:] = np.cumsum(counts)
    nl = int(begin[-1])
    lens = rng.integers(0, 700, nl).astype(np.uint32)
    # leaves past the leaf kernel's last length bucket (>= 63 SHA-256 blocks) mixed in: workgroups
    # order their leaves by block count, so every bucket and a ragged last workgroup must hash right
    lens[::97] = rng.integers(3900, 9000, lens[::97].size).astype(np.uint32)
    off = np.zeros(nl, np.uint64)
    off[1:] = np.cumsum(lens[:-1])
    arena = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
    ids, st = engine.merkle_tx_ids(arena, off, lens, begin)
    rids, rst = oracle_c.merkle_tx_ids(arena, off, lens, begin)
    assert np.array_equal(st, rst)
    assert np.array_equal(ids, rids)


def test_tx_verdicts_and():
    bitmap = np.array([0xFFFFFFFFFFFFFFF0, 0x1], np.uint64)
    begin = np.array([0, 4, 8, 64, 65, 65, 66], np.uint32)
    assert native.tx_verdicts(bitmap, begin).tolist() == [0, 1, 1, 1, 0, 0]


# ---------------------------------------------------------------- keyed path (per-key comb tables, f2)
def _dedupe(pk):
    keys, inv = np.unique(pk, axis=0, return_inverse=True)
    return keys, inv.reshape(-1).astype(np.uint32)


def test_keyed_golden_corpus(engine, corpus, manifest):
    """Every golden verdict and key status through the keyed path (torsion, mixed-order, invalid and
    non-canonical keys included), and again on a warm key pool (all hits)."""
    keys, kidx = _dedupe(corpus["pk"])
    for rep in range(2):
        before = engine.key_cache_stats(0)
        bitmap, status = engine.verify_batch_keyed(keys, kidx, corpus["sig"], corpus["arena"], corpus["off"],
                                                   corpus["len"])
        got = _bits(bitmap, len(kidx))
        bad = np.where(got != corpus["verdict"].astype(bool))[0]
        assert bad.size == 0, f"keyed mismatches in {sorted({manifest['classes'][corpus['cls'][i]] for i in bad})}"
        assert np.array_equal(status, corpus["status"])
        after = engine.key_cache_stats(0)
        if rep == 1:
            assert after["misses"] == before["misses"], "warm pool recomputed key tables"


def test_auto_keyed_path_matches_plain(engine, corpus):
    """cv_ed25519_verify_batch dedupes keys itself when they repeat (>= 2 signatures per key) in
    batches above the tri-chain size (4,096); smaller batches stay on the plain latency path."""
    small = np.tile(np.arange(len(corpus["pk"])), 4)[:4096]
    before = engine.key_cache_stats(0)
    bitmap, status = engine.verify_batch(corpus["pk"][small], corpus["sig"][small], corpus["arena"],
                                         corpus["off"][small], corpus["len"][small])
    assert np.array_equal(_bits(bitmap, small.size), corpus["verdict"][small].astype(bool))
    after = engine.key_cache_stats(0)
    assert after["hits"] + after["misses"] == before["hits"] + before["misses"], "keyed path taken at 4,096"
    idx = np.tile(np.arange(len(corpus["pk"])), 8)
    before = engine.key_cache_stats(0)
    bitmap, status = engine.verify_batch(corpus["pk"][idx], corpus["sig"][idx], corpus["arena"], corpus["off"][idx],
                                         corpus["len"][idx])
    assert np.array_equal(_bits(bitmap, idx.size), corpus["verdict"][idx].astype(bool))
    assert np.array_equal(status, corpus["status"][idx])
    after = engine.key_cache_stats(0)
    assert after["hits"] + after["misses"] > before["hits"] + before["misses"], "keyed path not taken"


def test_keyed_random_pool_vs_c_oracle(engine, oracle_c):
    rng = np.random.default_rng(21)
    n, pool = 6000, 37
    kseeds = rng.integers(0, 256, (pool, 32), dtype=np.uint8)
    kidx = rng.integers(0, pool, n).astype(np.uint32)
    lens = rng.integers(0, 200, n).astype(np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1])
    arena = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
    pk, sig = engine.sign_batch(kseeds[kidx], arena, off, lens)
    keys = pk[np.unique(kidx, return_index=True)[1]]
    keys_full = np.zeros((pool, 32), np.uint8)
    keys_full[np.unique(kidx)] = keys
    sig[1::5, 40] ^= 0x04
    sig[2::9, 63] |= 0x80
    sig[3::11, 5] ^= 0x01
    bitmap, status = engine.verify_batch_keyed(keys_full, kidx, sig, arena, off, lens)
    ref, rst = oracle_c.verify_batch(keys_full[kidx], sig, arena, off, lens, nthreads=8)
    assert np.array_equal(_bits(bitmap, n), ref.astype(bool))
    assert np.array_equal(status, rst)
    assert 0.4 < ref.mean() < 0.9


def test_keyed_pool_epoch_reset(engine, corpus):
    """A pool smaller than the working set is emptied and refilled between calls; verdicts stay exact."""
    from corda_amd import native
    e = native.Engine(1)
    try:
        e.key_cache_reserve(8)
        keys, kidx = _dedupe(corpus["pk"])
        for lo in range(0, len(kidx), 100):
            sl = slice(lo, lo + 100)
            bm, st = e.verify_batch_keyed(keys, kidx[sl], corpus["sig"][sl], corpus["arena"], corpus["off"][sl],
                                          corpus["len"][sl])
            assert np.array_equal(_bits(bm, len(kidx[sl])), corpus["verdict"][sl].astype(bool))
            assert np.array_equal(st, corpus["status"][sl])
    finally:
        e.close()


def test_keyed_device_baseline_size(engine):
    """C2 shape with a 1,024-key pool at full size on the keyed device path: all honest accepted, the
    1/16 corruption pattern exactly rejected."""
    import torch
    from corda_amd import workload
    n = 1_000_000
    b = workload.make_batch(engine, 0, n, 300, seed=77, key_pool=1024)
    bm = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda:0")
    args = (0, n, b.nkeys, b.pk.data_ptr(), b.key_index.data_ptr(), b.sig.data_ptr(), b.arena.data_ptr(),
            b.off.data_ptr(), b.len.data_ptr(), bm.data_ptr())
    engine.verify_device_keyed(*args, timed=True)
    assert native.bitmap_to_bools(bm.cpu().numpy().view(np.uint64), n).all()
    expect = workload.corrupt_fraction(b, 16).cpu().numpy()
    engine.verify_device_keyed(*args, timed=True)
    assert np.array_equal(native.bitmap_to_bools(bm.cpu().numpy().view(np.uint64), n), expect)


# ---------------------------------------------------------------- every kernel form at every size
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


@pytest.mark.parametrize("quad_max,tri_max", [(0, 0), (1 << 22, 0), (1 << 22, 1 << 20)])
def test_lane_quad_and_tri_forms_agree(engine, corpus, oracle_c, quad_max, tri_max):
    """Small batches normally run the 16-lanes-per-signature (tri-chain) or 4-lanes-per-signature
    (quad) Straus; force each form in turn (per-context options CV_OPT_QUAD_MAX / CV_OPT_TRI_MAX: (0, 0) =
    the throughput kernels at every size) over the golden corpus, keyed and plain, and a random batch."""
    with _opts(engine, quad_max=quad_max, tri_max=tri_max):
        bitmap, status = engine.verify_batch(corpus["pk"], corpus["sig"], corpus["arena"], corpus["off"], corpus["len"])
        assert np.array_equal(_bits(bitmap, len(corpus["pk"])), corpus["verdict"].astype(bool))
        assert np.array_equal(status, corpus["status"])
        keys, kidx = _dedupe(corpus["pk"])
        bitmap, status = engine.verify_batch_keyed(keys, kidx, corpus["sig"], corpus["arena"], corpus["off"],
                                                   corpus["len"])
        assert np.array_equal(_bits(bitmap, len(kidx)), corpus["verdict"].astype(bool))
        assert np.array_equal(status, corpus["status"])
        rng = np.random.default_rng(31)
        n = 3000
        seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        arena = rng.integers(0, 256, n * 32 + 16, dtype=np.uint8)
        off = np.arange(n, dtype=np.uint64) * 32
        ln = np.full(n, 32, np.uint32)
        pk, sig = engine.sign_batch(seeds, arena, off, ln)
        sig[::4, 33] ^= 2
        bitmap, _ = engine.verify_batch(pk, sig, arena, off, ln)
        ref, _ = oracle_c.verify_batch(pk, sig, arena, off, ln, nthreads=8)
        assert np.array_equal(_bits(bitmap, n), ref.astype(bool))


@pytest.mark.parametrize("n", [4096, 9001])
def test_latency_forms_corpus_and_oracle(engine, corpus, oracle_c, n):
    """The latency kernels at their default sizes (n = 4,096: tri chain, 9,001: quad): the golden corpus
    tiled to n records gives the pinned verdicts and statuses, and a corrupted random batch of n the C
    oracle's."""
    rng = np.random.default_rng(n + 7)
    sel = rng.integers(0, len(corpus["pk"]), n)
    bitmap, status = engine.verify_batch(corpus["pk"][sel], corpus["sig"][sel], corpus["arena"],
                                         corpus["off"][sel], corpus["len"][sel])
    assert np.array_equal(_bits(bitmap, n), corpus["verdict"][sel].astype(bool))
    assert np.array_equal(status, corpus["status"][sel])
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    arena = rng.integers(0, 256, n * 32 + 16, dtype=np.uint8)
    off = np.arange(n, dtype=np.uint64) * 32
    ln = np.full(n, 32, np.uint32)
    pk, sig = engine.sign_batch(seeds, arena, off, ln)
    sig[1::5, 35] ^= 4
    pk[2::7, 3] ^= 0x40
    bitmap, status = engine.verify_batch(pk, sig, arena, off, ln)
    ref, rst = oracle_c.verify_batch(pk, sig, arena, off, ln, nthreads=8)
    assert np.array_equal(_bits(bitmap, n), ref.astype(bool))
    assert np.array_equal(status, rst)


def test_throughput_form_small_and_ragged(engine, corpus, oracle_c):
    """The throughput kernels (scalars -> lane-pair points -> hs_straus with wave-ballot verdicts) forced onto
    small and ragged batches (CV_OPT_QUAD_MAX = 0): the golden corpus, ragged tails, and corrupted random
    batches (R, S, key, S >= 2^255, variable-length messages) against the C oracle."""
    with _opts(engine, quad_max=0):
        bitmap, status = engine.verify_batch(corpus["pk"], corpus["sig"], corpus["arena"], corpus["off"], corpus["len"])
        assert np.array_equal(_bits(bitmap, len(corpus["pk"])), corpus["verdict"].astype(bool))
        assert np.array_equal(status, corpus["status"])
        for n in (1, 63, 65, 257, 699, 1001):
            sel = np.arange(n) % len(corpus["pk"])
            bitmap, status = engine.verify_batch(corpus["pk"][sel], corpus["sig"][sel], corpus["arena"],
                                                 corpus["off"][sel], corpus["len"][sel])
            assert np.array_equal(_bits(bitmap, n), corpus["verdict"][sel].astype(bool))
            assert np.array_equal(status, corpus["status"][sel])
        rng = np.random.default_rng(41)
        n = 6000
        seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        lens = rng.integers(0, 200, n).astype(np.uint32)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(lens[:-1])
        arena = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
        pk, sig = engine.sign_batch(seeds, arena, off, lens)
        sig[1::7, rng.integers(0, 32)] ^= 0x04          # R corrupted (mostly off-curve / wrong point)
        sig[2::11, 31] |= 0x80                          # R sign bit forced
        sig[3::13, 63] |= 0x80                          # S >= 2^255
        sig[4::17, 40] ^= 0x01                          # S corrupted
        pk[5::19, 7] ^= 0x20                            # key corrupted
        pk[6::23, 5] ^= 0x10                            # key corrupted (often not a point)
        bitmap, status = engine.verify_batch(pk, sig, arena, off, lens)
        ref, rst = oracle_c.verify_batch(pk, sig, arena, off, lens, nthreads=8)
        assert np.array_equal(_bits(bitmap, n), ref.astype(bool))
        assert np.array_equal(status, rst)
        assert 0.4 < ref.mean() < 0.9


@pytest.mark.parametrize("mode,n", [(0, 200_003), (1, 200_003), (2, 200_003), (1, (1 << 22) + 200_003),
                                    (2, (1 << 22) + 200_003)])
def test_split_launch_plans_agree(engine, corpus, mode, n):
    """The drain-overlap sub-chunk plan (CV_OPT_DRAIN_SPLIT: 0 off, 1 auto, 2 always with a 25 % tail) over
    the golden corpus tiled to a ragged n through the device API — at 2^22 + 200,003 the batch is two
    workspace chunks and only the second one's last round is near-empty: every verdict and key-status byte
    follows its record, bits past n stay clear."""
    import torch
    rng = np.random.default_rng(7)
    idx = rng.integers(0, len(corpus["pk"]), n)
    dev = "cuda:0"
    pk = torch.from_numpy(np.ascontiguousarray(corpus["pk"][idx])).to(dev)
    sig = torch.from_numpy(np.ascontiguousarray(corpus["sig"][idx])).to(dev)
    arena = torch.from_numpy(np.concatenate([corpus["arena"], np.zeros(64, np.uint8)])).to(dev)
    off = torch.from_numpy(corpus["off"][idx].astype(np.uint64).view(np.int64)).to(dev)
    ln = torch.from_numpy(corpus["len"][idx].astype(np.uint32).view(np.int32)).to(dev)
    with _opts(engine, drain_split=mode, drain_split_pct=10 if mode == 1 else 25):
        bm = torch.full(((n + 63) // 64,), -1, dtype=torch.int64, device=dev)
        st = torch.full((n,), 7, dtype=torch.uint8, device=dev)
        engine.verify_device(0, n, pk.data_ptr(), sig.data_ptr(), arena.data_ptr(), off.data_ptr(), ln.data_ptr(),
                             bm.data_ptr(), st.data_ptr())
        engine.synchronize(0)
    bits = bm.cpu().numpy().view(np.uint64)
    assert np.array_equal(_bits(bits, n), corpus["verdict"][idx].astype(bool))
    assert np.array_equal(st.cpu().numpy(), corpus["status"][idx])
    assert int(bits[-1]) >> (n % 64) == 0


def test_host_buffer_api_split_size_exact_pattern(engine):
    """Host-buffer C-ABI (cv_ed25519_verify_batch: H2D, verify, D2H) at a size whose last Straus
    round is near-empty (200,003 distinct-key signatures over 300-byte messages): honest signatures
    accepted, every 16th (one S bit flipped) rejected, key status clear."""
    from corda_amd import workload
    n = 200_003
    b = workload.make_batch(engine, 0, n, 300, seed=123)
    expect = workload.corrupt_fraction(b, 16).cpu().numpy()
    pk, sig, arena, off, ln = b.to_host()
    bitmap, status = engine.verify_batch(pk, sig, arena, off, ln)
    assert np.array_equal(_bits(bitmap, n), expect)
    assert int(status.sum()) == 0
    assert int(bitmap[-1]) >> (n % 64) == 0
