"""Multi-rank path on CPU (gloo, world_size 2 and 3): shard ranges, bitmap all-gather, per-tx AND.

Each rank's shard verdicts come from the C oracle (test infrastructure) standing in for its GPU;
what is under test is the sharding/all-gather/commit logic the bench and the notary use.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from corda_amd import distributed as D

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pack(bits: np.ndarray) -> np.ndarray:
    pad = (-len(bits)) % 64
    b = np.concatenate([bits.astype(np.uint8), np.zeros(pad, np.uint8)])
    return np.packbits(b, bitorder="little").view("<u8").astype(np.uint64)


def _worker(rank, world, port, n, q):
    import sys
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import cv_oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = np.load(os.path.join(REPO, "tests", "golden", "ed25519_corpus.npz"))
    idx = np.arange(n) % len(z["pk"])
    b, e = D.shard_range(n, world, rank)
    v, _ = cv_oracle.verify_batch(z["pk"][idx[b:e]], z["sig"][idx[b:e]], z["arena"], z["off"][idx[b:e]],
                                  z["len"][idx[b:e]], nthreads=2)
    per = D.shard_words(n, world)
    local = np.zeros(per, np.uint64)
    words = _pack(v)
    local[: words.size] = words
    glob = D.gather_bitmap(torch.from_numpy(local.view(np.int64)), n)
    begin = torch.tensor(np.arange(0, n + 1, 7).tolist() + ([n] if n % 7 else []), dtype=torch.int64)
    txok = D.tx_verdicts_torch(glob, begin)
    q.put((rank, glob.numpy().view(np.uint64).copy(), txok.numpy().copy(), begin.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 699), (2, 1280), (3, 1000)])
def test_sharded_bitmap_allgather(world, n, corpus, oracle_c):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    idx = np.arange(n) % len(corpus["pk"])
    full, _ = oracle_c.verify_batch(corpus["pk"][idx], corpus["sig"][idx], corpus["arena"], corpus["off"][idx],
                                    corpus["len"][idx], nthreads=4)
    expect = _pack(full)
    for rank, glob, txok, begin in res:
        assert np.array_equal(glob, expect), f"rank {rank} gathered bitmap differs"
        for t in range(len(begin) - 1):
            assert bool(txok[t]) == bool(full[begin[t]:begin[t + 1]].all() and begin[t + 1] > begin[t])


def test_shard_ranges_cover_exactly():
    for n in [0, 1, 63, 64, 65, 1000, 64 * 1000 + 5]:
        for world in [1, 2, 3, 8]:
            prev = 0
            for r in range(world):
                b, e = D.shard_range(n, world, r)
                assert b == prev and b % 64 == 0 or b == n
                assert e >= b
                prev = e
            assert prev == n


def test_tx_verdicts_torch_matches_host_abi():
    from corda_amd import native
    rng = np.random.default_rng(0)
    bits = rng.random(1000) > 0.05
    bm = _pack(bits)
    begin = np.concatenate([[0], np.sort(rng.choice(np.arange(1, 1000), 150, replace=False)), [1000, 1000]])
    a = native.tx_verdicts(bm, begin.astype(np.uint32)).astype(bool)
    b = D.tx_verdicts_torch(torch.from_numpy(bm.view(np.int64)), torch.from_numpy(begin.astype(np.int64))).numpy()
    assert np.array_equal(a, b)
    assert not a[-1]            # empty signature list is not ok


# ---------------------------------------------------------------- sharded notary verification
class _FakeEngine:
    """Stands in for a rank's GPU engine on CPU (what is under test is the sharding and the bitmap
    all-gather, not the crypto): a signature 'verifies' iff its first byte is even, a key whose
    first byte is 0xEE 'is not a point'."""

    def verify_batch(self, pk, sig, arena, off, ln, want_status=True):
        from corda_amd import native
        bad_key = pk[:, 0] == 0xEE
        ok = (sig[:, 0] % 2 == 0) & ~bad_key
        return _pack(ok), np.where(bad_key, native.CV_SIG_BAD_KEY, 0).astype(np.uint8)


def _items(n):
    from corda_amd.crypto import EdDSAPublicKey, NullPublicKey, VerifyItem
    rng = np.random.default_rng(n)
    out = []
    for i in range(n):
        key = rng.integers(0, 256, 32, dtype=np.uint8)
        if i % 13 == 0:
            key[0] = 0xEE
        k = NullPublicKey if i % 29 == 0 else EdDSAPublicKey(key.tobytes())
        sig = rng.integers(0, 256, 63 if i % 31 == 0 else 64, dtype=np.uint8).tobytes()
        out.append(VerifyItem(k, rng.integers(0, 256, int(rng.integers(0, 80)), dtype=np.uint8).tobytes(), sig))
    return out


def _notary_worker(rank, world, port, n, q):
    from corda_amd.notary import verify_many_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    errs = verify_many_sharded(_items(n), _FakeEngine())
    q.put((rank, [(type(e).__name__, str(e)) if e is not None else None for e in errs]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 700), (3, 129)])
def test_notary_sharded_verify_matches_single_process(world, n):
    """BatchingNotary(group=...) verification: each rank verifies its 64-aligned slice, ONE
    all-gather of the verdict and key-status bitmaps, and every rank rebuilds exactly the per-item
    exceptions the single-process verify_many returns (prefilter, bad key, mismatch)."""
    from corda_amd.crypto import verify_many
    expect = [(type(e).__name__, str(e)) if e is not None else None for e in verify_many(_items(n), _FakeEngine())]
    assert any(x and x[0] == "InvalidKeyException" for x in expect) and any(x is None for x in expect)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_notary_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got in res:
        assert got == expect, f"rank {rank} differs"


def test_gather_bitmaps_single_rank():
    """gather_bitmaps layout on a 1-rank gloo group: (k, words) in, the same (k, ceil(n/64)) out."""
    port = _free_port()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        x = torch.arange(6, dtype=torch.int64).view(2, 3)
        assert torch.equal(D.gather_bitmaps(x, 150), x)
    finally:
        dist.destroy_process_group()
