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
