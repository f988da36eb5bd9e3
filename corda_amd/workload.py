"""Synthetic, device-resident workloads of the BASELINE.json configurations.

Keys and signatures are produced on the GPU by the engine's own signer (cv_ed25519_sign_device,
deterministic RFC 8032), so a 1M-signature batch is ready in well under a second and never leaves
HBM.  Seeds and messages come from torch's seeded generators (reproducible per seed and rank).

  C2  1M single-signer signatures, 300-byte messages, distinct key per signature (key_pool=None) or a
      1,024-key pool
  C4  notary batches of 2^k signatures over 32-byte tx ids with 1/16 adversarial items
  C5  32-byte messages (tx ids), the per-GPU shard of the 64M-signature run
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import native


@dataclass
class SigBatch:
    n: int
    pk: torch.Tensor       # (n, 32) uint8, device
    sig: torch.Tensor      # (n, 64) uint8, device
    arena: torch.Tensor    # (n*msg_len + 16,) uint8, device
    off: torch.Tensor      # (n,) int64 (read as uint64), device
    len: torch.Tensor      # (n,) int32 (read as uint32), device
    msg_len: int
    key_index: Optional[torch.Tensor] = None   # (n,) int32: key of signature i (key-pool batches)
    nkeys: int = 0                             # distinct keys = pk[:nkeys] (key-pool batches)

    def to_host(self, lo: int = 0, hi: Optional[int] = None):
        hi = self.n if hi is None else hi
        pk = self.pk[lo:hi].cpu().numpy()
        sig = self.sig[lo:hi].cpu().numpy()
        a0, a1 = lo * self.msg_len, hi * self.msg_len
        arena = self.arena[a0:a1].cpu().numpy()
        off = (np.arange(hi - lo, dtype=np.uint64) * self.msg_len)
        ln = np.full(hi - lo, self.msg_len, np.uint32)
        return pk, sig, arena, off, ln


def make_batch(engine: native.Engine, device: int, n: int, msg_len: int, seed: int = 20261015,
               key_pool: Optional[int] = None, stream: int = 0) -> SigBatch:
    dev = torch.device("cuda", device)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    nkeys = n if key_pool is None else key_pool
    key_seeds = torch.randint(0, 256, (nkeys, 32), dtype=torch.uint8, device=dev, generator=g)
    if key_pool is not None:
        key_seeds = key_seeds[torch.arange(n, device=dev) % key_pool].contiguous()
    arena = torch.randint(0, 256, (n * msg_len + 16,), dtype=torch.uint8, device=dev, generator=g)
    off = torch.arange(n, dtype=torch.int64, device=dev) * msg_len
    ln = torch.full((n,), msg_len, dtype=torch.int32, device=dev)
    pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    engine.sign_device(device, n, key_seeds.data_ptr(), arena.data_ptr(), off.data_ptr(), ln.data_ptr(),
                       pk.data_ptr(), sig.data_ptr(), stream)
    engine.synchronize(device)
    torch.cuda.synchronize(dev)
    if key_pool is not None:
        kidx = (torch.arange(n, device=dev) % key_pool).to(torch.int32)
        return SigBatch(n, pk, sig, arena, off, ln, msg_len, kidx, min(key_pool, n))
    return SigBatch(n, pk, sig, arena, off, ln, msg_len)


def adversarial_records(corpus_path: str):
    """The golden corpus's REJECTED records with 32-byte (tx-id-shaped) messages: (pk, sig, msgs) —
    the §8(a) adversarial classes (non-canonical / off-curve / small-order R and A, S >= L, the slide
    carry loss, cofactored-only, wrong message or key) with verdicts pinned by the oracle."""
    z = np.load(corpus_path)
    rej = np.nonzero(z["verdict"] == 0)[0]
    keep = [i for i in rej if int(z["len"][i]) == 32]
    msgs = np.stack([z["arena"][int(z["off"][i]):int(z["off"][i]) + 32] for i in keep])
    return z["pk"][keep], z["sig"][keep], msgs


def notary_batch(engine: native.Engine, device: int, n: int, adversarial, key_pool: Optional[int] = None,
                 seed: int = 4096):
    """C4 notary batch on the host (as the notary's JVM shim hands it over): n signatures over 32-byte
    tx ids, 8 signers per transaction, every 16th record replaced by the next adversarial record
    (cycling through adversarial_records).  Returns (pk, sig, arena, off, len, expected verdicts)."""
    b = make_batch(engine, device, n, 32, seed=seed + n, key_pool=key_pool)
    pk, sig, arena, off, ln = b.to_host()
    pk, sig, arena = pk.copy(), sig.copy(), arena.copy()
    expect = np.ones(n, bool)
    apk, asig, amsg = adversarial
    for j, i in enumerate(range(0, n, 16)):
        a = j % len(apk)
        pk[i], sig[i] = apk[a], asig[a]
        arena[i * 32:(i + 1) * 32] = amsg[a]
        expect[i] = False
    return pk, sig, np.concatenate([arena, np.zeros(16, np.uint8)]), off, ln, expect


def corrupt_fraction(batch: SigBatch, every: int = 16) -> torch.Tensor:
    """Flip one bit of S in every `every`-th signature (the C4 "1/16 adversarial" mix); returns the
    expected verdicts (bool tensor on the device)."""
    idx = torch.arange(0, batch.n, every, device=batch.sig.device)
    batch.sig[idx, 40] ^= 1
    expect = torch.ones(batch.n, dtype=torch.bool, device=batch.sig.device)
    expect[idx] = False
    return expect


@dataclass
class TxBatch:
    """C3-shaped transactions: leaf blobs (6 per tx: 2x120, 2x600, 2x300 bytes +-25 %), the claimed
    ids (= Merkle roots, computed once on the GPU at generation time), and `signers` signatures per
    transaction over its 32-byte id (SignedTransaction.kt:85: sigs cover id.bytes)."""
    ntx: int
    signers: int
    leaf_arena: torch.Tensor
    leaf_off: torch.Tensor
    leaf_len: torch.Tensor
    tx_begin: torch.Tensor       # (ntx+1,) int32
    ids: torch.Tensor            # (ntx, 32) uint8 claimed ids
    sigs: SigBatch               # ntx*signers records; message i = ids[i // signers]
    sig_tx_begin: torch.Tensor   # (ntx+1,) int64


LEAF_SHAPE = (120, 120, 600, 600, 300, 300)


def make_tx_batch(engine: native.Engine, device: int, ntx: int, signers: int = 8, seed: int = 20261015,
                  stream: int = 0) -> TxBatch:
    dev = torch.device("cuda", device)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    nleaf = len(LEAF_SHAPE)
    base = torch.tensor(LEAF_SHAPE, dtype=torch.float32, device=dev).repeat(ntx)
    scale = torch.rand(ntx * nleaf, device=dev, generator=g) * 0.5 + 0.75
    leaf_len = (base * scale).to(torch.int32)
    leaf_off = torch.zeros(ntx * nleaf, dtype=torch.int64, device=dev)
    leaf_off[1:] = torch.cumsum(leaf_len[:-1].to(torch.int64), 0)
    total = int(leaf_off[-1] + leaf_len[-1])
    arena = torch.randint(0, 256, (total + 16,), dtype=torch.uint8, device=dev, generator=g)
    tx_begin = torch.arange(0, ntx * nleaf + 1, nleaf, dtype=torch.int32, device=dev)
    ids = torch.empty((ntx, 32), dtype=torch.uint8, device=dev)
    ws = torch.empty(ntx * nleaf * 32, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    engine.merkle_device(device, ntx, ntx * nleaf, arena.data_ptr(), leaf_off.data_ptr(), leaf_len.data_ptr(),
                         tx_begin.data_ptr(), ws.data_ptr(), ids.data_ptr(), 0, stream)
    engine.synchronize(device)
    torch.cuda.synchronize(dev)
    n = ntx * signers
    key_seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device=dev, generator=g)
    off = (torch.arange(n, dtype=torch.int64, device=dev) // signers) * 32
    ln = torch.full((n,), 32, dtype=torch.int32, device=dev)
    pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    id_arena = torch.cat([ids.reshape(-1), torch.zeros(16, dtype=torch.uint8, device=dev)])
    # the key seeds and id arena above are written on torch's stream; with stream = 0 the signing runs on the
    # engine's own stream, which does not wait for them (it read half-written seeds: ~45,000 of 1M transactions
    # signed with garbage keys when the GPU was busy)
    torch.cuda.synchronize(dev)
    engine.sign_device(device, n, key_seeds.data_ptr(), id_arena.data_ptr(), off.data_ptr(), ln.data_ptr(),
                       pk.data_ptr(), sig.data_ptr(), stream)
    engine.synchronize(device)
    torch.cuda.synchronize(dev)
    sb = SigBatch(n, pk, sig, id_arena, off, ln, 32)
    sig_tx_begin = torch.arange(0, n + 1, signers, dtype=torch.int64, device=dev)
    return TxBatch(ntx, signers, arena, leaf_off, leaf_len, tx_begin, ids, sb, sig_tx_begin)
