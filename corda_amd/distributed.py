"""Multi-GPU sharding of a signature batch: one process per GPU, RCCL all-gather of verdict bitmaps.

Signatures are independent, so a batch of n signatures is cut into contiguous per-rank ranges whose
starts are multiples of 64 (each rank owns whole uint64 bitmap words).  Every rank verifies its
shard with no data-path communication; the only collective is one all-gather of the per-rank
bitmaps into the replicated global bitmap the notary commit step consumes.
With torch's "nccl" backend that all-gather is RCCL over xGMI; the same code runs on "gloo" for
the CPU tests.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """[begin, end) of rank's shard: contiguous, begin a multiple of 64, all but the last equal."""
    words = (n + 63) // 64
    per_words = (words + world - 1) // world
    b = min(n, rank * per_words * 64)
    e = min(n, (rank + 1) * per_words * 64)
    return b, e


def shard_words(n: int, world: int) -> int:
    """bitmap words per rank (the all-gather is uniform, the last shard is zero-padded)"""
    words = (n + 63) // 64
    return (words + world - 1) // world


def gather_bitmap(local_words: torch.Tensor, n: int, group=None) -> torch.Tensor:
    """All-gather each rank's shard bitmap (int64 words, length shard_words(n, world)) and return the
    global bitmap of ceil(n/64) words, identical on every rank."""
    world = dist.get_world_size(group)
    per = shard_words(n, world)
    if local_words.numel() != per:
        raise ValueError(f"local bitmap has {local_words.numel()} words, expected {per}")
    out = torch.empty(per * world, dtype=local_words.dtype, device=local_words.device)
    dist.all_gather_into_tensor(out, local_words.contiguous(), group=group)
    return out[: (n + 63) // 64]


def gather_bitmaps(local: torch.Tensor, n: int, group=None) -> torch.Tensor:
    """gather_bitmap for k bitmaps at once (local: (k, shard_words) int64 — e.g. verdict bits and
    key-status bits): ONE all-gather, returns (k, ceil(n/64)) global bitmaps on every rank."""
    world = dist.get_world_size(group)
    per = shard_words(n, world)
    k = local.shape[0]
    if local.shape != (k, per):
        raise ValueError(f"local bitmaps have shape {tuple(local.shape)}, expected ({k}, {per})")
    out = torch.empty(world * k * per, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local.contiguous().view(-1), group=group)
    return out.view(world, k, per).permute(1, 0, 2).reshape(k, world * per)[:, : (n + 63) // 64]


def tx_verdicts_torch(bitmap: torch.Tensor, tx_sig_begin: torch.Tensor) -> torch.Tensor:
    """Per-transaction AND of signature bits on whatever device the bitmap lives on (the commit step):
    tx t is ok iff it has at least one signature and all of [begin_t, begin_{t+1}) are set."""
    n = int(tx_sig_begin[-1])
    words = bitmap.to(torch.int64)
    bit_idx = torch.arange(n, device=bitmap.device)
    bits = (words[bit_idx >> 6] >> (bit_idx & 63)) & 1
    csum = torch.zeros(n + 1, dtype=torch.int64, device=bitmap.device)
    csum[1:] = torch.cumsum(bits, 0)
    b = tx_sig_begin[:-1].to(torch.int64)
    e = tx_sig_begin[1:].to(torch.int64)
    ok = (csum[e] - csum[b]) == (e - b)
    return ok & (e > b)
