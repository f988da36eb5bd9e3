"""Batched notary commit step on the GPU engine (BASELINE config C4 / SURVEY.md §8(a) a11).

The reference notarises one transaction per flow on the node's single thread:
  NotaryFlow.Service.call                core/src/main/kotlin/net/corda/flows/NotaryFlow.kt:96-113
    val wtx = stx.tx   (Merkle id recompute + check(temp.id == id), OUTSIDE the try: a mismatch is
                        an IllegalStateException that fails the flow, not a NotaryError)
    try { validateTimestamp -> beforeCommit -> commitInputStates -> sign(stx.id) }
    catch (NotaryException) -> Result.Error
  ValidatingNotaryFlow.beforeCommit      core/src/main/kotlin/net/corda/flows/ValidatingNotaryFlow.kt:24-52
    checkSignatures: stx.verifySignatures(notaryKey), SignaturesMissingException -> SignaturesMissing;
    SignatureException -> TransactionInvalid; anything else (IllegalStateException, InvalidKeyException)
    is re-thrown: the flow fails
  commitInputStates                      NotaryFlow.kt:133-141
    UniquenessException -> Conflict(tx, SignedData(serialized conflict, notary signature over it))
  TimestampChecker.isValid               core/.../node/services/TimestampChecker.kt:13-26

`BatchingNotary.notarise(requests)` runs that decision procedure for a whole batch: ONE Merkle call
recomputes every tx id (an empty transaction fails only its own request), ONE verify call checks
every signature of every transaction — sharded over the ranks of a process group when one is given,
each rank verifying its 64-aligned slice on its own GPU and ONE all-gather (RCCL under the "nccl"
backend) replicating the verdict and key-status bitmaps into the commit step — then inputs are
committed in request order (so conflicts resolve exactly as sequential flows would) and the notary
signs every accepted id and every conflict report in ONE GPU signing call.  Contract verification
and dependency resolution (ResolveTransactionsFlow) are out of scope.

A request that the reference answers with a Result carries `error` (a NotaryError); one whose flow
the reference fails by an exception carries `failure` (that exception) instead — the client sees
the flow end with it, never a notary signature.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

from . import native
from .crypto import (CompositeKey, DigitalSignature, EdDSAPublicKey, IllegalArgumentException, IllegalStateException,
                     InvalidKeyException, SignatureException, VerifyItem, _prefilter, verify_many, verify_with_ecdsa)
from .transactions import (MerkleTreeException, SecureHash, SignaturesMissingException, SignedTransaction,
                           WireTransaction, compute_ids)


# ---------------------------------------------------------------- timestamps (Structures.kt:412-423)
@dataclass(frozen=True)
class Timestamp:
    """Timestamp(after, before) in epoch seconds; at least one bound, after <= before."""
    after: Optional[float]
    before: Optional[float]

    def __post_init__(self):
        if self.after is None and self.before is None:
            raise IllegalArgumentException("At least one of before/after must be specified")
        if self.after is not None and self.before is not None and not self.after <= self.before:
            raise IllegalStateException("Check failed.")

    @staticmethod
    def around(time_s: float, tolerance_s: float) -> "Timestamp":
        return Timestamp(time_s - tolerance_s, time_s + tolerance_s)


class TimestampChecker:
    """TimestampChecker.kt:13-26: valid iff neither bound is further than `tolerance` from now."""

    def __init__(self, clock: Callable[[], float] = time.time, tolerance: float = 30.0):
        self.clock = clock
        self.tolerance = tolerance

    def is_valid(self, ts: Timestamp) -> bool:
        now = self.clock()
        if ts.before is not None and now - ts.before > self.tolerance:
            return False
        if ts.after is not None and ts.after - now > self.tolerance:
            return False
        return True


# ---------------------------------------------------------------- uniqueness (corda_amd/uniqueness.py)
from .uniqueness import (ConsumingTx, InMemoryUniquenessProvider, PersistentUniquenessProvider,  # noqa: E402,F401
                         UniquenessConflict, UniquenessException)


@dataclass
class SignedData:
    """SignedData.kt:14-39: serialized bytes + a signature over them; verified() checks the signature
    (SignatureException when it does not match) and returns the deserialized conflict."""
    raw: bytes
    sig: DigitalSignature.WithKey

    def verified(self, engine: Optional[native.Engine] = None) -> UniquenessConflict:
        verify_with_ecdsa(self.sig.by, self.raw, self.sig, engine)
        return UniquenessConflict.deserialize(self.raw)


# ---------------------------------------------------------------- NotaryError (NotaryFlow.kt:163-176)
class NotaryError:
    pass


@dataclass
class Conflict(NotaryError):
    tx: WireTransaction
    conflict: SignedData

    def __str__(self):
        return f"One or more input states for transaction {self.tx.id!r} have been used in another transaction"


@dataclass
class TimestampInvalid(NotaryError):
    pass


@dataclass
class TransactionInvalid(NotaryError):
    pass


@dataclass
class SignaturesMissing(NotaryError):
    missing_signers: set


class NotaryException(Exception):
    def __init__(self, error: NotaryError):
        super().__init__(f"Error response from Notary - {error}")
        self.error = error


# ---------------------------------------------------------------- requests and results
@dataclass
class SignRequest:
    stx: SignedTransaction
    caller: str
    input_refs: Optional[List[object]] = None     # StateRefs; default: the serialized input leaves
    timestamp: Optional[Timestamp] = None         # wtx.timestamp (the mirror's leaves are not decoded)


@dataclass
class Result:
    """Result.Success(sig) (ok), Result.Error(error), or the flow's failure exception (failure)."""
    ok: bool
    sig: Optional[DigitalSignature.WithKey] = None
    error: Optional[NotaryError] = None
    failure: Optional[Exception] = None

    def get_or_throw(self) -> DigitalSignature.WithKey:
        """What NotaryFlow.Client returns or throws (NotaryFlow.kt:56-72)."""
        if self.failure is not None:
            raise self.failure
        if self.error is not None:
            raise NotaryException(self.error)
        return self.sig


# ---------------------------------------------------------------- verification, sharded over ranks
def verify_many_sharded(items: Sequence[VerifyItem], engine, group=None) -> List[Optional[Exception]]:
    """verify_many over a process group: rank r verifies its 64-aligned slice of the items on its own
    engine; the verdict bits and the bad-key bits of every slice are replicated to every rank by ONE
    all-gather (distributed.gather_bitmaps; RCCL under "nccl", CPU tensors under "gloo"); every
    rank then rebuilds the same per-item exceptions verify_many returns for the whole list."""
    import torch
    import torch.distributed as dist
    from . import distributed as D

    n = len(items)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    b, e = D.shard_range(n, world, rank)
    per = D.shard_words(n, world)
    errs = verify_many(items[b:e], engine) if e > b else []
    ok = np.zeros(per * 64, bool)
    bad_key = np.zeros(per * 64, bool)
    for j, err in enumerate(errs):
        ok[j] = err is None
        bad_key[j] = isinstance(err, InvalidKeyException)
    local = np.stack([np.packbits(ok, bitorder="little").view("<i8"), np.packbits(bad_key, bitorder="little").view("<i8")])
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    glob = D.gather_bitmaps(torch.from_numpy(local).to(dev), n, group).cpu().numpy().view(np.uint64)
    okg = native.bitmap_to_bools(glob[0], n)
    badg = native.bitmap_to_bools(glob[1], n)
    out: List[Optional[Exception]] = []
    for i, it in enumerate(items):
        if okg[i]:
            out.append(None)
            continue
        pre = _prefilter(it)
        out.append(pre if pre is not None else
                   InvalidKeyException("not a valid GroupElement") if badg[i] else
                   SignatureException("Signature did not match"))
    return out


# ---------------------------------------------------------------- the notary
class BatchingNotary:
    def __init__(self, notary_seed: bytes, validating: bool = True, engine: Optional[native.Engine] = None,
                 uniqueness=None,
                 timestamp_checker: Optional[TimestampChecker] = None, group=None):
        self.engine = engine or native.default_engine()
        self.seed = np.frombuffer(bytes(notary_seed), np.uint8).reshape(1, 32)
        pk, _ = self.engine.sign_batch(self.seed, np.zeros(16, np.uint8), np.zeros(1, np.uint64),
                                       np.zeros(1, np.uint32))
        self.public_key = EdDSAPublicKey(pk[0].tobytes())
        self.owning_key: CompositeKey = self.public_key.composite
        self.validating = validating
        self.uniqueness = uniqueness if uniqueness is not None else InMemoryUniquenessProvider()
        self.timestamp_checker = timestamp_checker or TimestampChecker()
        self.group = group

    def _verify(self, items: List[VerifyItem]) -> List[Optional[Exception]]:
        if self.group is not None:
            return verify_many_sharded(items, self.engine, self.group)
        return verify_many(items, self.engine)

    def _sign(self, msgs: List[bytes]) -> List[DigitalSignature.WithKey]:
        """The notary key over every message, in one GPU signing call."""
        m = len(msgs)
        lens = np.fromiter((len(x) for x in msgs), np.uint32, count=m)
        offs = np.zeros(m, np.uint64)
        if m > 1:
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        arena = np.frombuffer(b"".join(msgs) + b"\0" * 16, np.uint8)
        _, sigs = self.engine.sign_batch(np.repeat(self.seed, m, axis=0), arena, offs, lens)
        return [DigitalSignature.WithKey(self.public_key, sigs[j].tobytes()) for j in range(m)]

    def notarise(self, requests: Sequence[SignRequest]) -> List[Result]:
        n = len(requests)
        results: List[Optional[Result]] = [None] * n
        # val wtx = stx.tx: every unknown id in one Merkle call, then check(temp.id == id) per request
        unknown = [r.stx._wtx for r in requests if r.stx._wtx._id is None]
        if unknown:
            compute_ids(unknown, self.engine)
        failed: List[Optional[Exception]] = [None] * n
        for k, r in enumerate(requests):
            try:
                r.stx.tx
            except (IllegalStateException, MerkleTreeException) as e:
                failed[k] = e
        # the signatures of every transaction in one verify call (validating notary only)
        first_bad: List[Optional[Exception]] = [None] * n
        if self.validating:
            items, begin = [], [0]
            for k, r in enumerate(requests):
                if failed[k] is None:
                    items.extend(VerifyItem(s.by, r.stx.id.bytes, s.bits) for s in r.stx.sigs)
                begin.append(len(items))
            errs = self._verify(items)
            for k in range(n):
                first_bad[k] = next((e for e in errs[begin[k]:begin[k + 1]] if e is not None), None)
        accepted: List[int] = []
        conflicts: List[tuple] = []
        to_commit: List[tuple] = []
        for k, r in enumerate(requests):
            if failed[k] is not None:
                results[k] = Result(False, failure=failed[k])
                continue
            if r.timestamp is not None and not self.timestamp_checker.is_valid(r.timestamp):
                results[k] = Result(False, error=TimestampInvalid())
                continue
            if self.validating:
                e = first_bad[k]
                if e is None:
                    try:
                        r.stx._finish_verify((self.owning_key,))
                    except SignaturesMissingException as ex:
                        results[k] = Result(False, error=SignaturesMissing(ex.missing))
                        continue
                    except Exception as ex:  # noqa: BLE001 - mirrored reference exceptions
                        e = ex
                if e is not None:
                    if isinstance(e, SignatureException):
                        results[k] = Result(False, error=TransactionInvalid())
                    else:                                      # ValidatingNotaryFlow.kt:35: else -> throw e
                        results[k] = Result(False, failure=e)
                    continue
            refs = r.input_refs if r.input_refs is not None else list(r.stx._wtx.inputs)
            to_commit.append((k, refs))
        # commitInputStates for the whole batch, decided in request order (uniqueness.py)
        reqs = [(refs, requests[k].stx.id, requests[k].caller) for k, refs in to_commit]
        if hasattr(self.uniqueness, "commit_batch"):
            decided = self.uniqueness.commit_batch(reqs)
        else:
            decided = []
            for states, tx_id, caller in reqs:
                try:
                    self.uniqueness.commit(states, tx_id, caller)
                    decided.append(None)
                except UniquenessException as ex:
                    decided.append(ex.error)
        for (k, _), c in zip(to_commit, decided):
            if c is None:
                accepted.append(k)
            else:
                conflicts.append((k, c.serialize()))
        msgs = [requests[k].stx.id.bytes for k in accepted] + [raw for _, raw in conflicts]
        sigs = self._sign(msgs) if msgs else []
        for j, k in enumerate(accepted):
            results[k] = Result(True, sig=sigs[j])
        for j, (k, raw) in enumerate(conflicts):
            results[k] = Result(False, error=Conflict(requests[k].stx.tx, SignedData(raw, sigs[len(accepted) + j])))
        return results  # type: ignore[return-value]
