"""Batched notary commit step on the GPU engine (BASELINE config C4 / SURVEY.md §8(a) a11).

The reference notarises one transaction per flow on the node's single thread:
  NotaryFlow.Service.call                core/src/main/kotlin/net/corda/flows/NotaryFlow.kt:97-113
    stx.tx (Merkle id recompute + check) -> validateTimestamp -> beforeCommit -> commitInputStates -> sign(stx.id)
  ValidatingNotaryFlow.beforeCommit      core/src/main/kotlin/net/corda/flows/ValidatingNotaryFlow.kt:24-45
    stx.verifySignatures(notaryKey): SignaturesMissingException -> NotaryError.SignaturesMissing,
    SignatureException -> NotaryError.TransactionInvalid
  UniquenessProvider.commit              core/src/main/kotlin/net/corda/core/node/services/UniquenessProvider.kt:13-15
    (InMemory / Persistent: conflicting inputs -> UniquenessException(Conflict))

`BatchingNotary.notarise(requests)` runs the same decision procedure for a whole batch: ONE Merkle
call recomputes every tx id, ONE verify call checks every signature of every transaction, the
per-transaction AND happens on the verdict bitmap, then inputs are committed in request order
(so conflicts resolve exactly as sequential flows would) and the notary signs every accepted id
in ONE GPU signing call.  Contract verification and dependency resolution (ResolveTransactionsFlow)
are out of scope and are not performed.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import native
from .crypto import (CompositeKey, DigitalSignature, EdDSAPublicKey, IllegalStateException, SignatureException,
                     VerifyItem, verify_many)
from .transactions import SecureHash, SignaturesMissingException, SignedTransaction, compute_ids


# ---------------------------------------------------------------- errors (NotaryError subclasses)
class NotaryError:
    pass


@dataclass
class Conflict(NotaryError):
    tx_id: SecureHash
    state_history: Dict[object, "ConsumingTx"]


@dataclass
class TransactionInvalid(NotaryError):
    cause: str = ""


@dataclass
class SignaturesMissing(NotaryError):
    missing: set


@dataclass
class TimestampInvalid(NotaryError):
    pass


@dataclass
class ConsumingTx:
    id: SecureHash
    input_index: int
    requesting_party: str


class UniquenessException(Exception):
    def __init__(self, conflict: Dict[object, ConsumingTx]):
        super().__init__("conflict")
        self.conflict = conflict


class InMemoryUniquenessProvider:
    """node/.../services/transactions/InMemoryUniquenessProvider.kt semantics: all-or-nothing commit."""

    def __init__(self):
        self.committed: Dict[object, ConsumingTx] = {}

    def commit(self, states: Sequence[object], tx_id: SecureHash, caller: str) -> None:
        conflict = {s: self.committed[s] for s in states if s in self.committed}
        if conflict:
            raise UniquenessException(conflict)
        for i, s in enumerate(states):
            self.committed[s] = ConsumingTx(tx_id, i, caller)


@dataclass
class SignRequest:
    stx: SignedTransaction
    caller: str
    input_refs: Optional[List[object]] = None     # StateRefs; default: the serialized input leaves
    timestamp_ok: bool = True                     # result of the (out-of-scope) TimestampChecker


@dataclass
class Result:
    ok: bool
    sig: Optional[DigitalSignature.WithKey] = None
    error: Optional[NotaryError] = None


class BatchingNotary:
    def __init__(self, notary_seed: bytes, validating: bool = True, engine: Optional[native.Engine] = None,
                 uniqueness: Optional[InMemoryUniquenessProvider] = None):
        self.engine = engine or native.default_engine()
        self.seed = np.frombuffer(bytes(notary_seed), np.uint8).reshape(1, 32)
        pk, _ = self.engine.sign_batch(self.seed, np.zeros(16, np.uint8), np.zeros(1, np.uint64),
                                       np.zeros(1, np.uint32))
        self.public_key = EdDSAPublicKey(pk[0].tobytes())
        self.owning_key = self.public_key.composite
        self.validating = validating
        self.uniqueness = uniqueness or InMemoryUniquenessProvider()

    def notarise(self, requests: Sequence[SignRequest]) -> List[Result]:
        n = len(requests)
        results: List[Optional[Result]] = [None] * n
        # stx.tx: recompute every id in one Merkle call, then check(temp.id == id)
        unknown = [r.stx._wtx for r in requests if r.stx._wtx._id is None]
        if unknown:
            compute_ids(unknown, self.engine)
        id_ok = [r.stx._wtx.id == r.stx.id for r in requests]
        # signatures of every transaction in one verify call (validating notary only)
        errs_per_tx: List[Optional[Exception]] = [None] * n
        if self.validating:
            items, begin = [], [0]
            for r in requests:
                items.extend(VerifyItem(s.by, r.stx.id.bytes, s.bits) for s in r.stx.sigs)
                begin.append(len(items))
            errs = verify_many(items, self.engine)
            for k in range(n):
                errs_per_tx[k] = next((e for e in errs[begin[k]:begin[k + 1]] if e is not None), None)
        to_sign = []
        for k, r in enumerate(requests):
            if not id_ok[k]:
                results[k] = Result(False, error=TransactionInvalid("transaction id does not match its contents"))
                continue
            if not r.timestamp_ok:
                results[k] = Result(False, error=TimestampInvalid())
                continue
            if self.validating:
                if errs_per_tx[k] is not None:
                    results[k] = Result(False, error=TransactionInvalid(str(errs_per_tx[k])))
                    continue
                try:
                    r.stx._finish_verify((self.owning_key,))
                except SignaturesMissingException as e:
                    results[k] = Result(False, error=SignaturesMissing(e.missing))
                    continue
                except (SignatureException, IllegalStateException) as e:
                    results[k] = Result(False, error=TransactionInvalid(str(e)))
                    continue
            refs = r.input_refs if r.input_refs is not None else list(r.stx._wtx.inputs)
            try:
                self.uniqueness.commit(refs, r.stx.id, r.caller)
            except UniquenessException as e:
                results[k] = Result(False, error=Conflict(r.stx.id, e.conflict))
                continue
            to_sign.append(k)
        if to_sign:
            msgs = b"".join(requests[k].stx.id.bytes for k in to_sign)
            m = len(to_sign)
            _, sigs = self.engine.sign_batch(np.repeat(self.seed, m, axis=0), np.frombuffer(msgs + b"\0" * 16, np.uint8),
                                             np.arange(m, dtype=np.uint64) * 32, np.full(m, 32, np.uint32))
            for j, k in enumerate(to_sign):
                results[k] = Result(True, sig=DigitalSignature.WithKey(self.public_key, sigs[j].tobytes()))
        return results  # type: ignore[return-value]
