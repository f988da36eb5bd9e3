"""Host-side mirror of Corda's transaction verification entry points, batched onto the GPU.

Mirrors:
  SecureHash (SHA-256, 32 bytes)                  core/src/main/kotlin/net/corda/core/crypto/SecureHash.kt:11-44
  WireTransaction.id = Merkle root of leaf hashes core/src/main/kotlin/net/corda/core/transactions/WireTransaction.kt:45-52
  calculateLeavesHashes / MerkleTree              core/src/main/kotlin/net/corda/core/transactions/MerkleTransaction.kt:26-101
  SignedTransaction.verifySignatures / checkSignaturesAreValid / SignaturesMissingException
                                                  core/src/main/kotlin/net/corda/core/transactions/SignedTransaction.kt:23-93

Kryo serialisation stays outside: a WireTransaction here is given as its leaf
byte blobs in the reference's order (inputs, outputs, attachments, commands) plus the
`mustSign` composite keys.  Leaf hashing and the tree run on the GPU (cv_merkle_tx_ids).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

from . import native
from .crypto import (CompositeKey, DigitalSignature, IllegalArgumentException, IllegalStateException,
                     SignatureException, VerifyItem, verify_many)


class MerkleTreeException(Exception):
    """net.corda.core.crypto.MerkleTreeException"""


class SecureHash:
    __slots__ = ("bytes",)

    def __init__(self, b: bytes):
        b = bytes(b)
        if len(b) != 32:
            raise IllegalArgumentException(f"Provided string is {len(b)} bytes not 32 bytes")
        self.bytes = b

    @staticmethod
    def parse(s: str) -> "SecureHash":
        return SecureHash(bytes.fromhex(s))

    def __eq__(self, other):
        return isinstance(other, SecureHash) and other.bytes == self.bytes

    def __hash__(self):
        return hash(self.bytes)

    def __repr__(self):
        return self.bytes.hex().upper()

    def prefix_chars(self, n: int = 6) -> str:
        return repr(self)[:n]


class WireTransaction:
    """Leaf blobs (serialized inputs, outputs, attachments, commands — in that order) + signers."""

    def __init__(self, inputs: Sequence[bytes] = (), outputs: Sequence[bytes] = (), attachments: Sequence[bytes] = (),
                 commands: Sequence[bytes] = (), must_sign: Sequence[CompositeKey] = (),
                 command_descriptions: Optional[Dict[CompositeKey, str]] = None, notary_key: Optional[CompositeKey] = None):
        self.inputs = [bytes(x) for x in inputs]
        self.outputs = [bytes(x) for x in outputs]
        self.attachments = [bytes(x) for x in attachments]
        self.commands = [bytes(x) for x in commands]
        self.must_sign = list(must_sign)
        self.command_descriptions = command_descriptions or {}
        self.notary_key = notary_key
        self._id: Optional[SecureHash] = None

    @property
    def leaves(self) -> List[bytes]:
        return self.inputs + self.outputs + self.attachments + self.commands

    @property
    def id(self) -> SecureHash:
        if self._id is None:
            compute_ids([self])
        return self._id


def compute_ids(txs: Sequence[WireTransaction], engine: Optional[native.Engine] = None) -> List[SecureHash]:
    """WireTransaction.id for many transactions in one GPU call (leaf SHA-256 + Merkle tree)."""
    leaves: List[bytes] = []
    begin = [0]
    for t in txs:
        leaves.extend(t.leaves)
        begin.append(len(leaves))
    lens = np.fromiter((len(b) for b in leaves), dtype=np.uint32, count=len(leaves))
    offs = np.zeros(len(leaves), np.uint64)
    if len(leaves) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = np.frombuffer(b"".join(leaves) + b"\0" * 16, np.uint8)
    eng = engine or native.default_engine()
    ids, st = eng.merkle_tx_ids(arena, offs, lens, np.array(begin, np.uint32))
    out = []
    for k, t in enumerate(txs):
        if st[k] == native.CV_TX_EMPTY:
            raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
        t._id = SecureHash(ids[k].tobytes())
        out.append(t._id)
    return out


class SignaturesMissingException(SignatureException):
    def __init__(self, missing, descriptions, id: SecureHash):
        super().__init__(f"Missing signatures for {descriptions} on transaction {id.prefix_chars()} for "
                         f"{', '.join(map(repr, missing))}")
        self.missing = set(missing)
        self.descriptions = list(descriptions)
        self.id = id


class SignedTransaction:
    """SignedTransaction(txBits, sigs, id) — `tx` stands in for the deserialised WireTransaction."""

    def __init__(self, tx: WireTransaction, sigs: Sequence[DigitalSignature.WithKey], id: SecureHash):
        if not sigs:
            raise IllegalArgumentException("Failed requirement.")          # require(sigs.isNotEmpty())
        self._wtx = tx
        self.sigs = list(sigs)
        self.id = id
        self._checked = False

    @property
    def tx(self) -> WireTransaction:
        """lazy deserialise + check(temp.id == id) (SignedTransaction.kt:34-38)"""
        if not self._checked:
            if self._wtx.id != self.id:
                raise IllegalStateException("Supplied transaction ID does not match deserialized transaction's ID - "
                                            "this is probably a problem in serialization/deserialization")
            self._checked = True
        return self._wtx

    def check_signatures_are_valid(self, engine: Optional[native.Engine] = None) -> None:
        """Throws SignatureException (or InvalidKeyException) for the FIRST bad signature, in order."""
        errs = verify_many([VerifyItem(s.by, self.id.bytes, s.bits) for s in self.sigs], engine)
        for e in errs:
            if e is not None:
                raise e

    def _missing_signatures(self):
        sig_keys = {s.by for s in self.sigs}
        return {k for k in self.tx.must_sign if not k.is_fulfilled_by(sig_keys)}

    def verify_signatures(self, *allowed_to_be_missing: CompositeKey, engine: Optional[native.Engine] = None
                          ) -> WireTransaction:
        self.check_signatures_are_valid(engine)
        return self._finish_verify(allowed_to_be_missing)

    def _finish_verify(self, allowed_to_be_missing) -> WireTransaction:
        missing = self._missing_signatures()
        if missing:
            needed = missing - set(allowed_to_be_missing)
            if needed:
                descr = [d for k, d in self.tx.command_descriptions.items() if k in needed]
                if self.tx.notary_key is not None and self.tx.notary_key in needed:
                    descr.append("notary")
                raise SignaturesMissingException(needed, descr, self.id)
        if self.tx.id != self.id:
            raise IllegalStateException("Check failed.")
        return self.tx


def verify_signatures_batch(stxs: Sequence[SignedTransaction], allowed_to_be_missing: Iterable[CompositeKey] = (),
                            engine: Optional[native.Engine] = None) -> List[Optional[Exception]]:
    """verifySignatures() over many transactions with ONE signature-verify call and ONE Merkle call
    (the ResolveTransactionsFlow / notary batch site).  Returns per transaction
    None (verified) or the exception the sequential reference would raise for it."""
    allowed = tuple(allowed_to_be_missing)
    items: List[VerifyItem] = []
    begin = [0]
    for stx in stxs:
        items.extend(VerifyItem(s.by, stx.id.bytes, s.bits) for s in stx.sigs)
        begin.append(len(items))
    errs = verify_many(items, engine)
    unknown = [s._wtx for s in stxs if s._wtx._id is None]
    if unknown:
        compute_ids(unknown, engine)
    out: List[Optional[Exception]] = []
    for k, stx in enumerate(stxs):
        first = next((e for e in errs[begin[k]:begin[k + 1]] if e is not None), None)
        if first is not None:
            out.append(first)
            continue
        try:
            stx._finish_verify(allowed)
            out.append(None)
        except Exception as e:  # noqa: BLE001 - mirrored reference exceptions
            out.append(e)
    return out
