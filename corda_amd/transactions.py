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
from .crypto import (CompositeKey, DigitalSignature, EdDSAPublicKey, IllegalArgumentException, IllegalStateException,
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
            if self._id is None:
                raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
        return self._id


def compute_ids(txs: Sequence[WireTransaction], engine: Optional[native.Engine] = None
                ) -> List[Optional[SecureHash]]:
    """WireTransaction.id for many transactions in one GPU call (leaf SHA-256 + Merkle tree).  Per
    transaction: its id, or None for a transaction with no leaves — whose `.id` then raises
    MerkleTreeException on its own (MerkleTree.getMerkleTree(emptyList), MerkleTransaction.kt), so
    one empty transaction does not fail the others in the batch."""
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
            out.append(None)
            continue
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


def verify_signatures_batch_fused(stxs: Sequence[SignedTransaction], allowed_to_be_missing: Iterable[CompositeKey] = (),
                                  engine: Optional[native.Engine] = None) -> List[Optional[Exception]]:
    """verify_signatures_batch through ONE cv_verify_transactions call (every id recomputed on the device and
    kept there as its signatures' message), with the same per-transaction exceptions as the sequential reference.

    The fused call verifies each signature over the RECOMPUTED id; the reference verifies over the CLAIMED id
    first (checkSignaturesAreValid, SignedTransaction.kt:82-87) and compares ids only afterwards (the `tx` getter,
    :34-38, and :70).  So a SignatureException must win over the IllegalStateException of a mismatched id, and
    the first failing signature names the exception.  Wherever the fused verdict does not settle that, the
    transaction takes the separate path — its signatures re-verified over the claimed id in one more call:
      - recomputed id != claimed id (a signature bad over the claimed id throws
        SignatureException, not IllegalStateException);
      - tx_ok == 0 with equal ids (which signature failed first, and whether its key is not a point);
      - no leaves (MerkleTreeException from `tx`) or a signature the host prefilter rejects (non-EdDSA key,
        wrong length): these never enter the fused call.
    Every honest transaction is decided by the fused call alone (INTEGRATION.md gives the JVM shim the same
    rule)."""
    allowed = tuple(allowed_to_be_missing)
    eng = engine or native.default_engine()
    fused, slow = [], []
    for k, stx in enumerate(stxs):
        conforming = all(isinstance(s.by, EdDSAPublicKey) and len(s.bits) == 64 for s in stx.sigs)
        (fused if conforming and stx._wtx.leaves else slow).append(k)
    out: List[Optional[Exception]] = [None] * len(stxs)
    decided = []
    if fused:
        leaves: List[bytes] = []
        lbegin, sbegin = [0], [0]
        pk, sig = [], []
        for k in fused:
            leaves.extend(stxs[k]._wtx.leaves)
            lbegin.append(len(leaves))
            for s in stxs[k].sigs:
                pk.append(s.by.encoded)
                sig.append(s.bits)
            sbegin.append(len(pk))
        lens = np.fromiter((len(b) for b in leaves), dtype=np.uint32, count=len(leaves))
        offs = np.zeros(len(leaves), np.uint64)
        if len(leaves) > 1:
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        arena = np.frombuffer(b"".join(leaves) + b"\0" * 16, np.uint8)
        pk_a = np.frombuffer(b"".join(pk), np.uint8).reshape(-1, 32)
        sig_a = np.frombuffer(b"".join(sig), np.uint8).reshape(-1, 64)
        ok, ids, _, _ = eng.verify_transactions(arena, offs, lens, np.array(lbegin, np.uint32), pk_a, sig_a,
                                                np.array(sbegin, np.uint32), want_status=False)
        for j, k in enumerate(fused):
            stxs[k]._wtx._id = SecureHash(ids[j].tobytes())          # the WireTransaction's own id
            (decided if ok[j] and stxs[k]._wtx._id == stxs[k].id else slow).append(k)
    if slow:
        slow.sort()
        items: List[VerifyItem] = []
        begin = [0]
        for k in slow:
            items.extend(VerifyItem(s.by, stxs[k].id.bytes, s.bits) for s in stxs[k].sigs)
            begin.append(len(items))
        errs = verify_many(items, eng)
        unknown = [stxs[k]._wtx for k in slow if stxs[k]._wtx._id is None and stxs[k]._wtx.leaves]
        if unknown:
            compute_ids(unknown, eng)
        for j, k in enumerate(slow):
            out[k] = next((e for e in errs[begin[j]:begin[j + 1]] if e is not None), None)
            if out[k] is None:
                decided.append(k)
    for k in decided:
        try:
            stxs[k]._finish_verify(allowed)
        except Exception as e:  # noqa: BLE001 - mirrored reference exceptions
            out[k] = e
    return out


# ---------------------------------------------------------------- filtered transactions
# Prover side (host): the full MerkleTree with its DuplicatedLeaf marks and PartialMerkleTree.build
# (MerkleTransaction.kt:49-101, PartialMerkleTree.kt:69-111) — object work the JVM does once per
# tear-off.  Verifier side (GPU): PartialMerkleTree.verify for many trees in one call
# (cv_partial_merkle_verify), the root recompute + multiset check of PartialMerkleTree.kt:117-144.
def _hash_concat(a: bytes, b: bytes) -> bytes:
    import hashlib
    return hashlib.sha256(a + b).digest()


class MerkleTree:
    """MerkleTree.Leaf / Node / DuplicatedLeaf (MerkleTransaction.kt:49-57)."""
    __slots__ = ("hash", "left", "right", "duplicated")

    def __init__(self, h: SecureHash, left=None, right=None, duplicated: bool = False):
        self.hash, self.left, self.right, self.duplicated = h, left, right, duplicated

    @staticmethod
    def get_merkle_tree(all_leaves_hashes: Sequence[SecureHash]) -> "MerkleTree":
        """MerkleTree.getMerkleTree / buildMerkleTree (MerkleTransaction.kt:66-99)."""
        lvl = [MerkleTree(h) for h in all_leaves_hashes]
        if len(lvl) < 1:
            raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
        while len(lvl) > 1:
            n = len(lvl)
            nxt = []
            for i in range(0, n, 2):
                left = lvl[i]
                right = MerkleTree(lvl[n - 1].hash, duplicated=True) if i + 1 > n - 1 else lvl[i + 1]
                nxt.append(MerkleTree(SecureHash(_hash_concat(left.hash.bytes, right.hash.bytes)), left, right))
            lvl = nxt
        return lvl[0]


class PartialTree:
    """PartialMerkleTree.PartialTree: IncludedLeaf / Leaf (hash set) or Node (children set)."""
    __slots__ = ("hash", "included", "left", "right")

    def __init__(self, h: Optional[SecureHash] = None, included: bool = False, left=None, right=None):
        self.hash, self.included, self.left, self.right = h, included, left, right


class PartialMerkleTree:
    LEAF, INCLUDED, NODE = 0, 1, 2

    def __init__(self, root: PartialTree):
        self.root = root

    @staticmethod
    def build(merkle_root: MerkleTree, include_hashes: Sequence[SecureHash]) -> "PartialMerkleTree":
        """PartialMerkleTree.build (PartialMerkleTree.kt:69-111)."""
        include = list(include_hashes)
        used: List[SecureHash] = []

        def rec(node: MerkleTree):
            if node.left is None:
                if not node.duplicated and node.hash in include:
                    used.append(node.hash)
                    return True, PartialTree(node.hash, included=True)
                return False, PartialTree(node.hash)
            lf, lt = rec(node.left)
            rf, rt = rec(node.right)
            if lf or rf:
                return True, PartialTree(left=lt, right=rt)
            return False, PartialTree(node.hash)

        _, tree = rec(merkle_root)
        if len(include) != len(used):
            raise MerkleTreeException("Some of the provided hashes are not in the tree.")
        return PartialMerkleTree(tree)

    def flatten(self, base: int = 0):
        """Post-order flat encoding of include/cordaverify.h (absolute indices from `base`)."""
        kind: List[int] = []
        left: List[int] = []
        right: List[int] = []
        hashes: List[bytes] = []

        def rec(n: PartialTree) -> int:
            if n.left is not None:
                li, ri = rec(n.left), rec(n.right)
                kind.append(self.NODE); left.append(li); right.append(ri); hashes.append(bytes(32))
            else:
                kind.append(self.INCLUDED if n.included else self.LEAF)
                left.append(0); right.append(0); hashes.append(n.hash.bytes)
            return base + len(kind) - 1

        rec(self.root)
        return kind, left, right, hashes

    def verify(self, merkle_root_hash: SecureHash, hashes_to_check: Sequence[SecureHash],
               engine: Optional[native.Engine] = None) -> bool:
        """PartialMerkleTree.verify (PartialMerkleTree.kt:117-124), on the GPU."""
        return verify_partial_trees([(self, merkle_root_hash, list(hashes_to_check))], engine)[0]


def verify_partial_trees(items, engine: Optional[native.Engine] = None) -> List[bool]:
    """Many PartialMerkleTree.verify(root, hashesToCheck) in ONE GPU call.  items: (pmt, root, hashes)."""
    kind: List[int] = []
    left: List[int] = []
    right: List[int] = []
    hashes: List[bytes] = []
    tb, cb = [0], [0]
    roots: List[bytes] = []
    checks: List[bytes] = []
    for pmt, root, hs in items:
        k, l, r, h = pmt.flatten(len(kind))
        kind += k; left += l; right += r; hashes += h
        tb.append(len(kind))
        roots.append(root.bytes)
        checks += [x.bytes for x in hs]
        cb.append(len(checks))
    eng = engine or native.default_engine()
    v, st = eng.partial_merkle_verify(np.array(kind, np.uint8), np.array(left, np.uint32), np.array(right, np.uint32),
                                      np.frombuffer(b"".join(hashes), np.uint8).reshape(-1, 32),
                                      np.array(tb, np.uint32), np.frombuffer(b"".join(roots), np.uint8).reshape(-1, 32),
                                      np.frombuffer(b"".join(checks), np.uint8).reshape(-1, 32) if checks
                                      else np.zeros((0, 32), np.uint8), np.array(cb, np.uint32))
    if (st != 0).any():
        raise IllegalArgumentException("malformed partial Merkle tree encoding")
    return [bool(x) for x in v]


class FilteredLeaves:
    """FilteredLeaves (MerkleTransaction.kt:105-119): the serialized leaves kept in the tear-off."""

    def __init__(self, inputs: Sequence[bytes] = (), outputs: Sequence[bytes] = (), attachments: Sequence[bytes] = (),
                 commands: Sequence[bytes] = ()):
        self.inputs, self.outputs = list(inputs), list(outputs)
        self.attachments, self.commands = list(attachments), list(commands)

    def get_filtered_hashes(self) -> List[SecureHash]:
        import hashlib
        return [SecureHash(hashlib.sha256(b).digest())
                for b in self.inputs + self.outputs + self.attachments + self.commands]


class FilteredTransaction:
    """FilteredTransaction (MerkleTransaction.kt:146-178)."""

    def __init__(self, filtered_leaves: FilteredLeaves, partial_merkle_tree: PartialMerkleTree):
        self.filtered_leaves = filtered_leaves
        self.partial_merkle_tree = partial_merkle_tree

    @staticmethod
    def build_merkle_transaction(wtx: WireTransaction, filter_inputs=lambda b: False, filter_outputs=lambda b: False,
                                 filter_attachments=lambda b: False, filter_commands=lambda b: False
                                 ) -> "FilteredTransaction":
        """FilteredTransaction.buildMerkleTransaction with FilterFuns over the serialized leaves."""
        import hashlib
        fl = FilteredLeaves([x for x in wtx.inputs if filter_inputs(x)], [x for x in wtx.outputs if filter_outputs(x)],
                            [x for x in wtx.attachments if filter_attachments(x)],
                            [x for x in wtx.commands if filter_commands(x)])
        full = MerkleTree.get_merkle_tree([SecureHash(hashlib.sha256(b).digest()) for b in wtx.leaves])
        return FilteredTransaction(fl, PartialMerkleTree.build(full, fl.get_filtered_hashes()))

    def verify(self, merkle_root_hash: SecureHash, engine: Optional[native.Engine] = None) -> bool:
        hashes = self.filtered_leaves.get_filtered_hashes()
        if len(hashes) == 0:
            raise MerkleTreeException("Transaction without included leaves.")
        return self.partial_merkle_tree.verify(merkle_root_hash, hashes, engine)


def verify_filtered_batch(items, engine: Optional[native.Engine] = None) -> List[bool]:
    """FilteredTransaction.verify(root) for many tear-offs in one GPU call.  items: (ftx, root)."""
    batch = []
    for ftx, root in items:
        hashes = ftx.filtered_leaves.get_filtered_hashes()
        if len(hashes) == 0:
            raise MerkleTreeException("Transaction without included leaves.")
        batch.append((ftx.partial_merkle_tree, root, hashes))
    return verify_partial_trees(batch, engine)
