"""Host-side mirror of Corda's signature API, backed by the MI355X engine.

Mirrors (names, argument meaning, error behaviour):
  DigitalSignature / DigitalSignature.WithKey   core/src/main/kotlin/net/corda/core/crypto/CryptoUtilities.kt:27-36
  OpaqueBytes (non-empty)                       core/src/main/kotlin/net/corda/core/serialization/ByteArrays.kt:12-15
  NullPublicKey / DummyPublicKey / NullSignature CryptoUtilities.kt:38-60
  PublicKey.verifyWithECDSA(content, sig)       CryptoUtilities.kt:90-96   -> verify_with_ecdsa
  CompositeKey (Leaf / Node / Builder)          core/src/main/kotlin/net/corda/core/crypto/CompositeKey.kt:22-148

Every verification goes through the GPU (corda_amd.native); batches are gathered into one C-ABI
call and the bitmap is scanned in input order, so "the first bad signature throws" ordering of the
reference's sequential loops is preserved.

Error mapping (reference -> here):
  sig.bits.size != 64              SignatureException("signature length is wrong")      (host prefilter)
  key not an EdDSAPublicKey        InvalidKeyException                                  (host prefilter)
  key bytes not a valid point      InvalidKeyException("not a valid GroupElement")      (GPU status byte;
                                   the reference throws IllegalArgumentException earlier, when the
                                   EdDSAPublicKey is built at deserialisation time)
  verify() == false                SignatureException("Signature did not match")
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import native


class SignatureException(Exception):
    """java.security.SignatureException"""


class InvalidKeyException(Exception):
    """java.security.InvalidKeyException"""


class IllegalArgumentException(ValueError):
    """kotlin require(...) failures"""


class IllegalStateException(RuntimeError):
    """kotlin check(...) failures"""


# ---------------------------------------------------------------- keys
class PublicKey:
    algorithm = "?"

    @property
    def encoded(self) -> bytes:
        raise NotImplementedError


class EdDSAPublicKey(PublicKey):
    """An Ed25519 public key as it travels on the wire (32 bytes, `Ed25519PublicKeySerializer`,
    reference core/.../serialization/Kryo.kt:294-304).  Point validity is decided on the GPU."""
    algorithm = "EdDSA"

    __slots__ = ("_b",)

    def __init__(self, encoded: bytes):
        encoded = bytes(encoded)
        if len(encoded) != 32:
            raise IllegalArgumentException("public-key length is wrong")
        self._b = encoded

    @property
    def encoded(self) -> bytes:
        return self._b

    def __eq__(self, other):
        return isinstance(other, EdDSAPublicKey) and other._b == self._b

    def __hash__(self):
        return hash(self._b)

    def __repr__(self):
        return f"EdDSAPublicKey({self._b.hex()[:16]}…)"

    @property
    def composite(self) -> "CompositeKey":
        return CompositeKey.Leaf(self)


class _NullPublicKey(PublicKey):
    algorithm = "NULL"

    @property
    def encoded(self) -> bytes:
        return b"\x00"

    def __repr__(self):
        return "NULL_KEY"


NullPublicKey = _NullPublicKey()


class DummyPublicKey(PublicKey):
    algorithm = "DUMMY"

    def __init__(self, s: str):
        self.s = s

    @property
    def encoded(self) -> bytes:
        return self.s.encode()

    def __eq__(self, other):
        return isinstance(other, DummyPublicKey) and other.s == self.s

    def __hash__(self):
        return hash(self.s)

    def __repr__(self):
        return f"PUBKEY[{self.s}]"


# ---------------------------------------------------------------- signatures
class OpaqueBytes:
    def __init__(self, bits: bytes):
        bits = bytes(bits)
        if len(bits) == 0:
            raise IllegalArgumentException("Byte Array must not be empty")
        self.bits = bits

    @property
    def bytes(self) -> bytes:
        return self.bits

    def __eq__(self, other):
        return isinstance(other, OpaqueBytes) and other.bits == self.bits

    def __hash__(self):
        return hash(self.bits)


class DigitalSignature(OpaqueBytes):
    class WithKey(OpaqueBytes):
        def __init__(self, by: PublicKey, bits: bytes):
            super().__init__(bits)
            self.by = by

        def verify_with_ecdsa(self, content) -> None:
            # verifyWithECDSA(content: OpaqueBytes): SecureHash is OpaqueBytes in the reference
            content = content.bytes if hasattr(content, "bytes") and not isinstance(content, bytes) else bytes(content)
            verify_with_ecdsa(self.by, content, self)


class LegallyIdentifiable(DigitalSignature.WithKey):
    def __init__(self, signer_name: str, by: PublicKey, bits: bytes):
        super().__init__(by, bits)
        self.signer = signer_name


NullSignature = DigitalSignature.WithKey(NullPublicKey, bytes(32))


# ---------------------------------------------------------------- batched verification core
@dataclass
class VerifyItem:
    key: PublicKey
    content: bytes
    sig_bits: bytes


def _prefilter(item: VerifyItem) -> Optional[Exception]:
    if not isinstance(item.key, EdDSAPublicKey):
        return InvalidKeyException(f"cannot identify EdDSA public key: {type(item.key).__name__}")
    if len(item.sig_bits) != 64:
        return SignatureException("signature length is wrong")
    return None


def verify_many(items: Sequence[VerifyItem], engine: Optional[native.Engine] = None) -> List[Optional[Exception]]:
    """Verifies every item in ONE engine call; returns, per item, None (valid) or the exception the
    reference would throw for it.  Host prefilter handles non-EdDSA keys and bad lengths."""
    n = len(items)
    out: List[Optional[Exception]] = [None] * n
    idx = []
    for i, it in enumerate(items):
        e = _prefilter(it)
        if e is not None:
            out[i] = e
        else:
            idx.append(i)
    if not idx:
        return out
    m = len(idx)
    pk = np.empty((m, 32), np.uint8)
    sig = np.empty((m, 64), np.uint8)
    lens = np.fromiter((len(items[i].content) for i in idx), dtype=np.uint32, count=m)
    offs = np.zeros(m, np.uint64)
    if m > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = np.frombuffer(b"".join(items[i].content for i in idx) + b"\0" * 16, np.uint8)
    for j, i in enumerate(idx):
        pk[j] = np.frombuffer(items[i].key.encoded, np.uint8)
        sig[j] = np.frombuffer(items[i].sig_bits, np.uint8)
    eng = engine or native.default_engine()
    bitmap, status = eng.verify_batch(pk, sig, arena, offs, lens)
    ok = native.bitmap_to_bools(bitmap, m)
    for j, i in enumerate(idx):
        if status[j] == native.CV_SIG_BAD_KEY:
            out[i] = InvalidKeyException("not a valid GroupElement")
        elif not ok[j]:
            out[i] = SignatureException("Signature did not match")
    return out


def verify_with_ecdsa(public_key: PublicKey, content: bytes, signature: OpaqueBytes,
                      engine: Optional[native.Engine] = None) -> None:
    """PublicKey.verifyWithECDSA (CryptoUtilities.kt:90-96): returns None or raises."""
    err = verify_many([VerifyItem(public_key, bytes(content), signature.bytes)], engine)[0]
    if err is not None:
        raise err


# ---------------------------------------------------------------- composite keys
class CompositeKey:
    """CompositeKey.kt:22-148: weighted-threshold key tree; fulfilment is pure host logic."""

    def is_fulfilled_by(self, keys) -> bool:
        raise NotImplementedError

    @property
    def keys(self) -> frozenset:
        raise NotImplementedError

    def contains_any(self, other_keys) -> bool:
        return bool(self.keys & set(other_keys))

    @property
    def single_key(self) -> PublicKey:
        ks = self.keys
        if len(ks) != 1:
            raise IllegalStateException("The key is composed of more than one PublicKey primitive")
        return next(iter(ks))

    class Leaf:
        pass

    class Node:
        pass

    class Builder:
        pass


class _Leaf(CompositeKey):
    def __init__(self, public_key: PublicKey):
        self.public_key = public_key

    def is_fulfilled_by(self, keys) -> bool:
        if isinstance(keys, PublicKey):
            keys = {keys}
        return self.public_key in set(keys)

    @property
    def keys(self) -> frozenset:
        return frozenset({self.public_key})

    def __eq__(self, other):
        return isinstance(other, _Leaf) and other.public_key == self.public_key

    def __hash__(self):
        return hash(self.public_key)

    def __repr__(self):
        return f"Leaf({self.public_key!r})"


class _Node(CompositeKey):
    def __init__(self, threshold: int, children: List[CompositeKey], weights: List[int]):
        self.threshold = threshold
        self.children = list(children)
        self.weights = list(weights)

    def is_fulfilled_by(self, keys) -> bool:
        if isinstance(keys, PublicKey):
            keys = {keys}
        keys = set(keys)
        total = sum(w for c, w in zip(self.children, self.weights) if c.is_fulfilled_by(keys))
        return total >= self.threshold

    @property
    def keys(self) -> frozenset:
        s = set()
        for c in self.children:
            s |= c.keys
        return frozenset(s)

    def __eq__(self, other):
        return (isinstance(other, _Node) and other.threshold == self.threshold and other.weights == self.weights
                and other.children == self.children)

    def __hash__(self):
        return hash((self.threshold, tuple(self.weights), tuple(self.children)))

    def __repr__(self):
        return "(" + ", ".join(map(repr, self.children)) + ")"


class _Builder:
    def __init__(self):
        self._children: List[CompositeKey] = []
        self._weights: List[int] = []

    def add_key(self, key: CompositeKey, weight: int = 1) -> "_Builder":
        self._children.append(key)
        self._weights.append(weight)
        return self

    def add_keys(self, *keys: CompositeKey) -> "_Builder":
        for k in keys:
            self.add_key(k)
        return self

    def build(self, threshold: Optional[int] = None) -> _Node:
        return _Node(len(self._children) if threshold is None else threshold, self._children, self._weights)


CompositeKey.Leaf = _Leaf
CompositeKey.Node = _Node
CompositeKey.Builder = _Builder
