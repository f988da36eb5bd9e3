"""CPU restatement of Corda's Merkle tree, partial Merkle tree and filtered-transaction checks
(pure Python, hashlib).  TEST INFRASTRUCTURE ONLY: nothing under corda_amd/ imports this module.

Restates (reference file:line):
  MerkleTree.getMerkleTree / buildMerkleTree (Leaf, Node, DuplicatedLeaf)
        core/src/main/kotlin/net/corda/core/transactions/MerkleTransaction.kt:49-101
  SecureHash.hashConcat = sha256(left32 || right32)      core/.../crypto/SecureHash.kt (hashConcat)
  PartialMerkleTree.build / buildPartialTree             core/src/main/kotlin/net/corda/core/crypto/PartialMerkleTree.kt:69-111
  PartialMerkleTree.verify (root recompute + multiset of included hashes)   PartialMerkleTree.kt:117-144
  FilteredTransaction.verify (empty -> MerkleTreeException)                 MerkleTransaction.kt:170-178

Pinned by the reference's own vectors: PartialMerkleTreeTest.kt:23-26 (root of "abcdef" Kryo chars,
F6D8FB37...1051) and every build/verify scenario of PartialMerkleTreeTest.kt:76-160
(tests/test_partial_merkle.py replays them).

Also defines the flat encoding the GPU kernel consumes (include/cordaverify.h,
cv_partial_merkle_verify): nodes of all trees concatenated; per node kind (0 Leaf, 1 IncludedLeaf,
2 Node), left/right child (absolute node indices, children before parents), leaf hash; the root is
the last node of each tree's range.
"""
from __future__ import annotations

import hashlib
from collections import Counter
from typing import List, Optional, Sequence, Tuple

LEAF, INCLUDED, NODE = 0, 1, 2


class MerkleTreeException(Exception):
    def __init__(self, reason: str):
        super().__init__(reason)
        self.reason = reason


def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def hash_concat(a: bytes, b: bytes) -> bytes:
    return sha256(a + b)


# ---------------------------------------------------------------- full tree (MerkleTransaction.kt:49-101)
class MTLeaf:
    def __init__(self, h: bytes):
        self.hash = h


class MTDuplicatedLeaf:
    def __init__(self, h: bytes):
        self.hash = h


class MTNode:
    def __init__(self, h: bytes, left, right):
        self.hash, self.left, self.right = h, left, right


def get_merkle_tree(leaves: Sequence[bytes]):
    lvl = [MTLeaf(h) for h in leaves]
    if len(lvl) < 1:
        raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
    while len(lvl) > 1:
        n = len(lvl)
        nxt = []
        for i in range(0, n, 2):
            left = lvl[i]
            right = MTDuplicatedLeaf(lvl[n - 1].hash) if i + 1 > n - 1 else lvl[i + 1]
            nxt.append(MTNode(hash_concat(left.hash, right.hash), left, right))
        lvl = nxt
    return lvl[0]


# ---------------------------------------------------------------- partial tree (PartialMerkleTree.kt)
class PTIncludedLeaf:
    def __init__(self, h: bytes):
        self.hash = h


class PTLeaf:
    def __init__(self, h: bytes):
        self.hash = h


class PTNode:
    def __init__(self, left, right):
        self.left, self.right = left, right


def _build_partial(root, include: Sequence[bytes], used: List[bytes]):
    if isinstance(root, MTLeaf):
        if root.hash in include:
            used.append(root.hash)
            return True, PTIncludedLeaf(root.hash)
        return False, PTLeaf(root.hash)
    if isinstance(root, MTDuplicatedLeaf):
        return False, PTLeaf(root.hash)
    lf, lt = _build_partial(root.left, include, used)
    rf, rt = _build_partial(root.right, include, used)
    if lf or rf:
        return True, PTNode(lt, rt)
    return False, PTLeaf(root.hash)


def build_partial(merkle_root, include: Sequence[bytes]):
    used: List[bytes] = []
    _, tree = _build_partial(merkle_root, list(include), used)
    if len(include) != len(used):
        raise MerkleTreeException("Some of the provided hashes are not in the tree.")
    return tree


def _verify_rec(node, used: List[bytes]) -> bytes:
    if isinstance(node, PTIncludedLeaf):
        used.append(node.hash)
        return node.hash
    if isinstance(node, PTLeaf):
        return node.hash
    return hash_concat(_verify_rec(node.left, used), _verify_rec(node.right, used))


def verify_partial(tree, merkle_root_hash: bytes, hashes_to_check: Sequence[bytes]) -> bool:
    used: List[bytes] = []
    r = _verify_rec(tree, used)
    if Counter(hashes_to_check) != Counter(used):
        return False
    return r == merkle_root_hash


def filtered_verify(tree, merkle_root_hash: bytes, filtered_hashes: Sequence[bytes]) -> bool:
    if len(filtered_hashes) == 0:
        raise MerkleTreeException("Transaction without included leaves.")
    return verify_partial(tree, merkle_root_hash, filtered_hashes)


# ---------------------------------------------------------------- flat encoding (GPU input)
def flatten(tree, base: int = 0) -> Tuple[List[int], List[int], List[int], List[bytes]]:
    """Post-order node list: (kind, left, right, hash) with absolute indices starting at `base`."""
    kind: List[int] = []
    left: List[int] = []
    right: List[int] = []
    hashes: List[bytes] = []

    def rec(n) -> int:
        if isinstance(n, PTNode):
            li = rec(n.left)
            ri = rec(n.right)
            kind.append(NODE); left.append(li); right.append(ri); hashes.append(bytes(32))
        else:
            kind.append(INCLUDED if isinstance(n, PTIncludedLeaf) else LEAF)
            left.append(0); right.append(0); hashes.append(n.hash)
        return base + len(kind) - 1

    rec(tree)
    return kind, left, right, hashes


def verify_flat(kind, left, right, hashes, b: int, e: int, root: bytes,
                check: Sequence[bytes]) -> Tuple[int, int]:
    """(verdict, status) of one flat tree: status 2 = not a tree encoding (children must precede
    their parent inside [b, e), every node but the last referenced exactly once)."""
    if e <= b:
        return 0, 2
    refs = Counter()
    dig: dict = {}
    for k in range(b, e):
        if kind[k] == NODE:
            l, r = left[k], right[k]
            if not (b <= l < k and b <= r < k) or l == r:
                return 0, 2
            refs[l] += 1
            refs[r] += 1
            dig[k] = hash_concat(dig[l], dig[r])
        elif kind[k] in (LEAF, INCLUDED):
            dig[k] = hashes[k]
        else:
            return 0, 2
    if any(refs[k] != 1 for k in range(b, e - 1)) or refs[e - 1] != 0:
        return 0, 2
    used = [dig[k] for k in range(b, e) if kind[k] == INCLUDED]
    ok = Counter(check) == Counter(used) and dig[e - 1] == root
    return (1 if ok else 0), 0
