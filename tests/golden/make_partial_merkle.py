#!/usr/bin/env python3
"""Generates tests/golden/partial_merkle_cases.npz: flat partial Merkle trees (the encoding of
cv_partial_merkle_verify) with expected verdicts/status from oracle/merkle_ref.py.

Cases: every verify scenario of the reference's PartialMerkleTreeTest.kt:76-160 on its "abcdef"
Kryo-char leaves (sha256 of bytes 07 00 <char>, the same leaves whose root is pinned at :23-26),
random trees (1..70 leaves) with honest, permuted, extra, missing, replaced and duplicated check
lists, wrong roots, tampered stored hashes, and malformed encodings.

    python tests/golden/make_partial_merkle.py
"""
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import merkle_ref as M  # noqa: E402

SEED = 20261016


def kryo_char(ch: str) -> bytes:
    return bytes([7, 0, ord(ch)])


def main():
    rng = random.Random(SEED)
    cases = []   # (name, kind, left, right, hashes(list), root, check, expect_verdict, expect_status)

    def add(name, tree, root, check):
        k, l, r, h = M.flatten(tree)
        v, st = M.verify_flat(k, l, r, h, 0, len(k), root, check)
        assert st == 0 and v == (1 if M.verify_partial(tree, root, check) else 0)
        cases.append((name, k, l, r, h, root, list(check), v, st))

    hashed = [M.sha256(kryo_char(c)) for c in "abcdef"]
    mt = M.get_merkle_tree(hashed)
    assert mt.hash.hex().upper() == "F6D8FB3720114F8D040D64F633B0D9178EB09A55AA7D62FAE1A070D1BF561051"
    # PartialMerkleTreeTest.kt
    incl = [hashed[3], hashed[5]]
    add("only_left_nodes_branch", M.build_partial(mt, incl), mt.hash, incl)                     # :83-87
    add("include_zero_leaves", M.build_partial(mt, []), mt.hash, [])                            # :90-93
    add("include_all_leaves", M.build_partial(mt, hashed), mt.hash, hashed)                     # :96-99
    add("too_many_leaves", M.build_partial(mt, incl), mt.hash, incl + [hashed[0]])              # :117-122
    add("too_little_leaves", M.build_partial(mt, incl + [hashed[0]]), mt.hash, incl)            # :125-130
    mt5 = M.get_merkle_tree(hashed[:5])
    add("duplicate_leaves", M.build_partial(mt5, [hashed[3], hashed[4]]), mt5.hash,
        [hashed[3], hashed[4], hashed[4]])                                                      # :133-139
    add("different_leaves", M.build_partial(mt, incl), mt.hash, [hashed[2], hashed[4]])         # :142-146
    add("wrong_root", M.build_partial(mt, incl), M.hash_concat(hashed[3], hashed[5]), incl)     # :149-154
    # random trees
    for t in range(400):
        n = rng.choice([1, 2, 3, 4, 5, 6, 7, 8, 9, 15, 16, 17, 31, 33, 64, 70])
        leaves = [M.sha256(rng.randbytes(rng.randint(1, 40))) for _ in range(n)]
        if rng.random() < 0.15 and n > 2:                       # repeated leaf values
            leaves[rng.randrange(n)] = leaves[rng.randrange(n)]
        full = M.get_merkle_tree(leaves)
        sub = [h for h in leaves if rng.random() < 0.3]
        try:
            pt = M.build_partial(full, sub)
        except M.MerkleTreeException:
            continue
        used = []
        M._verify_rec(pt, used)
        mode = t % 8
        check = list(used)
        root = full.hash
        if mode == 1:
            rng.shuffle(check)                                  # order does not matter (multiset)
        elif mode == 2:
            check.append(leaves[rng.randrange(n)])              # one too many
        elif mode == 3 and check:
            check.pop(rng.randrange(len(check)))                # one missing
        elif mode == 4 and check:
            check[rng.randrange(len(check))] = M.sha256(b"x%d" % t)   # replaced
        elif mode == 5:
            root = M.sha256(b"root%d" % t)                      # wrong root
        elif mode == 6 and check:
            check.append(check[0])                              # duplicated entry
        add(f"random_{t}_m{mode}", pt, root, check)
        if mode == 7:                                           # tamper a stored (cut) hash
            k, l, r, h = M.flatten(pt)
            idx = [i for i in range(len(k)) if k[i] == M.LEAF]
            if idx:
                i = rng.choice(idx)
                h = list(h)
                h[i] = bytes([h[i][0] ^ 1]) + h[i][1:]
                v, st = M.verify_flat(k, l, r, h, 0, len(k), full.hash, used)
                cases.append((f"random_{t}_tampered", k, l, r, h, full.hash, list(used), v, st))
    # malformed encodings (status 2)
    k, l, r, h = M.flatten(M.build_partial(mt, incl))
    root_i = len(k) - 1
    bad = []
    kk, ll, rr = list(k), list(l), list(r)
    ll[root_i] = root_i                                        # child not before its parent
    bad.append(("child_after_parent", kk, ll, rr, h))
    kk, ll, rr = list(k), list(l), list(r)
    rr[root_i] = ll[root_i]                                    # same child twice
    bad.append(("shared_child", kk, ll, rr, h))
    kk, ll, rr = list(k), list(l), list(r)
    kk.insert(0, M.LEAF); ll = [0] + [x + 1 for x in ll]; rr = [0] + [x + 1 for x in rr]
    hh = [bytes(32)] + list(h)
    bad.append(("dangling_node", kk, ll, rr, hh))
    kk = list(k); kk[0] = 7
    bad.append(("bad_kind", kk, list(l), list(r), h))
    for name, kk, ll, rr, hh in bad:
        v, st = M.verify_flat(kk, ll, rr, hh, 0, len(kk), mt.hash, incl)
        assert st == 2
        cases.append((name, kk, ll, rr, hh, mt.hash, incl, v, st))
    cases.append(("empty_tree", [], [], [], [], mt.hash, [], 0, 2))

    # concatenate with absolute indices
    kind, left, right, hashes, tb = [], [], [], [], [0]
    roots, checks, cb, ev, es, names = [], [], [0], [], [], []
    for name, k, l, r, h, root, check, v, st in cases:
        base = len(kind)
        kind += k
        left += [x + base for x in l]
        right += [x + base for x in r]
        hashes += list(h)
        tb.append(len(kind))
        roots.append(root)
        checks += list(check)
        cb.append(len(checks))
        ev.append(v)
        es.append(st)
        names.append(name)
    np.savez(os.path.join(HERE, "partial_merkle_cases.npz"),
             kind=np.array(kind, np.uint8), left=np.array(left, np.uint32), right=np.array(right, np.uint32),
             leaf_hash=np.frombuffer(b"".join(hashes) or bytes(32), np.uint8).reshape(-1, 32)[:max(len(kind), 1)],
             tree_begin=np.array(tb, np.uint32), root=np.frombuffer(b"".join(roots), np.uint8).reshape(-1, 32),
             check=np.frombuffer(b"".join(checks) or bytes(32), np.uint8).reshape(-1, 32)[:max(len(checks), 1)],
             check_begin=np.array(cb, np.uint32), verdict=np.array(ev, np.uint8), status=np.array(es, np.uint8),
             names=np.array(names))
    print(f"{len(cases)} partial trees, {len(kind)} nodes, {sum(ev)} verified, {sum(1 for s in es if s)} malformed")


if __name__ == "__main__":
    main()
