#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/ from the Python oracle.

    python tests/golden/make_golden.py            # rewrites ed25519_corpus.npz, merkle_cases.npz, manifest.json

Expected verdicts come from oracle/ed25519_ref.py (the literal eddsa-0.1.0 restatement, slide() and
all).  Honest signatures are cross-checked against OpenSSL's Ed25519 (`openssl pkeyutl -rawin`) when
the `openssl` CLI is present: signing is deterministic, so the bytes must be identical.

Corpus layout (SoA, one row per signature): pk[n,32], sig[n,64], msg arena + off[n] + len[n],
expected verdict[n] (0/1), expected status[n] (0 ok, 1 bad key encoding), cls[n] (index into
manifest["classes"]).  Length-malformed inputs (sig != 64 B, key != 32 B) cannot be expressed in the
fixed-width C-ABI records; they live in manifest["length_cases"] for the host-mirror tests.
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import ed25519_ref as E  # noqa: E402

SEED = 20261015
P, L = E.P, E.L


def key_seed(i: int) -> bytes:
    """key seed_i = SHA-256("cv-key" || u64le(i))."""
    return hashlib.sha256(b"cv-key" + i.to_bytes(8, "little")).digest()


def msg_bytes(j: int, n: int) -> bytes:
    """SHA-512 counter stream keyed by "cv-msg" || u64le(j)."""
    out = b""
    c = 0
    while len(out) < n:
        out += hashlib.sha512(b"cv-msg" + j.to_bytes(8, "little") + c.to_bytes(8, "little")).digest()
        c += 1
    return out[:n]


class Corpus:
    def __init__(self):
        self.rows = []
        self.classes = []

    def add(self, cls: str, pk: bytes, msg: bytes, sig: bytes, expect=None):
        assert len(pk) == 32 and len(sig) == 64
        st, ok = E.verify_ex(pk, msg, sig)
        if expect is not None:
            assert (st, ok) == expect, (cls, st, ok, expect)
        if cls not in self.classes:
            self.classes.append(cls)
        self.rows.append((self.classes.index(cls), pk, msg, sig, int(ok), st))
        return st, ok


def openssl_sign(seed: bytes, msg: bytes):
    if shutil.which("openssl") is None:
        return None
    with tempfile.TemporaryDirectory() as td:
        kd = os.path.join(td, "k.der")
        with open(kd, "wb") as f:
            f.write(bytes.fromhex("302e020100300506032b657004220420") + seed)
        kp = os.path.join(td, "k.pem")
        mp = os.path.join(td, "m.bin")
        with open(mp, "wb") as f:
            f.write(msg)
        subprocess.run(["openssl", "pkey", "-inform", "DER", "-in", kd, "-out", kp], check=True,
                       capture_output=True)
        r = subprocess.run(["openssl", "pkeyutl", "-sign", "-rawin", "-inkey", kp, "-in", mp], check=True,
                           capture_output=True)
        return r.stdout


def enc_y(y_raw: int, sign: int) -> bytes:
    b = bytearray(y_raw.to_bytes(32, "little"))
    b[31] = (b[31] & 0x7F) | (sign << 7)
    return bytes(b)


def forge_small_order_key(pk: bytes, msg: bytes, rng: random.Random):
    """Signature accepted by eddsa-0.1.0 for a small-order key A (unknown secret): choose R = [s]B - [j]A'
    so that [h](-A) lands on the same torsion offset (h mod 8 == j mod ord(A))."""
    A = E.decode_point_0_1_0(pk)
    abyte = E.pt_encode(A)
    for _ in range(400):
        s = rng.randrange(L)
        for j in range(8):
            R = E.pt_add(E.pt_mul(s, E.BASE), E.pt_neg(E.pt_mul(j, A)))
            rb = E.pt_encode(R)
            h = int.from_bytes(hashlib.sha512(rb + abyte + msg).digest(), "little") % L
            if E.pt_eq(E.pt_mul(h, A), E.pt_mul(j, A)):
                return rb + s.to_bytes(32, "little")
    raise RuntimeError("no forgery found")


def build_ed25519(c: Corpus, rng: random.Random, stats: dict):
    # ---- RFC 8032 §7.1 TEST 1 (recalled; reproduced by the oracle and by OpenSSL)
    sk1 = bytes.fromhex("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    pk1 = bytes.fromhex("d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a")
    sig1 = bytes.fromhex("e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc6"
                         "1e39701cf9b46bd25bf5f0595bbe24655141438e7a100b")
    assert E.public_key_of(sk1) == pk1 and E.sign(sk1, b"") == sig1
    c.add("rfc8032", pk1, b"", sig1, (0, True))

    # ---- Corda test keys: DUMMY_NOTARY_KEY = entropyToKeyPair(20), DUMMY_CASH_ISSUER_KEY = entropyToKeyPair(10)
    xcheck = 0
    seeds = [E.entropy_to_seed(20), E.entropy_to_seed(10)] + [key_seed(i) for i in range(40)]
    for k, seed in enumerate(seeds):
        pk = E.public_key_of(seed)
        for j in range(3):
            txid = hashlib.sha256(msg_bytes(1000 * k + j, 64)).digest()          # M = 32-byte tx id
            sig = E.sign(seed, txid)
            if xcheck < 24:
                o = openssl_sign(seed, txid)
                if o is not None:
                    assert o == sig, "OpenSSL disagrees with the oracle signer"
                    xcheck += 1
            c.add("corda_honest", pk, txid, sig, (0, True))
            bad = bytearray(txid)
            bad[5] ^= 1                                                          # TransactionSerializationTests.kt:72-75
            c.add("wrong_message", pk, bytes(bad), sig, (0, False))
    # ---- message-length sweep across SHA-512 block boundaries (64 + len over 112/128/240/256)
    for ln in [0, 1, 3, 31, 32, 33, 47, 48, 49, 63, 64, 111, 112, 113, 127, 128, 175, 176, 177, 191, 192,
               255, 256, 300, 301, 511, 1000]:
        seed = key_seed(500 + ln)
        m = msg_bytes(2000 + ln, ln)
        sig = E.sign(seed, m)
        if xcheck < 40 and ln > 0:          # pkeyutl -rawin refuses an empty input file
            o = openssl_sign(seed, m)
            if o is not None:
                assert o == sig
                xcheck += 1
        c.add("msg_len_sweep", E.public_key_of(seed), m, sig, (0, True))
    # ---- ~300-byte messages (config C2 shape)
    for i in range(64):
        seed = key_seed(3000 + i)
        m = msg_bytes(3000 + i, 300)
        c.add("msg300", E.public_key_of(seed), m, E.sign(seed, m), (0, True))
    # ---- wrong key / foreign signature (SignedDataTest.kt:22-29)
    for i in range(16):
        sa, sb = key_seed(4000 + i), key_seed(5000 + i)
        m = msg_bytes(4000 + i, 32)
        c.add("wrong_key", E.public_key_of(sb), m, E.sign(sa, m), (0, False))
    # ---- random bit flips anywhere in R or S
    for i in range(48):
        seed = key_seed(6000 + i)
        m = msg_bytes(6000 + i, 32)
        sig = bytearray(E.sign(seed, m))
        sig[rng.randrange(64)] ^= 1 << rng.randrange(8)
        c.add("bitflip", E.public_key_of(seed), m, bytes(sig), (0, False))
    stats["openssl_crosschecked"] = xcheck

    # ---- adversarial: A with non-canonical y in [p, p+18] (both sign bits)
    for k in range(19):
        for sgn in (0, 1):
            pk = enc_y(P + k, sgn)
            m = msg_bytes(7000 + 2 * k + sgn, 32)
            try:
                E.decode_point_0_1_0(pk)
            except E.InvalidKeyError:
                c.add("A_noncanonical_y", pk, m, bytes(64), (1, False))
                continue
            if k in (0, 1):                     # y = 0 (order 4) and y = 1 (identity): forgeable
                c.add("A_noncanonical_y", pk, m, forge_small_order_key(pk, m, rng), (0, True))
            c.add("A_noncanonical_y", pk, m, msg_bytes(7100 + k, 64))
    # ---- A with x = 0 and sign bit 1 (y = 1 identity, y = -1 order 2)
    for y in (1, P - 1):
        pk = enc_y(y, 1)
        for j in range(3):
            m = msg_bytes(7200 + 10 * (y & 1) + j, 32)
            c.add("A_x0_sign1", pk, m, forge_small_order_key(pk, m, rng), (0, True))
        # the same forgery with the canonical sign bit is also accepted; a random sig is rejected
        c.add("A_x0_sign1", pk, m, msg_bytes(7300 + (y & 1), 64))
    # identity key: R = [S]B verifies ANY message (S arbitrary)
    ident = enc_y(1, 0)
    for j in range(3):
        s = rng.randrange(L)
        sig = E.pt_encode(E.pt_mul(s, E.BASE)) + s.to_bytes(32, "little")
        c.add("A_small_order", ident, msg_bytes(7400 + j, 32), sig, (0, True))
    # ---- A not on curve
    n_off = 0
    y = 2
    while n_off < 24:
        pk = enc_y(y, y & 1)
        try:
            E.decode_point_0_1_0(pk)
        except E.InvalidKeyError:
            c.add("A_not_on_curve", pk, msg_bytes(7500 + n_off, 32), msg_bytes(7600 + n_off, 64), (1, False))
            n_off += 1
        y = y * 7 + 3
        y %= P
    # ---- A small-order: the 8 torsion points (canonical encodings), forged and random sigs
    tors = E.torsion_points()
    for ti, T in enumerate(tors):
        pk = E.pt_encode(T)
        for j in range(2):
            m = msg_bytes(7700 + 4 * ti + j, 32)
            c.add("A_small_order", pk, m, forge_small_order_key(pk, m, rng), (0, True))
        c.add("A_small_order", pk, msg_bytes(7750 + ti, 32), msg_bytes(7760 + ti, 64))
    # ---- A mixed order: A = [a]B + T; honest sig (accepted iff h ≡ 0 mod ord T) and crafted accepted sig
    for ti in range(1, 8):
        T = tors[ti]
        seed = key_seed(8000 + ti)
        a, prefix, _ = E.seed_to_keypair(seed)
        Amix = E.pt_add(E.pt_mul(a, E.BASE), T)
        pk = E.pt_encode(Amix)
        for j in range(3):
            m = msg_bytes(8000 + 10 * ti + j, 32)
            r = rng.randrange(L)
            R = E.pt_mul(r, E.BASE)
            rb = E.pt_encode(R)
            h = int.from_bytes(hashlib.sha512(rb + pk + m).digest(), "little") % L
            c.add("A_mixed_order", pk, m, rb + ((r + h * a) % L).to_bytes(32, "little"))
            # crafted: R_j = [r]B - [j]T with h_j ≡ j (mod ord T)
            for jj in range(8):
                Rj = E.pt_add(R, E.pt_neg(E.pt_mul(jj, T)))
                rjb = E.pt_encode(Rj)
                hj = int.from_bytes(hashlib.sha512(rjb + pk + m).digest(), "little") % L
                if E.pt_eq(E.pt_mul(hj, T), E.pt_mul(jj, T)):
                    c.add("A_mixed_order", pk, m, rjb + ((r + hj * a) % L).to_bytes(32, "little"), (0, True))
                    break
    # ---- non-canonical R: identity key + S = 0 gives R' = identity; encode R as y = p + 1
    for sgn in (0, 1):
        m = msg_bytes(8100 + sgn, 32)
        c.add("R_noncanonical", ident, m, enc_y(P + 1, sgn) + bytes(32), (0, False))
    c.add("R_noncanonical", ident, msg_bytes(8102, 32), enc_y(1, 0) + bytes(32), (0, True))
    for i in range(8):                                   # honest sig with R's y pushed past p (y < 19 never)
        seed = key_seed(8200 + i)
        m = msg_bytes(8200 + i, 32)
        sig = bytearray(E.sign(seed, m))
        sig[31] |= 0x7F
        sig[0:31] = b"\xff" * 31
        c.add("R_noncanonical", E.public_key_of(seed), m, bytes(sig), (0, False))
    # ---- R not on curve / random R
    for i in range(8):
        seed = key_seed(8300 + i)
        m = msg_bytes(8300 + i, 32)
        sig = E.sign(seed, m)
        c.add("R_not_on_curve", E.public_key_of(seed), m, msg_bytes(8350 + i, 32) + sig[32:], (0, False))
    # ---- S + k·L (no S < L check); k large enough pushes S past 2^255 where slide may drop the carry
    for i in range(6):
        seed = key_seed(8400 + i)
        m = msg_bytes(8400 + i, 32)
        sig = E.sign(seed, m)
        s = int.from_bytes(sig[32:], "little")
        for k in range(1, 16):
            s2 = s + k * L
            if s2 >= 1 << 256:
                continue
            c.add("S_plus_kL", E.public_key_of(seed), m, sig[:32] + s2.to_bytes(32, "little"))
    # ---- S with bit 255 set and a top run of ones: carry loss -> effective S - 2^256
    n_drop_acc = n_drop_rej = n_nodrop_acc = 0
    i = 0
    while (n_drop_acc < 12 or n_drop_rej < 6 or n_nodrop_acc < 8) and i < 4000:
        seed = key_seed(9000 + i)
        m = msg_bytes(9000 + i, 32)
        sig = E.sign(seed, m)
        s = int.from_bytes(sig[32:], "little")
        pk = E.public_key_of(seed)
        i += 1
        # drop-accept: S ≡ s + 2^256 (mod L), S in [2^255, 2^256) and slide drops the carry
        base = (s + (1 << 256)) % L
        cands = [base + j * L for j in range(16) if (1 << 255) <= base + j * L < (1 << 256)]
        rng.shuffle(cands)
        for S2 in cands:
            sb = S2.to_bytes(32, "little")
            if E.slide_drops_carry(sb) and n_drop_acc < 12:
                c.add("S_carry_loss", pk, m, sig[:32] + sb, (0, True))
                n_drop_acc += 1
                break
        # drop-reject: S ≡ s (mod L) but carry dropped -> wrong scalar
        cands = [s + j * L for j in range(16) if (1 << 255) <= s + j * L < (1 << 256)]
        for S2 in cands:
            sb = S2.to_bytes(32, "little")
            if E.slide_drops_carry(sb):
                if n_drop_rej < 6:
                    c.add("S_carry_loss", pk, m, sig[:32] + sb, (0, False))
                    n_drop_rej += 1
            elif n_nodrop_acc < 8:
                c.add("S_ge_2^255_no_loss", pk, m, sig[:32] + sb, (0, True))
                n_nodrop_acc += 1
    # all-ones S (effective -1) with the identity key: R' = [-1]B
    c.add("S_carry_loss", ident, msg_bytes(9999, 32), E.pt_encode(E.pt_neg(E.BASE)) + b"\xff" * 32, (0, True))
    # ---- valid only under the cofactored equation: R = [r]B + T8
    for i in range(8):
        seed = key_seed(9500 + i)
        a, prefix, pk = E.seed_to_keypair(seed)
        m = msg_bytes(9500 + i, 32)
        r = rng.randrange(L)
        R = E.pt_add(E.pt_mul(r, E.BASE), tors[1 + (i % 7)])
        rb = E.pt_encode(R)
        h = int.from_bytes(hashlib.sha512(rb + pk + m).digest(), "little") % L
        c.add("cofactored_only", pk, m, rb + ((r + h * a) % L).to_bytes(32, "little"), (0, False))
    # ---- all-zero / all-ones signatures under honest keys
    for i in range(4):
        pk = E.public_key_of(key_seed(9600 + i))
        c.add("degenerate_sig", pk, msg_bytes(9600 + i, 32), bytes(64), (0, False))
        c.add("degenerate_sig", pk, msg_bytes(9610 + i, 32), b"\xff" * 64, (0, False))


def length_cases():
    seed = key_seed(1)
    pk = E.public_key_of(seed)
    m = msg_bytes(1, 32)
    sig = E.sign(seed, m)
    out = []
    for sl in (0, 63, 65, 128):
        s = (sig + sig)[:sl]
        out.append({"pk": pk.hex(), "msg": m.hex(), "sig": s.hex(), "status": E.verify_ex(pk, m, s)[0]})
    for kl in (31, 33):
        k = (pk + pk)[:kl]
        out.append({"pk": k.hex(), "msg": m.hex(), "sig": sig.hex(), "status": E.verify_ex(k, m, sig)[0]})
    return out


def sha256(b):
    return hashlib.sha256(b).digest()


def merkle_root(leaves):
    if not leaves:
        return None
    lvl = list(leaves)
    while len(lvl) > 1:
        if len(lvl) % 2:
            lvl.append(lvl[-1])
        lvl = [sha256(lvl[i] + lvl[i + 1]) for i in range(0, len(lvl), 2)]
    return lvl[0]


def build_merkle(rng: random.Random):
    """Transactions as lists of leaf blobs.  tx 0 is PartialMerkleTreeTest.kt:23-26 ("abcdef" Kryo chars)."""
    txs = []
    txs.append([bytes([7, 0, ord(ch)]) for ch in "abcdef"])
    txs.append([bytes([7, 0, ord("a")])])                  # one leaf: root = leaf hash (:60-64)
    txs.append([bytes([7, 0, ord(ch)]) for ch in "abc"])  # odd level duplication (:67-74)
    txs.append([])                                         # empty: MerkleTreeException (:55-57)
    for n in list(range(1, 18)) + [31, 32, 33, 64, 100]:
        txs.append([msg_bytes(20000 + 100 * n + k, rng.randint(0, 700)) for k in range(n)])
    for k in range(24):                                    # C3 shape: 6 leaves, 2x120, 2x600, 2x300 +-25%
        shape = [120, 120, 600, 600, 300, 300]
        txs.append([msg_bytes(30000 + 10 * k + q, int(s * rng.uniform(0.75, 1.25))) for q, s in enumerate(shape)])
    # blob sizes across SHA-256 padding boundaries
    txs.append([msg_bytes(40000 + ln, ln) for ln in [0, 1, 55, 56, 57, 63, 64, 65, 119, 120, 128, 1000]])
    arena = bytearray()
    off, ln, begin = [], [], [0]
    roots, status = [], []
    for t in txs:
        for blob in t:
            off.append(len(arena))
            ln.append(len(blob))
            arena += blob
        begin.append(len(off))
        r = merkle_root([sha256(b) for b in t])
        roots.append(r if r is not None else bytes(32))
        status.append(0 if r is not None else 1)
    assert roots[0].hex().upper() == "F6D8FB3720114F8D040D64F633B0D9178EB09A55AA7D62FAE1A070D1BF561051"
    return dict(arena=np.frombuffer(bytes(arena), np.uint8), leaf_off=np.array(off, np.uint64),
                leaf_len=np.array(ln, np.uint32), tx_leaf_begin=np.array(begin, np.uint32),
                ids=np.frombuffer(b"".join(roots), np.uint8).reshape(-1, 32),
                status=np.array(status, np.uint8))


def main():
    rng = random.Random(SEED)
    c = Corpus()
    stats = {}
    build_ed25519(c, rng, stats)
    n = len(c.rows)
    pk = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    arena = bytearray()
    off = np.zeros(n, np.uint64)
    ln = np.zeros(n, np.uint32)
    verdict = np.zeros(n, np.uint8)
    status = np.zeros(n, np.uint8)
    cls = np.zeros(n, np.uint8)
    for i, (ci, p_, m_, s_, ok, st) in enumerate(c.rows):
        pk[i] = np.frombuffer(p_, np.uint8)
        sig[i] = np.frombuffer(s_, np.uint8)
        off[i] = len(arena)
        ln[i] = len(m_)
        arena += m_
        verdict[i] = ok
        status[i] = st
        cls[i] = ci
    np.savez(os.path.join(HERE, "ed25519_corpus.npz"), pk=pk, sig=sig,
             arena=np.frombuffer(bytes(arena) or b"\0", np.uint8), off=off, len=ln, verdict=verdict,
             status=status, cls=cls)
    mk = build_merkle(rng)
    np.savez(os.path.join(HERE, "merkle_cases.npz"), **mk)
    per_class = {name: {"n": int((cls == i).sum()), "accepted": int(verdict[cls == i].sum()),
                        "bad_key": int((status[cls == i] == 1).sum())} for i, name in enumerate(c.classes)}
    manifest = {
        "generator": "tests/golden/make_golden.py",
        "oracle": "oracle/ed25519_ref.py (eddsa-0.1.0 verify restatement, literal slide())",
        "seed": SEED,
        "n_signatures": n,
        "classes": c.classes,
        "per_class": per_class,
        "openssl_crosschecked_honest_signatures": stats.get("openssl_crosschecked", 0),
        "length_cases": length_cases(),
        "merkle": {"n_tx": int(mk["ids"].shape[0]),
                   "golden_root_PartialMerkleTreeTest_kt_25":
                       "F6D8FB3720114F8D040D64F633B0D9178EB09A55AA7D62FAE1A070D1BF561051"},
        "sha256_kat": {"file": "bank-of-london-cp.jar.bin",
                       "source": "samples/trader-demo/src/main/resources/bank-of-london-cp.jar (data only, hashed)",
                       "sha256": "decd098666b9657314870e192ced0c3519c2c9d395507a238338f8d003929de9",
                       "ref": "samples/trader-demo/src/main/kotlin/net/corda/traderdemo/flow/SellerFlow.kt:23"},
    }
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(json.dumps(per_class, indent=1))
    print("signatures:", n, "openssl cross-checked:", stats.get("openssl_crosschecked"))


if __name__ == "__main__":
    main()
