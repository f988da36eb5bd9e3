"""Pins the oracle (test infrastructure) before anything is checked against it.

- RFC 8032 §7.1 TEST 1 and OpenSSL's Ed25519 (deterministic signatures must match byte for byte)
- the Python literal restatement (slide() and all) vs the independent C restatement on the whole
  golden corpus (adversarial classes included)
- the reference's own Merkle golden root (PartialMerkleTreeTest.kt:23-26) and its 1-leaf / odd-level
  cases (:60-74), and the SHA-256 KAT of the prospectus jar (SellerFlow.kt:23)
"""
import hashlib
import os
import random
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

import ed25519_ref as E

HERE = os.path.dirname(os.path.abspath(__file__))


def test_rfc8032_test1():
    sk = bytes.fromhex("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    assert E.public_key_of(sk).hex() == "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a"
    sig = E.sign(sk, b"")
    assert sig.hex() == ("e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701"
                         "cf9b46bd25bf5f0595bbe24655141438e7a100b")
    assert E.verify(E.public_key_of(sk), b"", sig)


@pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI absent")
def test_openssl_crosscheck_signing():
    rng = random.Random(4)
    for i in range(4):
        seed = bytes(rng.randrange(256) for _ in range(32))
        msg = bytes(rng.randrange(256) for _ in range(1 + 37 * i))
        with tempfile.TemporaryDirectory() as td:
            with open(os.path.join(td, "k.der"), "wb") as f:
                f.write(bytes.fromhex("302e020100300506032b657004220420") + seed)
            with open(os.path.join(td, "m"), "wb") as f:
                f.write(msg)
            subprocess.run(["openssl", "pkey", "-inform", "DER", "-in", os.path.join(td, "k.der"), "-out",
                            os.path.join(td, "k.pem")], check=True, capture_output=True)
            out = subprocess.run(["openssl", "pkeyutl", "-sign", "-rawin", "-inkey", os.path.join(td, "k.pem"), "-in",
                                  os.path.join(td, "m")], check=True, capture_output=True).stdout
        assert out == E.sign(seed, msg)


def test_c_oracle_matches_golden(corpus, oracle_c):
    v, s = oracle_c.verify_batch(corpus["pk"], corpus["sig"], corpus["arena"], corpus["off"], corpus["len"], 4)
    assert np.array_equal(v, corpus["verdict"])
    assert np.array_equal(s, corpus["status"])


def test_python_literal_matches_golden_sample(corpus, manifest):
    """The committed verdicts reproduce from the literal Python restatement (one item per class)."""
    seen = set()
    for i in range(len(corpus["pk"])):
        c = int(corpus["cls"][i])
        if c in seen:
            continue
        seen.add(c)
        m = corpus["arena"][corpus["off"][i]:corpus["off"][i] + corpus["len"][i]].tobytes()
        st, ok = E.verify_ex(corpus["pk"][i].tobytes(), m, corpus["sig"][i].tobytes())
        assert (st, int(ok)) == (int(corpus["status"][i]), int(corpus["verdict"][i])), manifest["classes"][c]
    assert len(seen) == len(manifest["classes"])


def test_corpus_covers_adversarial_classes(manifest):
    pc = manifest["per_class"]
    for cls in ["A_noncanonical_y", "A_x0_sign1", "A_not_on_curve", "A_small_order", "A_mixed_order",
                "R_noncanonical", "R_not_on_curve", "S_plus_kL", "S_carry_loss", "S_ge_2^255_no_loss",
                "cofactored_only", "wrong_message", "wrong_key"]:
        assert pc[cls]["n"] > 0, cls
    # eddsa-0.1.0 quirks must show up as ACCEPTED items, not only rejections
    for cls in ["A_noncanonical_y", "A_x0_sign1", "A_small_order", "A_mixed_order", "S_plus_kL", "S_carry_loss"]:
        assert pc[cls]["accepted"] > 0, cls
    assert pc["cofactored_only"]["accepted"] == 0


def test_length_cases(manifest):
    for case in manifest["length_cases"]:
        st, ok = E.verify_ex(bytes.fromhex(case["pk"]), bytes.fromhex(case["msg"]), bytes.fromhex(case["sig"]))
        assert st == case["status"] and st != E.ST_OK and not ok


def test_slide_drop_needs_bit255():
    """slide() drops its top carry only when bit 255 of S is set (the GPU fast path relies on it)."""
    rng = random.Random(9)
    for _ in range(3000):
        v = rng.getrandbits(255)                    # bit 255 clear
        assert not E.slide_drops_carry(v.to_bytes(32, "little"))
    for k in range(1, 24):                          # runs of ones right below bit 255
        for low in (0, (1 << 200) - 1, rng.getrandbits(230)):
            v = (((1 << k) - 1) << (255 - k)) | (low & ((1 << (255 - k)) - 1))
            assert not E.slide_drops_carry(v.to_bytes(32, "little"))
    assert E.slide_drops_carry(b"\xff" * 32)        # S = 2^256 - 1 -> effective -1
    assert E.slide_value(b"\xff" * 32) == -1


def test_merkle_golden_root_and_cases(merkle_cases, oracle_c):
    sha = lambda b: hashlib.sha256(b).digest()
    leaves = [sha(bytes([7, 0, ord(c)])) for c in "abcdef"]
    ids, st = oracle_c.merkle_tx_ids(merkle_cases["arena"], merkle_cases["leaf_off"], merkle_cases["leaf_len"],
                                     merkle_cases["tx_leaf_begin"])
    assert ids[0].tobytes().hex().upper() == "F6D8FB3720114F8D040D64F633B0D9178EB09A55AA7D62FAE1A070D1BF561051"
    assert ids[1].tobytes() == leaves[0]                               # one node: root = leaf
    h1 = sha(leaves[0] + leaves[1])
    h2 = sha(leaves[2] + leaves[2])
    assert ids[2].tobytes() == sha(h1 + h2)                            # odd level duplicates the last node
    assert st[3] == 1                                                  # empty -> MerkleTreeException
    assert np.array_equal(ids, merkle_cases["ids"]) and np.array_equal(st, merkle_cases["status"])


def test_sha256_jar_kat(oracle_c):
    data = open(os.path.join(HERE, "golden", "bank-of-london-cp.jar.bin"), "rb").read()
    assert len(data) == 71644
    assert oracle_c.sha256(data).hex() == "decd098666b9657314870e192ced0c3519c2c9d395507a238338f8d003929de9"


def test_entropy_to_seed_matches_biginteger():
    assert E.entropy_to_seed(20) == b"\x14" + bytes(31)          # DUMMY_NOTARY_KEY
    assert E.entropy_to_seed(10) == b"\x0a" + bytes(31)          # DUMMY_CASH_ISSUER_KEY
    assert E.entropy_to_seed(255)[:2] == b"\x00\xff"             # sign byte kept, then copyOf(32)
    assert len(E.entropy_to_seed(1 << 300)) == 32
