"""The product's per-lane device code (corda_amd/csrc/*.h, __host__ __device__) run on the CPU via
tests/host_harness.cpp and checked against the oracle: catches logic and limb-bound bugs without a
GPU.  The GPU parity tests (test_gpu_parity.py) then check the compiled kernels themselves."""
import ctypes
import os
import random

import numpy as np
import pytest

import ed25519_ref as E

P, L = E.P, E.L


def _b(x: bytes):
    return (ctypes.c_uint8 * max(1, len(x))).from_buffer_copy(x + b"\0")


def _out(n):
    return (ctypes.c_uint8 * n)()


def _int(o):
    return int.from_bytes(bytes(o), "little")


def test_field_ops_random_and_extreme(host_harness):
    H = host_harness
    rng = random.Random(1)
    vals = [0, 1, 2, 19, P - 1, P, P + 1, P + 18, 2**255 - 1, 2**254, 2**128 + 7] + \
           [rng.randrange(2**255) for _ in range(300)]
    for a in vals:
        c = rng.choice(vals)
        o = _out(32)
        H.cvh_fe_mul(_b(a.to_bytes(32, "little")), _b(c.to_bytes(32, "little")), o)
        assert _int(o) == a * c % P
        H.cvh_fe_sq(_b(a.to_bytes(32, "little")), o, 0)
        assert _int(o) == a * a % P
        H.cvh_fe_sq(_b(a.to_bytes(32, "little")), o, 1)
        assert _int(o) == 2 * a * a % P
        H.cvh_fe_invert(_b(a.to_bytes(32, "little")), o)
        assert _int(o) == pow(a, P - 2, P)


OFF = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]


def _limb_val(v):
    return sum(x * (1 << o) for x, o in zip(v, OFF))


def test_field_mul_at_limb_bounds(host_harness):
    """Unsigned limbs at the documented precondition edges (cv_field.h): mul f <= 8M, g <= 3.3M;
    sq f <= 3.3M.  The harness is built with CV_BOUNDS_CHECK, so it also asserts the preconditions."""
    H = host_harness
    rng = random.Random(2)
    W = [26, 25] * 5

    def limbs(mult):
        return [min(int(rng.choice([mult, mult * 0.999, rng.random() * mult, 0.0]) * (1 << W[i])),
                    int(mult * (1 << W[i])) - 1) for i in range(10)]

    for trial in range(400):
        a = limbs(8.0)
        b = limbs(3.29)
        c = limbs(3.29)
        A = (ctypes.c_uint32 * 10)(*a)
        B = (ctypes.c_uint32 * 10)(*b)
        C = (ctypes.c_uint32 * 10)(*c)
        o = _out(32)
        H.cvh_fe_mul_limbs(A, B, o)
        assert _int(o) == _limb_val(a) * _limb_val(b) % P
        H.cvh_fe_sq_limbs(C, o)
        assert _int(o) == _limb_val(c) ** 2 % P
        H.cvh_fe_to_bytes_limbs(A, o)
        assert _int(o) == _limb_val(a) % P


def test_interleaved_mul_sq_at_limb_bounds(host_harness):
    """fe_mul_n<4> / fe_sq_n<4, DBL> (sequential-carry columns, the forms the group formulas use) at
    the precondition edges: mul f <= 8M, g <= 3.3M; sq f <= 3.3M, chain 2 doubled."""
    H = host_harness
    rng = random.Random(12)
    W = [26, 25] * 5

    def limbs(mult):
        return [min(int(rng.choice([mult, mult * 0.999, rng.random() * mult, 0.0]) * (1 << W[i])),
                    int(mult * (1 << W[i])) - 1) for i in range(10)]

    for trial in range(150):
        a = [limbs(8.0) for _ in range(4)]
        b = [limbs(3.29) for _ in range(4)]
        A = (ctypes.c_uint32 * 40)(*sum(a, []))
        B = (ctypes.c_uint32 * 40)(*sum(b, []))
        o = _out(128)
        H.cvh_fe_mul4_limbs(A, B, o)
        for m in range(4):
            assert int.from_bytes(bytes(o)[32 * m:32 * m + 32], "little") == _limb_val(a[m]) * _limb_val(b[m]) % P
        H.cvh_fe_sq4_limbs(B, o)
        for m in range(4):
            exp = _limb_val(b[m]) ** 2 * (2 if m == 2 else 1) % P
            assert int.from_bytes(bytes(o)[32 * m:32 * m + 32], "little") == exp


def test_sc_reduce(host_harness):
    H = host_harness
    rng = random.Random(3)
    cases = [bytes(64), b"\xff" * 64, L.to_bytes(64, "little"), (L - 1).to_bytes(64, "little"),
             (2 * L).to_bytes(64, "little"), (2**512 - L).to_bytes(64, "little")]
    cases += [rng.getrandbits(512).to_bytes(64, "little") for _ in range(3000)]
    for x in cases:
        o = _out(32)
        H.cvh_sc_reduce(_b(x), o)
        assert _int(o) == int.from_bytes(x, "little") % L


def test_sc_muladd(host_harness):
    H = host_harness
    rng = random.Random(4)
    for _ in range(500):
        a, b, c = (rng.getrandbits(256) for _ in range(3))
        o = _out(32)
        H.cvh_sc_muladd(_b(a.to_bytes(32, "little")), _b(b.to_bytes(32, "little")), _b(c.to_bytes(32, "little")), o)
        assert _int(o) == (a * b + c) % L


def test_slide_replay_and_effective_scalar(host_harness):
    H = host_harness
    rng = random.Random(5)
    for i in range(1500):
        s = rng.getrandbits(256)
        if i % 3 == 0:
            s |= 1 << 255
        if i % 7 == 0:
            s |= ((1 << rng.randrange(1, 40)) - 1) << (256 - 40)
        sb = s.to_bytes(32, "little")
        assert H.cvh_slide_drops(_b(sb)) == int(E.slide_drops_carry(sb))
        o = _out(32)
        H.cvh_effective_s(_b(sb), o)
        assert _int(o) == E.slide_value(sb) % L


def test_signed_digits(host_harness):
    H = host_harness
    rng = random.Random(6)
    for _ in range(200):
        s = rng.getrandbits(255).to_bytes(32, "little")
        assert sum(H.cvh_digit16(_b(s), k) * 16**k for k in range(64)) == int.from_bytes(s, "little")
        assert sum(H.cvh_digit256(_b(s), k) * 256**k for k in range(32)) == int.from_bytes(s, "little")
        assert all(-8 <= H.cvh_digit16(_b(s), k) <= 8 for k in range(64))
        assert all(-128 <= H.cvh_digit256(_b(s), k) <= 128 for k in range(32))


def test_comb_row_digits(host_harness):
    """The keyed comb's row digits (digit256_row, static word indices): equal to digit256(h, 8 j + u) for every
    row j and window u, on random scalars and on the carry edges (bytes 0x7f / 0x80 / 0xff at word borders)."""
    H = host_harness
    rng = random.Random(16)
    cases = [rng.getrandbits(255).to_bytes(32, "little") for _ in range(300)]
    cases += [bytes([b]) * 31 + bytes([b & 0x7f]) for b in (0x00, 0x7f, 0x80, 0xff)]
    cases += [bytes(4 * q) + b"\x80\x00\x00\x00" + bytes(28 - 4 * q) for q in range(7)]
    for s in cases:
        for j in range(4):
            for u in range(8):
                assert H.cvh_digit256_row(_b(s), j, u) == H.cvh_digit256(_b(s), 8 * j + u), (s.hex(), j, u)


def test_radix65536_digit_pairs(host_harness):
    """The throughput group's basepoint digits (cv_scalar.h digits65536_pairs): 16 signed radix-2^16
    digits of w < L with the carry propagated, in [-2^15, 2^15), packed (d_j, d_(j+8)) as 16-bit
    two's complement; sum d_k 2^(16k) = w exactly, on random w and on every carry boundary."""
    import ctypes
    H = host_harness
    L = 2**252 + 27742317777372353535851937790883648493
    rng = random.Random(16)
    cases = [0, 1, L - 1, 2**252, 2**253 - 1]
    cases += [(0x7fff << (16 * k)) | (1 << (16 * k - 1) if k else 0) for k in range(15)]      # x = 2^15 - 1 + carry
    cases += [0x8000 << (16 * k) for k in range(15)] + [(2**(16 * k) - 1) for k in range(1, 16)]
    cases += [rng.randrange(L) for _ in range(3000)]
    out = (ctypes.c_uint32 * 8)()
    for w in cases:
        w %= 2**253
        H.cvh_digits65536(_b(w.to_bytes(32, "little")), out)
        d = []
        for half in (0, 1):
            for j in range(8):
                x = (out[j] >> (16 * half)) & 0xffff
                d.append(x - 0x10000 if x >= 0x8000 else x)
        assert all(-2**15 <= x < 2**15 for x in d)
        assert sum(x * 2**(16 * k) for k, x in enumerate(d)) == w, hex(w)


def test_sha512_and_sha256(host_harness):
    import hashlib
    H = host_harness
    rng = random.Random(7)
    for ln in [0, 1, 31, 47, 48, 49, 55, 56, 57, 63, 64, 111, 112, 113, 119, 120, 121, 127, 128, 200, 300, 1000]:
        pre = bytes(rng.randrange(256) for _ in range(64))
        m = bytes(rng.randrange(256) for _ in range(ln))
        o = _out(64)
        H.cvh_sha512(_b(pre), 64, _b(m), ln, o)
        assert bytes(o) == hashlib.sha512(pre + m).digest()
        H.cvh_sha512(_b(pre[:32]), 32, _b(m), ln, o)
        assert bytes(o) == hashlib.sha512(pre[:32] + m).digest()
        o2 = _out(32)
        H.cvh_sha256(_b(m), ln, o2)
        assert bytes(o2) == hashlib.sha256(m).digest()
        for shift in (1, 2, 3, 5):                       # unaligned message starts
            buf = (ctypes.c_uint8 * (ln + 16)).from_buffer_copy(bytes(shift) + m + bytes(16 - shift))
            H.cvh_sha512(_b(pre), 64, ctypes.byref(buf, shift), ln, o)
            assert bytes(o) == hashlib.sha512(pre + m).digest()
            H.cvh_sha256(ctypes.byref(buf, shift), ln, o2)
            assert bytes(o2) == hashlib.sha256(m).digest()


def test_verify_logic_on_golden_corpus(host_harness, corpus, manifest):
    H = host_harness
    bad = []
    for i in range(len(corpus["pk"])):
        m = corpus["arena"][corpus["off"][i]:corpus["off"][i] + corpus["len"][i]].tobytes()
        st = ctypes.c_int(0)
        v = H.cvh_verify(_b(corpus["pk"][i].tobytes()), _b(corpus["sig"][i].tobytes()), _b(m), len(m),
                         ctypes.byref(st))
        if v != corpus["verdict"][i] or st.value != corpus["status"][i]:
            bad.append(manifest["classes"][corpus["cls"][i]])
    assert not bad, sorted(set(bad))


def test_keyed_comb_logic_on_golden_corpus(host_harness, corpus, manifest):
    """The per-key comb path (cv_key_prep + cv_keyed_hs + cv_comb_straus: 4 rows of 64-bit digits,
    60 doublings) reproduces every golden verdict, torsion / mixed-order / invalid keys included."""
    H = host_harness
    bad = []
    for i in range(len(corpus["pk"])):
        m = corpus["arena"][corpus["off"][i]:corpus["off"][i] + corpus["len"][i]].tobytes()
        st = ctypes.c_int(0)
        v = H.cvh_verify_keyed(_b(corpus["pk"][i].tobytes()), _b(corpus["sig"][i].tobytes()), _b(m), len(m),
                               ctypes.byref(st))
        if v != corpus["verdict"][i] or st.value != corpus["status"][i]:
            bad.append(manifest["classes"][corpus["cls"][i]])
    assert not bad, sorted(set(bad))


def test_sign_logic_matches_oracle(host_harness):
    H = host_harness
    rng = random.Random(8)
    for i in range(12):
        seed = bytes(rng.randrange(256) for _ in range(32))
        m = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 320)))
        pk, sg = _out(32), _out(64)
        H.cvh_sign(_b(seed), _b(m), len(m), pk, sg)
        assert bytes(pk) == E.public_key_of(seed)
        assert bytes(sg) == E.sign(seed, m)


def test_merkle_logic(host_harness, merkle_cases):
    import hashlib
    H = host_harness
    m = merkle_cases
    for t in range(len(m["ids"])):
        b, e = int(m["tx_leaf_begin"][t]), int(m["tx_leaf_begin"][t + 1])
        leaves = b"".join(hashlib.sha256(m["arena"][m["leaf_off"][k]:m["leaf_off"][k] + m["leaf_len"][k]].tobytes())
                          .digest() for k in range(b, e))
        o = _out(32)
        ok = H.cvh_merkle_root(_b(leaves), e - b, o)
        assert ok == (1 - int(m["status"][t]))
        if ok:
            assert bytes(o) == m["ids"][t].tobytes()


def test_verify_batch_logic_chunks(host_harness, corpus, manifest):
    """prep + straus + chunked finish (Montgomery batch inversion over 8 signatures per lane, invalid
    keys mixed into the chunks, ragged tail) reproduces every golden verdict."""
    H = host_harness
    rng = np.random.default_rng(0)
    for order in [np.arange(len(corpus["pk"])), rng.permutation(len(corpus["pk"]))[:613]]:
        n = order.size
        pk = np.ascontiguousarray(corpus["pk"][order])
        sig = np.ascontiguousarray(corpus["sig"][order])
        off = np.ascontiguousarray(corpus["off"][order])
        ln = np.ascontiguousarray(corpus["len"][order])
        arena = np.concatenate([corpus["arena"], np.zeros(16, np.uint8)])
        verdict = np.zeros(n, np.uint8)
        status = np.zeros(n, np.uint8)
        vp = ctypes.c_void_p
        H.cvh_verify_batch(ctypes.c_uint32(n), pk.ctypes.data_as(vp), sig.ctypes.data_as(vp), arena.ctypes.data_as(vp),
                           off.ctypes.data_as(vp), ln.ctypes.data_as(vp), verdict.ctypes.data_as(vp),
                           status.ctypes.data_as(vp))
        assert np.array_equal(verdict, corpus["verdict"][order])
        assert np.array_equal(status, corpus["status"][order])


@pytest.fixture(params=[0.0, 2.0 ** -26, -(2.0 ** -26), 2.0 ** -12, -(2.0 ** -12)],
                ids=["exact_div", "rcp+2^-26", "rcp-2^-26", "rcp+2^-12", "rcp-2^-12"])
def rcp(host_harness, request):
    """the device computes the lattice quotients with v_rcp_f64 + two Newton steps (cv_qdiv), the
    host build with an exact division; these runs emulate the device sequence on the host from initial
    reciprocals far worse than the hardware's (relative error 2^-26 and 2^-12, both signs)."""
    host_harness.cvh_set_rcp_emulation.argtypes = [ctypes.c_double]
    host_harness.cvh_set_rcp_emulation(request.param)
    yield request.param
    host_harness.cvh_set_rcp_emulation(0.0)


def test_exact_loop_quotients_just_below_integers(host_harness, rcp):
    """The exact loop's quotient step (cv_exact_quotient + cv_submul8) on r0 = k r1 - d with d tiny (the true
    quotient just below the integer k, where a rounded-up estimate would underflow the remainder), r0 = k r1
    exactly, and random pairs: q <= floor(r0 / r1) always (the remainder never wraps), and q is at most one
    short of it for quotients below 2^32."""
    H = host_harness
    H.cvh_exact_step.restype = ctypes.c_uint32
    rng = random.Random(99 + int(rcp * 2 ** 30))
    cases = []
    for _ in range(4000):
        r1 = rng.randrange(2 ** 128, 2 ** rng.randrange(129, 225))
        k = rng.choice([1, 2, 3, rng.randrange(2, 2 ** 32), 2 ** 32 - 1, 2 ** rng.randrange(1, 32)])
        for d in (0, 1, 2, rng.randrange(1, 2 ** 20), -1, -rng.randrange(1, 2 ** 20)):
            r0 = k * r1 - d
            if r1 <= r0 < 2 ** 256:
                cases.append((r0, r1))
    for r0, r1 in cases:
        out = _out(32)
        q = H.cvh_exact_step(_b(r0.to_bytes(32, "little")), _b(r1.to_bytes(32, "little")), out)
        rem = int.from_bytes(bytes(out), "little")
        true_q = r0 // r1
        assert 1 <= q <= true_q, (r0, r1, q, true_q)
        assert rem == r0 - q * r1
        if true_q < 2 ** 32:
            assert true_q - q <= 1 and rem < 2 * r1


def test_halfsize_lattice_properties(host_harness, rcp):
    """sc_halfsize: u = v h (mod 8L), v odd, w = -v s (mod L), |u|, |v| < 16^nwin; the fallback
    (h, 1) only when no short odd-v vector exists.  Random h, s plus edge scalars; with the exact division
    and with the device's reciprocal sequence emulated (rcp)."""
    H = host_harness
    rng = random.Random(7)
    cases = [(0, 0), (1, 5), (L - 1, L - 1), (2**128 - 1, 3), (2**128, 1), (2**252, 7), (8, 9)]
    cases += [(rng.randrange(L), rng.randrange(L)) for _ in range(3000)]
    wins = []
    fallbacks = 0
    for ci, (h, s) in enumerate(cases):
        out = _out(96)
        vn, nw = ctypes.c_int(0), ctypes.c_int(0)
        ok = H.cvh_halfsize(_b(h.to_bytes(32, "little")), _b(s.to_bytes(32, "little")), out, ctypes.byref(vn),
                            ctypes.byref(nw))
        o = bytes(out)
        u, va, w = (int.from_bytes(o[32 * k:32 * k + 32], "little") for k in range(3))
        v = -va if vn.value else va
        assert v % 2 == 1
        assert (u - v * h) % (8 * L) == 0
        assert w == (-v * s) % L
        assert u >= 0 and max(u, va) < 16 ** nw.value
        if ok:
            assert nw.value <= 36
            wins.append(nw.value)
        else:
            fallbacks += 1
            assert ci < 7, "fallback on a random scalar"    # only degenerate edge lattices fall back
            assert (u, v, nw.value) == (h, 1, 64)
    assert fallbacks <= 3
    assert sum(wins) / len(wins) < 34.0


def test_halfsize_verify_logic_on_golden_corpus(host_harness, corpus, manifest):
    """The half-size verify ([v]R + [u]A + [w]B == O with canonical R decoding) reproduces every
    golden verdict: non-canonical / off-curve / small-order R, torsion keys, S >= L, carry loss."""
    H = host_harness
    bad = []
    sc = (ctypes.c_uint32 * 73)()          # CV_HS_DIGWORDS
    for i in range(len(corpus["pk"])):
        m = corpus["arena"][corpus["off"][i]:corpus["off"][i] + corpus["len"][i]].tobytes()
        st = ctypes.c_int(0)
        v = H.cvh_verify_hs(_b(corpus["pk"][i].tobytes()), _b(corpus["sig"][i].tobytes()), _b(m), len(m),
                            ctypes.byref(st), sc)
        if v != corpus["verdict"][i] or st.value != corpus["status"][i]:
            bad.append(manifest["classes"][corpus["cls"][i]])
    assert not bad, sorted(set(bad))


@pytest.mark.parametrize("lat", [0, 1])
def test_fused_halfsize_prep_logic_on_golden_corpus(host_harness, corpus, manifest, lat):
    """The fused prep (hash, lattice, A and R decoded as one interleaved pair, both tables; lat = the
    latency field forms of small batches) + the half-size Straus reproduce every golden verdict."""
    H = host_harness
    bad = []
    for i in range(len(corpus["pk"])):
        m = corpus["arena"][corpus["off"][i]:corpus["off"][i] + corpus["len"][i]].tobytes()
        st = ctypes.c_int(0)
        v = H.cvh_verify_hs_fused(_b(corpus["pk"][i].tobytes()), _b(corpus["sig"][i].tobytes()), _b(m), len(m),
                                  ctypes.byref(st), lat)
        if v != corpus["verdict"][i] or st.value != corpus["status"][i]:
            bad.append(manifest["classes"][corpus["cls"][i]])
    assert not bad, sorted(set(bad))


def test_slide_replay_structured(host_harness):
    """The word-skipping slide() replay (cv_scalar.h) against the literal oracle on structured
    scalars: all-ones with one hole at every position, a top bit over low runs of every length,
    sparse words with the top bit set, and alternating patterns."""
    H = host_harness
    full = (1 << 256) - 1
    cases = [full ^ (1 << k) for k in range(256)]
    cases += [(1 << 255) | ((1 << k) - 1) for k in range(256)]
    cases += [(1 << 255) | (((1 << 20) - 1) << k) for k in range(0, 235, 7)]
    cases += [(1 << 255) | (1 << k) | (1 << (k + 7)) for k in range(0, 240, 5)]
    cases += [int("10" * 128, 2), int("01" * 128, 2) | (1 << 255), int("1110" * 64, 2), int("1000001" * 36, 2) | (1 << 255)]
    rng = random.Random(11)
    for _ in range(300):
        s = (1 << 255) | rng.getrandbits(255)
        s &= ~(rng.getrandbits(256) & rng.getrandbits(256))      # sparse holes
        cases.append(s | (1 << 255))
    cases += [(1 << 255) | rng.getrandbits(255) for _ in range(3000)]      # dense random
    for s in cases:
        sb = (s & full).to_bytes(32, "little")
        assert H.cvh_slide_drops(_b(sb)) == int(E.slide_drops_carry(sb)), hex(s)


def test_tri_digit_words(host_harness, rcp):
    """The tri form's 64 window words from the rolled constant-shift recoding equal the digit16 definition
    (and word 64 the window count) for random (h, s), the degenerate lattices that fall back to (h, 1) with
    64 windows, and scalars whose nibbles sit at the recoding's edges (all ones, alternating, top bits)."""
    H = host_harness
    H.cvh_tri_digit_words_mismatch.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    rng = random.Random(2024)
    L = 2**252 + 27742317777372353535851937790883648493
    hs = [0, 1, 2**128, 2**252, L - 1, 2**253 - 1, int("8" * 63, 16) % L, int("7" * 63, 16) % L]
    hs += [rng.randrange(L) for _ in range(2000)]
    for i, h in enumerate(hs):
        s = rng.randrange(L) if i % 3 else (L - 1 - i)
        assert H.cvh_tri_digit_words_mismatch(h.to_bytes(32, "little"), s.to_bytes(32, "little")) == 0, (hex(h), hex(s))


def test_split_odd_multiple_tables(host_harness, corpus):
    """The latency prep's four-lanes-per-signature form builds each point's 9-entry table k*P in two
    halves (entries 0,1,3,5,7 and 2,4,6,8, the same instruction stream on both lanes): every entry of
    the halves is the same point as the one-lane table's (projectively: (Y+X)/Z, (Y-X)/Z, 2dT/Z, Z != 0)
    and the decode flags agree, for every golden key and R (valid, non-canonical, small-order,
    undecodable -> identity) and 200 random encodings."""
    host_harness.cvh_table_split_mismatch.argtypes = [ctypes.c_char_p, ctypes.c_int]
    encs = [(bytes(corpus["pk"][i]), 0) for i in range(len(corpus["pk"]))]
    encs += [(bytes(corpus["sig"][i][:32]), 1) for i in range(len(corpus["sig"]))]
    rng = np.random.default_rng(77)
    encs += [(rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), int(k & 1)) for k in range(200)]
    bad = [(e.hex(), r) for e, r in encs if host_harness.cvh_table_split_mismatch(e, r) != 0]
    assert not bad, bad[:5]



def test_tx_sig_refs_and_verdicts(host_harness):
    """cv_verify_transactions' per-lane logic (cv_tx_of_sig, cv_tx_all_valid in cv_verify.h, the bodies of
    cv_tx_sig_refs_kernel / cv_tx_verdict_kernel): on ragged signature lists with runs of empty transactions,
    every signature maps to the transaction whose range holds it (numpy searchsorted), and a transaction's
    verdict is "at least one signature, all bits set" — equal to the host ABI's cv_tx_verdicts."""
    from corda_amd import native
    h = host_harness
    u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
    u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
    h.cvh_tx_of_sig.argtypes = [ctypes.c_uint32, ctypes.c_uint32, u32p]
    h.cvh_tx_of_sig.restype = ctypes.c_uint32
    h.cvh_tx_all_valid.argtypes = [ctypes.c_uint32, ctypes.c_uint32, u64p]
    rng = np.random.default_rng(81)
    for nt, maxs in ((1, 5), (7, 3), (300, 70), (2000, 9)):
        counts = rng.integers(0, maxs + 1, nt)
        counts[rng.random(nt) < 0.3] = 0                         # runs of transactions without signatures
        counts[-1] = max(counts[-1], 1)
        tsb = np.zeros(nt + 1, np.uint32)
        tsb[1:] = np.cumsum(counts)
        ns = int(tsb[-1])
        want = np.searchsorted(tsb, np.arange(ns), side="right") - 1
        got = np.array([h.cvh_tx_of_sig(g, nt, tsb) for g in range(ns)])
        assert np.array_equal(got, want), nt
        bits = rng.random(ns) < 0.98
        words = np.zeros((ns + 63) // 64, np.uint64)
        for j in np.nonzero(bits)[0]:
            words[j // 64] |= np.uint64(1) << np.uint64(j % 64)
        ok = np.array([h.cvh_tx_all_valid(int(tsb[t]), int(tsb[t + 1]), words) for t in range(nt)], np.uint8)
        ref = np.array([int(counts[t] > 0 and bits[tsb[t]:tsb[t + 1]].all()) for t in range(nt)], np.uint8)
        assert np.array_equal(ok, ref) and 0 < ref.sum()
        assert np.array_equal(ok, native.tx_verdicts(words, tsb))


def test_limb_bounds_on_max_limb_encodings(host_harness):
    """fe_sub computes |k p_i - g_i| + f_i, which equals f + k p - g only while every limb
    g_i <= k p_i, so that bound is exact, not slack.  The checking build (CV_BOUNDS_CHECK: every fe_sub /
    fe_sub_carry_even asserts g_i <= k p_i and every multiply its column bound, aborting on a violation) runs
    every verify form — half-size, fused prep in both field forms, full width, keyed comb — over encodings whose
    limbs sit at their maxima: keys and R with y in [2^255 - 64, 2^255) (non-canonical y >= p included) and
    y = 2^255 - 2^j, both sign bits; S at 2^256 - 1, 2^255 and around L; verdicts and key status equal the
    oracle's."""
    H = host_harness
    rng = random.Random(20261018)
    ys = [(1 << 255) - 1 - k for k in range(64)] + [(1 << 255) - (1 << j) for j in range(1, 255, 7)]
    encs = []
    for y in ys:
        for sign in (0, 1):
            e = (y | (sign << 255)).to_bytes(32, "little")
            try:
                E.decode_point_0_1_0(e)
                encs.append(e)
            except Exception:
                pass
    assert len(encs) >= 40
    svals = [(1 << 256) - 1, 1 << 255, (1 << 255) + 12345, L, L - 1, L + 1, (1 << 253) + rng.getrandbits(200)]
    cases = []
    for _ in range(160):
        pk, r = rng.choice(encs), rng.choice(encs)
        s = rng.choice(svals)
        cases.append((pk, r + s.to_bytes(32, "little"), rng.randbytes(rng.choice([0, 32, 300]))))
    # the same max-limb R over a real key, and honest signatures rewritten to the non-canonical key encoding
    seed = bytes(range(32))
    pk_h = E.public_key_of(seed)
    for r in encs[:24]:
        cases.append((pk_h, r + ((1 << 256) - 1).to_bytes(32, "little"), b"corda"))
    bad = []
    sc = (ctypes.c_uint32 * 73)()
    for pk, sig, m in cases:
        st_ref, ok_ref = E.verify_ex(pk, m, sig)
        want = (1 if (st_ref == 0 and ok_ref) else 0, 0 if st_ref == 0 else 1)
        for form in ("hs", "fused0", "fused1", "full", "keyed"):
            st = ctypes.c_int(0)
            if form == "hs":
                v = H.cvh_verify_hs(_b(pk), _b(sig), _b(m), len(m), ctypes.byref(st), sc)
            elif form.startswith("fused"):
                v = H.cvh_verify_hs_fused(_b(pk), _b(sig), _b(m), len(m), ctypes.byref(st), int(form[-1]))
            elif form == "full":
                v = H.cvh_verify(_b(pk), _b(sig), _b(m), len(m), ctypes.byref(st))
            else:
                v = H.cvh_verify_keyed(_b(pk), _b(sig), _b(m), len(m), ctypes.byref(st))
            if (v, st.value) != want:
                bad.append((form, pk.hex()[:16], sig.hex()[:16], (v, st.value), want))
    assert not bad, bad[:8]
