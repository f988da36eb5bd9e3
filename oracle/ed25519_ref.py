"""CPU restatement of `net.i2p.crypto:eddsa:0.1.0` Ed25519 verification (pure Python, big ints).

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (`corda_amd/`) may import this module;
only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg use it, as the checker.

What it restates
----------------
The reference verifies every signature through
    PublicKey.verifyWithECDSA(content, sig)        core/src/main/kotlin/net/corda/core/crypto/CryptoUtilities.kt:90-96
        EdDSAEngine().initVerify(key); update(content); verify(sig.bytes)
with the external jar `net.i2p.crypto:eddsa:0.1.0` pinned at core/build.gradle:80 (not vendored in
the reference).  Keys reach the engine as `EdDSAPublicKey(EdDSAPublicKeySpec(bytes, ed25519Curve))`
(core/src/main/kotlin/net/corda/core/serialization/Kryo.kt:300-303, CryptoUtilities.kt:77,126-128).

The eddsa-0.1.0 semantics restated here ("EdDSAEngine 0.1.0 verify semantics"):
  1. sig length != 64            -> SignatureException ("signature length is wrong")
  2. key decode (GroupElement(curve, bytes)):
       y = low 255 bits, NOT reduced mod p (y in [p, 2^255) accepted as y mod p);
       x = (u v^3)(u v^7)^((p-5)/8), fixed by sqrt(-1) if v x^2 == -u, else IllegalArgumentException;
       if isNegative(x) != bit255: x = -x      (x == 0 with sign bit 1 is accepted)
  3. Abyte = A.toByteArray()  (canonical re-encoding; used in the hash)
  4. h = SHA-512(R || Abyte || M) mod L
  5. S = sig[32:64] raw, no S < L check
  6. R' = B.doubleScalarMultiplyVariableTime(-A, h, S) using ref10 slide() recoding; slide drops a
     carry out of bit 255, so the effective scalar is S - 2^256 in that case
  7. accept iff R'.toByteArray() == sig[0:32] byte for byte (cofactorless, no small-order checks)

Parity status: the honest-path behaviour is pinned by RFC 8032 vectors and by OpenSSL/node Ed25519
(tests/golden/make_golden.py cross-checks).  Edge-case behaviour (non-canonical, small-order, S >= L,
carry loss) is "parity unpinned" by the reference's own tests: it follows the
recalled 0.1.0 source as listed above.
"""
from __future__ import annotations

import hashlib
from typing import Optional, Tuple

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
D2 = (2 * D) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)

# status codes (mirror include/cordaverify.h CV_SIG_*)
ST_OK = 0
ST_BAD_KEY = 1       # IllegalArgumentException("not a valid GroupElement") at key construction
ST_BAD_SIG_LEN = 2   # SignatureException("signature length is wrong")
ST_BAD_KEY_LEN = 3   # IllegalArgumentException("public-key length is wrong")


class InvalidKeyError(ValueError):
    pass


# ---------------------------------------------------------------- field helpers
def _inv(x: int) -> int:
    return pow(x, P - 2, P)


def _is_negative(x: int) -> int:
    """FieldElement.isNegative(): low bit of the canonical encoding."""
    return (x % P) & 1


# ---------------------------------------------------------------- points (extended coords, exact)
# A point is (X, Y, Z, T) with x = X/Z, y = Y/Z, xy = T/Z.  The a=-1 twisted Edwards unified
# addition is complete on the whole curve (d non-square), so these give exact group arithmetic for
# every point including torsion points.
IDENT = (0, 1, 1, 0)


def pt_add(p, q):
    X1, Y1, Z1, T1 = p
    X2, Y2, Z2, T2 = q
    a = (Y1 - X1) * (Y2 - X2) % P
    b = (Y1 + X1) * (Y2 + X2) % P
    c = T1 * D2 % P * T2 % P
    d = Z1 * 2 * Z2 % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def pt_dbl(p):
    return pt_add(p, p)


def pt_neg(p):
    X, Y, Z, T = p
    return ((-X) % P, Y, Z, (-T) % P)


def pt_from_affine(x, y):
    return (x % P, y % P, 1, x * y % P)


def pt_affine(p):
    X, Y, Z, _ = p
    zi = _inv(Z)
    return (X * zi % P, Y * zi % P)


def pt_encode(p) -> bytes:
    """GroupElement.toByteArray(): canonical y, sign of x in bit 255."""
    x, y = pt_affine(p)
    s = bytearray(y.to_bytes(32, "little"))
    s[31] |= (x & 1) << 7
    return bytes(s)


def pt_eq(p, q) -> bool:
    return pt_affine(p) == pt_affine(q)


def pt_mul(k: int, p):
    """[k]p for k >= 0 by plain double-and-add (exact)."""
    r = IDENT
    q = p
    while k:
        if k & 1:
            r = pt_add(r, q)
        q = pt_dbl(q)
        k >>= 1
    return r


_BY = 4 * _inv(5) % P


def _recover_x_std(y: int, sign: int) -> int:
    xx = (y * y - 1) * _inv(D * y * y + 1) % P
    x = pow(xx, (P + 3) // 8, P)
    if (x * x - xx) % P != 0:
        x = x * SQRT_M1 % P
    if (x & 1) != sign:
        x = P - x
    return x


BASE = pt_from_affine(_recover_x_std(_BY, 0), _BY)


# ---------------------------------------------------------------- eddsa-0.1.0 key decode
def decode_point_0_1_0(s: bytes):
    """GroupElement(Curve, byte[]) of eddsa 0.1.0 (raises InvalidKeyError)."""
    if len(s) != 32:
        raise InvalidKeyError("public-key length is wrong")
    y_raw = int.from_bytes(s, "little") & ((1 << 255) - 1)      # bit 255 masked, NOT reduced
    y = y_raw % P
    yy = y * y % P
    u = (yy - 1) % P
    v = (yy * D + 1) % P
    v3 = v * v % P * v % P
    x = v3 * v3 % P * v % P * u % P                              # u v^7
    x = pow(x, (P - 5) // 8, P)                                  # pow22523
    x = v3 * u % P * x % P
    vxx = x * x % P * v % P
    if (vxx - u) % P != 0:
        if (vxx + u) % P != 0:
            raise InvalidKeyError("not a valid GroupElement")
        x = x * SQRT_M1 % P
    if _is_negative(x) != (s[31] >> 7) & 1:
        x = (-x) % P
    return pt_from_affine(x, y)


# ---------------------------------------------------------------- ref10 slide (GroupElement.slide)
def slide(a: bytes):
    r = [(a[i >> 3] >> (i & 7)) & 1 for i in range(256)]
    for i in range(256):
        if r[i]:
            b = 1
            while b <= 6 and i + b < 256:
                if r[i + b]:
                    if r[i] + (r[i + b] << b) <= 15:
                        r[i] += r[i + b] << b
                        r[i + b] = 0
                    elif r[i] - (r[i + b] << b) >= -15:
                        r[i] -= r[i + b] << b
                        for k in range(i + b, 256):
                            if not r[k]:
                                r[k] = 1
                                break
                            r[k] = 0
                    else:
                        break
                b += 1
    return r


def slide_value(a: bytes) -> int:
    """Integer value the slide digits represent (S, or S - 2^256 when the top carry is dropped)."""
    return sum(d << i for i, d in enumerate(slide(a)))


def slide_drops_carry(a: bytes) -> bool:
    return slide_value(a) != int.from_bytes(a, "little")


def _odd_multiples(p):
    """dblPrecmp: [1,3,5,...,15]·p"""
    p2 = pt_dbl(p)
    out = [p]
    for _ in range(7):
        out.append(pt_add(out[-1], p2))
    return out


_BASE_ODD = _odd_multiples(BASE)


def double_scalar_mult_vartime(neg_a, a_scalar: bytes, b_scalar: bytes):
    """GroupElement.doubleScalarMultiplyVariableTime(A, a, b) with this = B: [a]A + [b]B, literal."""
    aslide = slide(a_scalar)
    bslide = slide(b_scalar)
    a_tab = _odd_multiples(neg_a)
    r = IDENT
    i = 255
    while i >= 0 and aslide[i] == 0 and bslide[i] == 0:
        i -= 1
    while i >= 0:
        r = pt_dbl(r)
        if aslide[i] > 0:
            r = pt_add(r, a_tab[aslide[i] // 2])
        elif aslide[i] < 0:
            r = pt_add(r, pt_neg(a_tab[(-aslide[i]) // 2]))
        if bslide[i] > 0:
            r = pt_add(r, _BASE_ODD[bslide[i] // 2])
        elif bslide[i] < 0:
            r = pt_add(r, pt_neg(_BASE_ODD[(-bslide[i]) // 2]))
        i -= 1
    return r


# ---------------------------------------------------------------- verify (EdDSAEngine.engineVerify)
def sc_reduce(h64: bytes) -> bytes:
    return (int.from_bytes(h64, "little") % L).to_bytes(32, "little")


def verify_ex(pk: bytes, msg: bytes, sig: bytes, literal: bool = True) -> Tuple[int, bool]:
    """Returns (status, accepted).  status != ST_OK means the reference throws instead of returning."""
    if len(pk) != 32:
        return ST_BAD_KEY_LEN, False
    try:
        A = decode_point_0_1_0(pk)
    except InvalidKeyError:
        return ST_BAD_KEY, False
    if len(sig) != 64:
        return ST_BAD_SIG_LEN, False
    abyte = pt_encode(A)
    h = sc_reduce(hashlib.sha512(sig[:32] + abyte + msg).digest())
    s = sig[32:64]
    neg_a = pt_neg(A)
    if literal:
        r = double_scalar_mult_vartime(neg_a, h, s)
    else:
        r = pt_add(pt_mul(int.from_bytes(h, "little"), neg_a),
                   pt_mul(slide_value(s) % L, BASE))
    return ST_OK, pt_encode(r) == sig[:32]


def verify(pk: bytes, msg: bytes, sig: bytes) -> bool:
    st, ok = verify_ex(pk, msg, sig)
    return st == ST_OK and ok


def abyte_of(pk: bytes) -> bytes:
    """EdDSAPublicKey.getAbyte() for a wire encoding (canonical re-encoding)."""
    return pt_encode(decode_point_0_1_0(pk))


# ---------------------------------------------------------------- signing side (fixtures only)
def seed_to_keypair(seed: bytes):
    """EdDSAPrivateKeySpec(seed, ed25519): h = SHA-512(seed), clamp, A = aB.  Returns (a, prefix, Abyte)."""
    assert len(seed) == 32
    h = bytearray(hashlib.sha512(seed).digest())
    h[0] &= 248
    h[31] &= 63
    h[31] |= 64
    a = int.from_bytes(h[:32], "little")
    return a, bytes(h[32:]), pt_encode(pt_mul(a, BASE))


def sign(seed: bytes, msg: bytes) -> bytes:
    """EdDSAEngine.engineSign (RFC 8032 Ed25519, deterministic)."""
    a, prefix, A = seed_to_keypair(seed)
    r = int.from_bytes(hashlib.sha512(prefix + msg).digest(), "little") % L
    R = pt_encode(pt_mul(r, BASE))
    k = int.from_bytes(hashlib.sha512(R + A + msg).digest(), "little") % L
    S = (r + k * a) % L
    return R + S.to_bytes(32, "little")


def entropy_to_seed(entropy: int) -> bytes:
    """entropyToKeyPair(BigInteger): BigInteger.toByteArray().copyOf(32) (CryptoUtilities.kt:123-130)."""
    if entropy == 0:
        b = b"\x00"
    else:
        n = (entropy.bit_length() + 8) // 8          # two's complement minimal length (sign bit)
        b = entropy.to_bytes(n, "big", signed=True)
    return (b + b"\x00" * 32)[:32]


def public_key_of(seed: bytes) -> bytes:
    return seed_to_keypair(seed)[2]


def point_from_bytes_std(b: bytes):
    """Strict RFC 8032 decode (used only to build adversarial inputs)."""
    y = int.from_bytes(b, "little") & ((1 << 255) - 1)
    return decode_point_0_1_0(b) if y < P else None


# torsion: the 8 points of order dividing 8
def torsion_points():
    # a point of order 8: x^2 = (y^2-1)/(dy^2+1) with y satisfying the order-8 condition; found by
    # multiplying a random curve point by L (clears the prime-order part).
    pts = []
    y = 2
    while True:
        xx = (y * y - 1) * _inv(D * y * y + 1) % P
        x = pow(xx, (P + 3) // 8, P)
        if (x * x - xx) % P != 0:
            x = x * SQRT_M1 % P
        if (x * x - xx) % P == 0:
            q = pt_mul(L, pt_from_affine(x, y))
            # order of q divides 8
            if not pt_eq(pt_mul(4, q), IDENT):      # order exactly 8
                break
        y += 1
    t = IDENT
    for _ in range(8):
        pts.append(t)
        t = pt_add(t, q)
    return pts
