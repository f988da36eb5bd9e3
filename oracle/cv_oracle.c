/*
 * cv_oracle.c — plain-C CPU restatement of the reference's signature-verification hot path.
 *
 * TEST INFRASTRUCTURE ONLY: the checker for the HIP engine and the `cpu_baseline` leg of bench.py.
 * Nothing in corda_amd/ links or loads this library.
 *
 * Restates (see oracle/ed25519_ref.py for the full semantics list and parity status):
 *   - PublicKey.verifyWithECDSA                       core/.../crypto/CryptoUtilities.kt:90-96
 *     -> net.i2p.crypto:eddsa:0.1.0 EdDSAEngine.engineVerify (external, pinned core/build.gradle:80)
 *        key decode GroupElement(curve, bytes) (no y reduction, x=0/sign=1 accepted),
 *        Abyte = canonical re-encoding, h = SHA-512(R||Abyte||M) mod L, S raw (no S<L check),
 *        R' = doubleScalarMultiplyVariableTime(-A, h, S) with ref10 slide() (drops the top carry),
 *        byte compare of R'.toByteArray() with sig[0:32].
 *   - SignedTransaction.checkSignaturesAreValid       core/.../transactions/SignedTransaction.kt:82-87
 *   - WireTransaction.id = MerkleTree root            core/.../transactions/WireTransaction.kt:52,
 *     MerkleTree.getMerkleTree / buildMerkleTree      core/.../transactions/MerkleTransaction.kt:66-99
 *     (sha256(left||right), odd level duplicates the last node, 1 leaf = root, 0 leaves = error)
 *   - SecureHash.sha256                               core/.../crypto/SecureHash.kt:33
 *
 * Arithmetic: radix 2^51 field (5 x 64-bit limbs, unsigned __int128 products) and extended twisted
 * Edwards coordinates — deliberately a different representation from the GPU kernel (radix 2^25.5,
 * fixed-window Straus), so the two are independent implementations of the same semantics.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

typedef unsigned __int128 u128;

/* ============================================================ SHA-2 (FIPS 180-4) */
static const uint64_t K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

static uint64_t ror64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
static uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static void sha512_block(uint64_t st[8], const uint8_t *blk) {
    uint64_t w[80];
    for (int i = 0; i < 16; i++) {
        uint64_t v = 0;
        for (int j = 0; j < 8; j++) v = (v << 8) | blk[8 * i + j];
        w[i] = v;
    }
    for (int i = 16; i < 80; i++) {
        uint64_t s0 = ror64(w[i - 15], 1) ^ ror64(w[i - 15], 8) ^ (w[i - 15] >> 7);
        uint64_t s1 = ror64(w[i - 2], 19) ^ ror64(w[i - 2], 61) ^ (w[i - 2] >> 6);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 80; i++) {
        uint64_t t1 = h + (ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41)) + ((e & f) ^ (~e & g)) + K512[i] + w[i];
        uint64_t t2 = (ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

/* SHA-512 over the concatenation of up to 3 byte strings. */
static void sha512_3(uint8_t out[64], const uint8_t *p1, size_t n1, const uint8_t *p2, size_t n2,
                     const uint8_t *p3, size_t n3) {
    uint64_t st[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                      0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                      0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    uint8_t buf[128];
    size_t fill = 0;
    const uint8_t *ps[3] = {p1, p2, p3};
    size_t ns[3] = {n1, n2, n3};
    uint64_t total = 0;
    for (int k = 0; k < 3; k++) {
        for (size_t i = 0; i < ns[k]; i++) {
            buf[fill++] = ps[k][i];
            if (fill == 128) { sha512_block(st, buf); fill = 0; }
        }
        total += ns[k];
    }
    buf[fill++] = 0x80;
    if (fill > 112) {
        while (fill < 128) buf[fill++] = 0;
        sha512_block(st, buf);
        fill = 0;
    }
    while (fill < 120) buf[fill++] = 0;
    uint64_t bits = total * 8;
    for (int j = 0; j < 8; j++) buf[120 + j] = (uint8_t)(bits >> (56 - 8 * j));
    sha512_block(st, buf);
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t)(st[i] >> (56 - 8 * j));
}

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static void sha256_block(uint32_t st[8], const uint8_t *blk) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) |
               ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ror32(w[i - 15], 7) ^ ror32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ror32(w[i - 2], 17) ^ ror32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
        uint32_t t1 = h + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

void cvo_sha256(uint8_t out[32], const uint8_t *p, size_t n) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                      0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint8_t buf[64];
    size_t i = 0;
    for (; i + 64 <= n; i += 64) sha256_block(st, p + i);
    size_t rem = n - i;
    memcpy(buf, p + i, rem);
    buf[rem++] = 0x80;
    if (rem > 56) {
        while (rem < 64) buf[rem++] = 0;
        sha256_block(st, buf);
        rem = 0;
    }
    while (rem < 56) buf[rem++] = 0;
    uint64_t bits = (uint64_t)n * 8;
    for (int j = 0; j < 8; j++) buf[56 + j] = (uint8_t)(bits >> (56 - 8 * j));
    sha256_block(st, buf);
    for (int k = 0; k < 8; k++)
        for (int j = 0; j < 4; j++) out[4 * k + j] = (uint8_t)(st[k] >> (24 - 8 * j));
}

void cvo_sha512(uint8_t out[64], const uint8_t *p, size_t n) { sha512_3(out, p, n, 0, 0, 0, 0); }

/* ============================================================ GF(2^255-19), radix 2^51 */
typedef struct { uint64_t v[5]; } fe;
#define M51 ((1ULL << 51) - 1)

static void fe_carry(fe *h) {
    uint64_t c;
    for (int r = 0; r < 2; r++) {
        c = h->v[0] >> 51; h->v[0] &= M51; h->v[1] += c;
        c = h->v[1] >> 51; h->v[1] &= M51; h->v[2] += c;
        c = h->v[2] >> 51; h->v[2] &= M51; h->v[3] += c;
        c = h->v[3] >> 51; h->v[3] &= M51; h->v[4] += c;
        c = h->v[4] >> 51; h->v[4] &= M51; h->v[0] += 19 * c;
    }
}
static void fe_0(fe *h) { memset(h, 0, sizeof *h); }
static void fe_1(fe *h) { fe_0(h); h->v[0] = 1; }
static void fe_add(fe *h, const fe *f, const fe *g) {
    for (int i = 0; i < 5; i++) h->v[i] = f->v[i] + g->v[i];
    fe_carry(h);
}
/* f - g + 4p (limbs of f,g < 2^52) */
static void fe_sub(fe *h, const fe *f, const fe *g) {
    static const uint64_t p4[5] = {0x1FFFFFFFFFFFB4ULL, 0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL,
                                   0x1FFFFFFFFFFFFCULL, 0x1FFFFFFFFFFFFCULL};
    for (int i = 0; i < 5; i++) h->v[i] = f->v[i] + p4[i] - g->v[i];
    fe_carry(h);
}
static void fe_neg(fe *h, const fe *f) { fe z; fe_0(&z); fe_sub(h, &z, f); }
static void fe_mul(fe *h, const fe *f, const fe *g) {
    const uint64_t *a = f->v, *b = g->v;
    u128 r0 = (u128)a[0] * b[0] + (u128)(19 * a[1]) * b[4] + (u128)(19 * a[2]) * b[3] +
              (u128)(19 * a[3]) * b[2] + (u128)(19 * a[4]) * b[1];
    u128 r1 = (u128)a[0] * b[1] + (u128)a[1] * b[0] + (u128)(19 * a[2]) * b[4] +
              (u128)(19 * a[3]) * b[3] + (u128)(19 * a[4]) * b[2];
    u128 r2 = (u128)a[0] * b[2] + (u128)a[1] * b[1] + (u128)a[2] * b[0] +
              (u128)(19 * a[3]) * b[4] + (u128)(19 * a[4]) * b[3];
    u128 r3 = (u128)a[0] * b[3] + (u128)a[1] * b[2] + (u128)a[2] * b[1] + (u128)a[3] * b[0] +
              (u128)(19 * a[4]) * b[4];
    u128 r4 = (u128)a[0] * b[4] + (u128)a[1] * b[3] + (u128)a[2] * b[2] + (u128)a[3] * b[1] +
              (u128)a[4] * b[0];
    uint64_t c;
    uint64_t o0 = (uint64_t)r0 & M51; r1 += (uint64_t)(r0 >> 51);
    uint64_t o1 = (uint64_t)r1 & M51; r2 += (uint64_t)(r1 >> 51);
    uint64_t o2 = (uint64_t)r2 & M51; r3 += (uint64_t)(r2 >> 51);
    uint64_t o3 = (uint64_t)r3 & M51; r4 += (uint64_t)(r3 >> 51);
    uint64_t o4 = (uint64_t)r4 & M51; c = (uint64_t)(r4 >> 51);
    u128 t0 = (u128)o0 + (u128)19 * c;
    o0 = (uint64_t)t0 & M51;
    o1 += (uint64_t)(t0 >> 51);
    h->v[0] = o0; h->v[1] = o1; h->v[2] = o2; h->v[3] = o3; h->v[4] = o4;
}
static void fe_sq(fe *h, const fe *f) { fe_mul(h, f, f); }
static void fe_sqn(fe *h, const fe *f, int n) {
    fe_sq(h, f);
    for (int i = 1; i < n; i++) fe_sq(h, h);
}
/* canonical little-endian encoding */
static void fe_tobytes(uint8_t s[32], const fe *f) {
    fe t = *f;
    fe_carry(&t);
    /* t < 2^255 + small; subtract p if t >= p */
    uint64_t q = (t.v[0] + 19) >> 51;
    q = (t.v[1] + q) >> 51;
    q = (t.v[2] + q) >> 51;
    q = (t.v[3] + q) >> 51;
    q = (t.v[4] + q) >> 51;
    t.v[0] += 19 * q;
    uint64_t c;
    c = t.v[0] >> 51; t.v[0] &= M51; t.v[1] += c;
    c = t.v[1] >> 51; t.v[1] &= M51; t.v[2] += c;
    c = t.v[2] >> 51; t.v[2] &= M51; t.v[3] += c;
    c = t.v[3] >> 51; t.v[3] &= M51; t.v[4] += c;
    t.v[4] &= M51;
    uint64_t w[4];
    w[0] = t.v[0] | (t.v[1] << 51);
    w[1] = (t.v[1] >> 13) | (t.v[2] << 38);
    w[2] = (t.v[2] >> 26) | (t.v[3] << 25);
    w[3] = (t.v[3] >> 39) | (t.v[4] << 12);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}
/* low 255 bits, NOT reduced (eddsa 0.1.0 Ed25519LittleEndianEncoding.decode masks bit 255 only) */
static void fe_frombytes(fe *h, const uint8_t s[32]) {
    uint64_t w[4];
    for (int i = 0; i < 4; i++) {
        uint64_t v = 0;
        for (int j = 7; j >= 0; j--) v = (v << 8) | s[8 * i + j];
        w[i] = v;
    }
    h->v[0] = w[0] & M51;
    h->v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
    h->v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
    h->v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
    h->v[4] = (w[3] >> 12) & M51;
}
static int fe_isnonzero(const fe *f) {
    uint8_t s[32];
    fe_tobytes(s, f);
    uint8_t r = 0;
    for (int i = 0; i < 32; i++) r |= s[i];
    return r != 0;
}
static int fe_isnegative(const fe *f) {
    uint8_t s[32];
    fe_tobytes(s, f);
    return s[0] & 1;
}
/* z^(2^252-3) */
static void fe_pow22523(fe *out, const fe *z) {
    fe z2, z9, z11, z_5_0, z_10_0, z_20_0, z_50_0, z_100_0, t;
    fe_sq(&z2, z);
    fe_sqn(&t, &z2, 2);
    fe_mul(&z9, &t, z);
    fe_mul(&z11, &z9, &z2);
    fe_sq(&t, &z11);
    fe_mul(&z_5_0, &t, &z9);
    fe_sqn(&t, &z_5_0, 5);
    fe_mul(&z_10_0, &t, &z_5_0);
    fe_sqn(&t, &z_10_0, 10);
    fe_mul(&z_20_0, &t, &z_10_0);
    fe_sqn(&t, &z_20_0, 20);
    fe_mul(&t, &t, &z_20_0);
    fe_sqn(&t, &t, 10);
    fe_mul(&z_50_0, &t, &z_10_0);
    fe_sqn(&t, &z_50_0, 50);
    fe_mul(&z_100_0, &t, &z_50_0);
    fe_sqn(&t, &z_100_0, 100);
    fe_mul(&t, &t, &z_100_0);
    fe_sqn(&t, &t, 50);
    fe_mul(&t, &t, &z_50_0);
    fe_sqn(&t, &t, 2);
    fe_mul(out, &t, z);
}
/* z^(p-2) = z^(2^255-21) */
static void fe_invert(fe *out, const fe *z) {
    fe t, z3;
    fe_pow22523(&t, z);      /* z^(2^252-3) */
    fe_sqn(&t, &t, 3);       /* z^(2^255-24) */
    fe_sq(&z3, z);
    fe_mul(&z3, &z3, z);     /* z^3 */
    fe_mul(out, &t, &z3);    /* z^(2^255-21) */
}

static fe FE_D, FE_D2, FE_SQRTM1;
static pthread_once_t consts_once = PTHREAD_ONCE_INIT;

static void fe_from_u64s(fe *h, const uint64_t w[4]) {
    uint8_t s[32];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
    fe_frombytes(h, s);
}

/* ============================================================ points */
typedef struct { fe X, Y, Z, T; } ge;

static void ge_ident(ge *r) { fe_0(&r->X); fe_1(&r->Y); fe_1(&r->Z); fe_0(&r->T); }

/* unified a=-1 extended addition (complete for d non-square) */
static void ge_add(ge *r, const ge *p, const ge *q) {
    fe a, b, c, d, e, f, g, h, t;
    fe_sub(&a, &p->Y, &p->X);
    fe_sub(&t, &q->Y, &q->X);
    fe_mul(&a, &a, &t);
    fe_add(&b, &p->Y, &p->X);
    fe_add(&t, &q->Y, &q->X);
    fe_mul(&b, &b, &t);
    fe_mul(&c, &p->T, &q->T);
    fe_mul(&c, &c, &FE_D2);
    fe_mul(&d, &p->Z, &q->Z);
    fe_add(&d, &d, &d);
    fe_sub(&e, &b, &a);
    fe_sub(&f, &d, &c);
    fe_add(&g, &d, &c);
    fe_add(&h, &b, &a);
    fe_mul(&r->X, &e, &f);
    fe_mul(&r->Y, &g, &h);
    fe_mul(&r->Z, &f, &g);
    fe_mul(&r->T, &e, &h);
}
static void ge_neg(ge *r, const ge *p) {
    fe_neg(&r->X, &p->X);
    r->Y = p->Y;
    r->Z = p->Z;
    fe_neg(&r->T, &p->T);
}
static void ge_tobytes(uint8_t s[32], const ge *p) {
    fe zi, x, y;
    fe_invert(&zi, &p->Z);
    fe_mul(&x, &p->X, &zi);
    fe_mul(&y, &p->Y, &zi);
    fe_tobytes(s, &y);
    s[31] |= (uint8_t)(fe_isnegative(&x) << 7);
}

static ge GE_B;
static ge GE_B_ODD[8];

static void odd_multiples(ge out[8], const ge *p) {
    ge p2;
    ge_add(&p2, p, p);
    out[0] = *p;
    for (int i = 1; i < 8; i++) ge_add(&out[i], &out[i - 1], &p2);
}

static void init_consts(void) {
    /* d = -121665/121666, 2d, sqrt(-1), basepoint: canonical little-endian 64-bit words */
    static const uint64_t d_w[4] = {0x75eb4dca135978a3ULL, 0x00700a4d4141d8abULL,
                                    0x8cc740797779e898ULL, 0x52036cee2b6ffe73ULL};
    static const uint64_t i_w[4] = {0xc4ee1b274a0ea0b0ULL, 0x2f431806ad2fe478ULL,
                                    0x2b4d00993dfbd7a7ULL, 0x2b8324804fc1df0bULL};
    static const uint64_t bx_w[4] = {0xc9562d608f25d51aULL, 0x692cc7609525a7b2ULL,
                                     0xc0a4e231fdd6dc5cULL, 0x216936d3cd6e53feULL};
    static const uint64_t by_w[4] = {0x6666666666666658ULL, 0x6666666666666666ULL,
                                     0x6666666666666666ULL, 0x6666666666666666ULL};
    fe_from_u64s(&FE_D, d_w);
    fe_add(&FE_D2, &FE_D, &FE_D);
    fe_from_u64s(&FE_SQRTM1, i_w);
    fe_from_u64s(&GE_B.X, bx_w);
    fe_from_u64s(&GE_B.Y, by_w);
    fe_1(&GE_B.Z);
    fe_mul(&GE_B.T, &GE_B.X, &GE_B.Y);
    odd_multiples(GE_B_ODD, &GE_B);
}

/* eddsa 0.1.0 GroupElement(curve, bytes); returns 0 on success, -1 for "not a valid GroupElement" */
static int ge_decode_0_1_0(ge *A, const uint8_t s[32]) {
    fe y, yy, u, v, v3, x, vxx, chk;
    fe_frombytes(&y, s);
    fe_sq(&yy, &y);
    fe one;
    fe_1(&one);
    fe_sub(&u, &yy, &one);
    fe_mul(&v, &yy, &FE_D);
    fe_add(&v, &v, &one);
    fe_sq(&v3, &v);
    fe_mul(&v3, &v3, &v);
    fe_sq(&x, &v3);
    fe_mul(&x, &x, &v);
    fe_mul(&x, &x, &u);
    fe_pow22523(&x, &x);
    fe_mul(&x, &x, &v3);
    fe_mul(&x, &x, &u);
    fe_sq(&vxx, &x);
    fe_mul(&vxx, &vxx, &v);
    fe_sub(&chk, &vxx, &u);
    if (fe_isnonzero(&chk)) {
        fe_add(&chk, &vxx, &u);
        if (fe_isnonzero(&chk)) return -1;
        fe_mul(&x, &x, &FE_SQRTM1);
    }
    if (fe_isnegative(&x) != ((s[31] >> 7) & 1)) fe_neg(&x, &x);
    A->X = x;
    A->Y = y;
    fe_1(&A->Z);
    fe_mul(&A->T, &x, &y);
    return 0;
}

/* ref10 slide(), as GroupElement.slide in eddsa 0.1.0 */
static void slide(signed char r[256], const uint8_t a[32]) {
    for (int i = 0; i < 256; i++) r[i] = 1 & (a[i >> 3] >> (i & 7));
    for (int i = 0; i < 256; i++) {
        if (!r[i]) continue;
        for (int b = 1; b <= 6 && i + b < 256; b++) {
            if (!r[i + b]) continue;
            if (r[i] + (r[i + b] << b) <= 15) {
                r[i] = (signed char)(r[i] + (r[i + b] << b));
                r[i + b] = 0;
            } else if (r[i] - (r[i + b] << b) >= -15) {
                r[i] = (signed char)(r[i] - (r[i + b] << b));
                for (int k = i + b; k < 256; k++) {
                    if (!r[k]) { r[k] = 1; break; }
                    r[k] = 0;
                }
            } else {
                break;
            }
        }
    }
}

/* sc_reduce: 64-byte little-endian integer mod L (schoolbook long division on 32-bit words) */
static void sc_reduce64(uint8_t out[32], const uint8_t in[64]) {
    static const uint32_t Lw[8] = {0x5cf5d3ed, 0x5812631a, 0xa2f79cd6, 0x14def9de,
                                   0x00000000, 0x00000000, 0x00000000, 0x10000000};
    uint32_t x[17] = {0};
    for (int i = 0; i < 16; i++)
        x[i] = (uint32_t)in[4 * i] | ((uint32_t)in[4 * i + 1] << 8) | ((uint32_t)in[4 * i + 2] << 16) |
               ((uint32_t)in[4 * i + 3] << 24);
    /* bitwise restoring reduction from the top: r = (r*2 + bit) mod L, 512 steps */
    uint32_t r[9] = {0};
    for (int bit = 511; bit >= 0; bit--) {
        uint32_t carry = (x[bit >> 5] >> (bit & 31)) & 1;
        for (int i = 0; i < 9; i++) {
            uint32_t nc = r[i] >> 31;
            r[i] = (r[i] << 1) | carry;
            carry = nc;
        }
        /* if r >= L: r -= L */
        int ge = 1;
        for (int i = 8; i >= 0; i--) {
            uint32_t li = i < 8 ? Lw[i] : 0;
            if (r[i] != li) { ge = r[i] > li; break; }
        }
        if (ge) {
            uint64_t br = 0;
            for (int i = 0; i < 9; i++) {
                uint64_t li = i < 8 ? Lw[i] : 0;
                uint64_t t = (uint64_t)r[i] - li - br;
                r[i] = (uint32_t)t;
                br = (t >> 63) & 1;
            }
        }
    }
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(r[i] >> (8 * j));
}

enum { CVO_OK = 0, CVO_BAD_KEY = 1 };

/* Returns status (0 ok, 1 bad key encoding); *accept = verdict. */
int cvo_verify(const uint8_t pk[32], const uint8_t sig[64], const uint8_t *msg, size_t mlen, int *accept) {
    pthread_once(&consts_once, init_consts);
    *accept = 0;
    ge A;
    if (ge_decode_0_1_0(&A, pk) != 0) return CVO_BAD_KEY;
    uint8_t abyte[32], hfull[64], h[32];
    ge_tobytes(abyte, &A);
    sha512_3(hfull, sig, 32, abyte, 32, msg, mlen);
    sc_reduce64(h, hfull);
    ge negA, atab[8];
    ge_neg(&negA, &A);
    odd_multiples(atab, &negA);
    signed char as[256], bs[256];
    slide(as, h);
    slide(bs, sig + 32);
    int i = 255;
    while (i >= 0 && !as[i] && !bs[i]) i--;
    ge r, t;
    ge_ident(&r);
    for (; i >= 0; i--) {
        ge_add(&r, &r, &r);
        if (as[i] > 0) ge_add(&r, &r, &atab[as[i] / 2]);
        else if (as[i] < 0) { ge_neg(&t, &atab[(-as[i]) / 2]); ge_add(&r, &r, &t); }
        if (bs[i] > 0) ge_add(&r, &r, &GE_B_ODD[bs[i] / 2]);
        else if (bs[i] < 0) { ge_neg(&t, &GE_B_ODD[(-bs[i]) / 2]); ge_add(&r, &r, &t); }
    }
    uint8_t rc[32];
    ge_tobytes(rc, &r);
    *accept = memcmp(rc, sig, 32) == 0;
    return CVO_OK;
}

/* canonical re-encoding of a wire key (EdDSAPublicKey.getAbyte); returns status */
int cvo_abyte(const uint8_t pk[32], uint8_t abyte[32]) {
    pthread_once(&consts_once, init_consts);
    ge A;
    if (ge_decode_0_1_0(&A, pk) != 0) return CVO_BAD_KEY;
    ge_tobytes(abyte, &A);
    return CVO_OK;
}

/* ============================================================ batch + threads */
typedef struct {
    size_t begin, end;
    const uint8_t *pk, *sig, *arena;
    const uint64_t *off;
    const uint32_t *len;
    uint8_t *verdict, *status;
} vjob;

static void *vworker(void *arg) {
    vjob *j = (vjob *)arg;
    for (size_t i = j->begin; i < j->end; i++) {
        int ok = 0;
        int st = cvo_verify(j->pk + 32 * i, j->sig + 64 * i, j->arena + j->off[i], j->len[i], &ok);
        j->verdict[i] = (uint8_t)ok;
        if (j->status) j->status[i] = (uint8_t)st;
    }
    return 0;
}

/* verdict[i] in {0,1} (one byte per signature), status optional.  nthreads >= 1. */
int cvo_verify_batch(size_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                     const uint64_t *off, const uint32_t *len, uint8_t *verdict, uint8_t *status,
                     int nthreads) {
    pthread_once(&consts_once, init_consts);
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > n) nthreads = n ? (int)n : 1;
    pthread_t th[256];
    vjob jobs[256];
    if (nthreads > 256) nthreads = 256;
    size_t per = (n + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        size_t b = per * t, e = b + per;
        if (b > n) b = n;
        if (e > n) e = n;
        jobs[t] = (vjob){b, e, pk, sig, arena, off, len, verdict, status};
        if (nthreads == 1) vworker(&jobs[t]);
        else pthread_create(&th[t], 0, vworker, &jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], 0);
    return 0;
}

/* ============================================================ Merkle tx ids */
/* Returns per-tx status: 0 ok, 1 empty leaf list (MerkleTreeException). */
int cvo_merkle_root(const uint8_t *leaf_hashes, size_t nleaves, uint8_t root[32]) {
    if (nleaves == 0) return 1;
    uint8_t *lvl = (uint8_t *)malloc(32 * nleaves);
    memcpy(lvl, leaf_hashes, 32 * nleaves);
    size_t n = nleaves;
    while (n > 1) {
        size_t m = (n + 1) / 2;
        for (size_t i = 0; i < m; i++) {
            uint8_t cat[64];
            memcpy(cat, lvl + 32 * (2 * i), 32);
            memcpy(cat + 32, lvl + 32 * (2 * i + 1 < n ? 2 * i + 1 : n - 1), 32);
            cvo_sha256(lvl + 32 * i, cat, 64);
        }
        n = m;
    }
    memcpy(root, lvl, 32);
    free(lvl);
    return 0;
}

int cvo_merkle_tx_ids(size_t ntx, const uint8_t *arena, const uint64_t *leaf_off,
                      const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, uint8_t *ids,
                      uint8_t *status) {
    for (size_t t = 0; t < ntx; t++) {
        uint32_t b = tx_leaf_begin[t], e = tx_leaf_begin[t + 1];
        size_t nl = e - b;
        uint8_t *lh = (uint8_t *)malloc(32 * (nl ? nl : 1));
        for (size_t k = 0; k < nl; k++) cvo_sha256(lh + 32 * k, arena + leaf_off[b + k], leaf_len[b + k]);
        int st = cvo_merkle_root(lh, nl, ids + 32 * t);
        if (st) memset(ids + 32 * t, 0, 32);
        if (status) status[t] = (uint8_t)st;
        free(lh);
    }
    return 0;
}
