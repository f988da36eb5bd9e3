// cv_verify.h — the per-lane verify / sign / Merkle procedures, written once as __host__ __device__
// code: the GPU kernels (cv_kernels.hip) run them one record per lane, and the CPU test harness
// (tests/host_harness.cpp) runs the very same code on the host to debug the kernel logic without a
// GPU.  The harness is test infrastructure; the product path is the GPU kernel.
#pragma once
#include "cv_field.h"
#include "cv_group.h"
#include "cv_scalar.h"
#include "cv_sha.h"
#include "cv_tables.h"

// k*B for a signed digit k in [-128, 128] from the precomp table (LDS on the GPU), rows STRIDE words
// apart (a multiple of 4: each row is eight 16-B reads)
template <int STRIDE = CV_BTAB_STRIDE>
CV_HD void btab_select(ge_precomp &r, const uint32_t *btab, int k) {
    const int m = k < 0 ? -k : k;
    const uint4 *row = reinterpret_cast<const uint4 *>(btab + m * STRIDE);
    uint32_t t[32];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const uint4 v = row[q];
        t[4 * q] = v.x; t[4 * q + 1] = v.y; t[4 * q + 2] = v.z; t[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 10; i++) {
        r.yplusx.v[i] = t[i];
        r.yminusx.v[i] = t[10 + i];
        r.xy2d.v[i] = t[20 + i];
    }
    ge_precomp_cneg(r, k < 0);
}

// [k]B for a scalar k < 2^255: signed radix-256 digits from the table, 32 madds + 248 doublings.
__host__ __device__ __forceinline__ void ge_scalarmult_base(ge_p3 &R, const uint32_t k[8], const uint32_t *btab) {
    ge_p3_identity(R);
    ge_p1p1 t;
    ge_p2 q;
    for (int j = 31; j >= 0; j--) {
        if (j != 31) {
            ge_p3_to_p2(q, R);
#pragma unroll 1
            for (int d = 0; d < 7; d++) {
                ge_p2_dbl(t, q);
                ge_p1p1_to_p2(q, t);
            }
            ge_p2_dbl(t, q);
            ge_p1p1_to_p3(R, t);
        }
        ge_precomp e;
        btab_select(e, btab, digit256(k, j));
        ge_madd(t, R, e);
        ge_p1p1_to_p3(R, t);
    }
}

CV_HD void ge_p3_encode(uint32_t w[8], const ge_p3 &p) {
    ge_p2 q;
    ge_p3_to_p2(q, p);
    ge_p2_encode(w, q);
}

// ---------------------------------------------------------------- verify: three phases
// eddsa-0.1.0 EdDSAEngine.verify, split so each GPU kernel keeps a small register working set:
//   phase 1 (prep)   : decode A, Abyte, h = SHA-512(R||Abyte||M) mod L, s = effective S mod L,
//                      table of k*(-A), k = 1..8 (cached form) -> workspace
//   phase 2 (straus) : R' = [h](-A) + [s]B by joint fixed-window Straus -> (X:Y:Z) in workspace
//   phase 3 (finish) : Z^-1 by Montgomery's trick over CV_FIN_CHUNK consecutive signatures per lane,
//                      encode R', byte-compare with R, verdict bits
// Invalid keys are replaced by the identity in phase 1 (verdict forced false) so that every Z
// entering the batch inversion is a non-zero coordinate of a genuine curve point.

#define CV_TAB_ENTRIES 9            // k*P, k = 0..8 (entry 0 = the identity: a digit 0 is a plain lookup)
#define CV_TAB_WORDS (CV_TAB_ENTRIES * 40)
#define CV_HS_WORDS 16              // h (8 words) || s (8 words)
#define CV_R_WORDS 32               // X, Y, Z (10 limbs each) + 2 pad (16-B aligned records)
#define CV_FIN_CHUNK 8              // signatures per lane in the finish phase
// radix-2^16 basepoint rows k * 2^(64 r) * B (r = 0..3, k = 0..2^15; see CV_HS_BWORD below)
#define CV_BW16_ENTRIES 32769
#define CV_BW16_ROWS 4
#define CV_BW16_ROW (CV_BW16_ENTRIES * CV_BTAB_STRIDE)

CV_HD void fe_store(uint32_t *p, const fe &f) {
#pragma unroll
    for (int i = 0; i < 10; i++) p[i] = f.v[i];
}
CV_HD void fe_load(fe &f, const uint32_t *p) {
#pragma unroll
    for (int i = 0; i < 10; i++) f.v[i] = p[i];
}
CV_HD void ge_cached_store(uint32_t *p, const ge_cached &c) {
    fe_store(p, c.YplusX);
    fe_store(p + 10, c.YminusX);
    fe_store(p + 20, c.Z);
    fe_store(p + 30, c.T2d);
}
// 40 words, 16-byte aligned: ten 16-byte loads
CV_HD void ge_cached_load(ge_cached &c, const uint32_t *p) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    uint32_t t[40];
#pragma unroll
    for (int j = 0; j < 10; j++) {
        const uint4 v = q[j];
        t[4 * j] = v.x; t[4 * j + 1] = v.y; t[4 * j + 2] = v.z; t[4 * j + 3] = v.w;
    }
    fe_load(c.YplusX, t);
    fe_load(c.YminusX, t + 10);
    fe_load(c.Z, t + 20);
    fe_load(c.T2d, t + 30);
}

CV_HD void ge_p3_neg(ge_p3 &r, const ge_p3 &a) {
    fe_neg(r.X, a.X);
    fe_carry(r.X, r.X);
    r.Y = a.Y;
    r.Z = a.Z;
    fe_neg(r.T, a.T);
    fe_carry(r.T, r.T);
}

// tab[k] = k * P (k = 0..8) in cached form, 40 words per entry (16-B aligned); entry 0 is the
// identity (1, 1, 1, 0), so a window digit of 0 is the same lookup as any other (no identity select)
__host__ __device__ __forceinline__ void ge_cached_multiples8(uint32_t *tab, const ge_p3 &P1) {
    ge_cached c1, c;
    ge_p3 P;
    ge_cached_identity(c);
    ge_cached_store(tab, c);
    ge_p3_to_cached(c1, P1);
    ge_cached_store(tab + 40, c1);
    ge_p1p1 t;
    ge_p3_dbl(t, P1);
    ge_p1p1_to_p3(P, t);
    ge_p3_to_cached(c, P);
    ge_cached_store(tab + 80, c);
#pragma unroll 1
    for (int k = 3; k <= 8; k++) {
        ge_add(t, P, c1);
        ge_p1p1_to_p3(P, t);
        ge_p3_to_cached(c, P);
        ge_cached_store(tab + 40 * k, c);
    }
}

// Half of ge_cached_multiples8's table, the same instructions on both halves (two lanes per point in
// the latency prep, no divergence): both compute 2P and its cached form c2, then three additions
// Q += x with x = c1 (half 0: 3P) or c2 (half 1: 4P = 2P + 2P by the complete addition), then Q += c2
// twice — half 0 stores entries 0, 1, 3, 5, 7, half 1 entries 2, 4, 6, 8.  Each lane's chain is
// 1 doubling + 3 additions instead of 1 + 6.
__host__ __device__ __forceinline__ void ge_cached_multiples8_half(uint32_t *tab, const ge_p3 &P1, bool half1) {
    ge_cached c1, c2, c;
    ge_p3 Q;
    ge_p1p1 t;
    ge_p3_to_cached(c1, P1);
    ge_p3_dbl(t, P1);
    ge_p1p1_to_p3(Q, t);
    ge_p3_to_cached(c2, Q);
    if (half1) {
        ge_cached_store(tab + 80, c2);
    } else {
        ge_cached_identity(c);
        ge_cached_store(tab, c);
        ge_cached_store(tab + 40, c1);
    }
    // step 1 operand: c1 (half 0) or c2 (half 1), limb-wise, through an opaque lane mask: a plain select of the
    // two structs' limbs is canonicalised into a select of their addresses, which kept both in scratch
    ge_cached x;
    uint32_t m = half1 ? 0xffffffffu : 0u;
#ifdef __HIP_DEVICE_COMPILE__
    asm("" : "+v"(m));
#endif
#pragma unroll
    for (int i = 0; i < 10; i++) {
        x.YplusX.v[i] = (c2.YplusX.v[i] & m) | (c1.YplusX.v[i] & ~m);
        x.YminusX.v[i] = (c2.YminusX.v[i] & m) | (c1.YminusX.v[i] & ~m);
        x.Z.v[i] = (c2.Z.v[i] & m) | (c1.Z.v[i] & ~m);
        x.T2d.v[i] = (c2.T2d.v[i] & m) | (c1.T2d.v[i] & ~m);
    }
    const int k0 = half1 ? 4 : 3;
    // step 0 adds x, steps 1 and 2 add c2: written out, not as a reference select (`s == 0 ? x : c2` is a
    // pointer select when SROA runs, before the loop is unrolled, and it kept both operands in scratch)
    ge_add(t, Q, x);
    ge_p1p1_to_p3(Q, t);
    ge_p3_to_cached(c, Q);
    ge_cached_store(tab + 40 * k0, c);
#pragma unroll
    for (int s = 1; s < 3; s++) {
        ge_add(t, Q, c2);
        ge_p1p1_to_p3(Q, t);
        ge_p3_to_cached(c, Q);
        ge_cached_store(tab + 40 * (k0 + 2 * s), c);
    }
}

// Phase 1.  Returns key_ok.  hs = h || s (16 words), tab = CV_TAB_WORDS words (16-B aligned).
template <bool LAT = false> __host__ __device__ __forceinline__ bool cv_verify_prep(const uint32_t aw[8], const uint32_t rw[8], const uint32_t sw[8],
                                               const uint8_t *msg, uint32_t mlen, uint32_t *hs, uint32_t *tab) {
    // hash first (its state is dead before the point decode starts: small live set)
    {
        uint32_t pre[16], dig[16], h[8], abyte[8];
        ge_abyte_from_key(abyte, aw);
#pragma unroll
        for (int q = 0; q < 8; q++) { pre[q] = rw[q]; pre[8 + q] = abyte[q]; }
        sha512_pre_msg(dig, pre, 64, msg, mlen);
        sc_reduce512(h, dig);
#pragma unroll
        for (int q = 0; q < 8; q++) hs[q] = h[q];
    }
    {
        uint32_t s[8];
        sc_effective_s(s, sw);
#pragma unroll
        for (int q = 0; q < 8; q++) hs[8 + q] = s[q];
    }
    ge_p3 A, nA;
    const bool key_ok = ge_decode_0_1_0<LAT>(A, aw);
    if (!key_ok) ge_p3_identity(A);
    ge_p3_neg(nA, A);
    ge_cached_multiples8(tab, nA);
    return key_ok;
}

// Phase 2: R' = sum_w 16^w (a_w * (-A) + [w even] b_{w/2} * B) as (X:Y:Z).
// Each window: 4 doublings (3 end in p2, the last in p3 for the add), the -A add, and every other
// window the B madd; the window always ends in p2 (no T needed by the next doubling).
__host__ __device__ __forceinline__ void cv_verify_straus(const uint32_t *btab, const uint32_t *hs, const uint32_t *tab,
                                                 ge_p2 &out) {
    uint32_t h[8], s[8];
#pragma unroll
    for (int q = 0; q < 8; q++) { h[q] = hs[q]; s[q] = hs[8 + q]; }
    ge_p2 R;
    ge_p2_identity(R);
#pragma unroll 1
    for (int w = 63; w >= 0; w--) {
        ge_p1p1 t;
        ge_p3 R3;
        if (w != 63) {
            ge_p2_dbl(t, R);
            ge_p1p1_to_p2(R, t);
            ge_p2_dbl(t, R);
            ge_p1p1_to_p2(R, t);
            ge_p2_dbl(t, R);
            ge_p1p1_to_p2(R, t);
            ge_p2_dbl(t, R);
            ge_p1p1_to_p3(R3, t);
        } else {
            ge_p3_identity(R3);
        }
        {
            const int a = digit16(h, w);
            const int m = a < 0 ? -a : a;
            ge_cached e;
            ge_cached_load(e, tab + 40 * m);                 // entry 0 = identity: always one lookup
            ge_cached_cneg(e, a < 0);
            ge_add(t, R3, e);
        }
        if ((w & 1) == 0) {
            ge_p1p1_to_p3(R3, t);
            ge_precomp e;
            btab_select(e, btab, digit256(s, w >> 1));
            ge_madd(t, R3, e);
        }
        ge_p1p1_to_p2(R, t);
    }
    out = R;
}

// Phase 3 for `cnt` (<= CV_FIN_CHUNK) consecutive signatures: Rs = their (X,Y,Z) records
// (CV_R_WORDS apart), rws = their R words (16 words apart: the sig records), ok = key_ok flags.
// Returns the verdict bits (bit k = signature k).
template <bool LAT = false> __host__ __device__ __forceinline__ uint32_t cv_verify_finish(const uint32_t *Rs, const uint32_t *sigw,
                                                               const uint8_t *ok, int cnt) {
    // slots past cnt use Z = 1 so every loop below has static indices (no private-memory arrays)
    fe pre[CV_FIN_CHUNK];
    fe acc;
    fe_one(acc);
#pragma unroll
    for (int k = 0; k < CV_FIN_CHUNK; k++) {
        fe z, one;
        fe_one(one);
        if (k < cnt) fe_load(z, Rs + k * CV_R_WORDS + 20);
        else z = one;
        fe_mul_m<LAT>(acc, z, acc);
        pre[k] = acc;
    }
    fe inv;
    fe_invert<LAT>(inv, acc);
    uint32_t bits = 0;
#pragma unroll
    for (int k = CV_FIN_CHUNK - 1; k >= 0; k--) {
        fe zi, z, x, y, one;
        fe_one(one);
        if (k) fe_mul_m<LAT>(zi, inv, pre[k - 1]);
        else zi = inv;
        if (k < cnt) {
            fe_load(z, Rs + k * CV_R_WORDS + 20);
            fe_load(x, Rs + k * CV_R_WORDS);
            fe_load(y, Rs + k * CV_R_WORDS + 10);
        } else {
            z = one;
            x = one;
            y = one;
        }
        if (k) fe_mul_m<LAT>(inv, z, inv);
        fe_mul_m<LAT>(x, x, zi);
        fe_mul_m<LAT>(y, y, zi);
        uint32_t yw[8], xw[8];
        fe_to_words(yw, y);
        fe_to_words(xw, x);
        yw[7] |= (xw[0] & 1u) << 31;
        uint32_t diff = 0;
        if (k < cnt) {
#pragma unroll
            for (int q = 0; q < 8; q++) diff |= yw[q] ^ sigw[16 * k + q];
            if (diff == 0 && ok[k]) bits |= 1u << k;
        }
    }
    return bits;
}

// Single-signature convenience (host harness): the three phases back to back.
__host__ __device__ __forceinline__ bool cv_verify_one(const uint32_t *btab, const uint32_t aw[8], const uint32_t rw[8],
                                              const uint32_t sw[8], const uint8_t *msg, uint32_t mlen,
                                              bool *key_ok_out) {
    uint32_t hs[CV_HS_WORDS];
    alignas(16) uint32_t tab[CV_TAB_WORDS];
    alignas(16) uint32_t Rrec[CV_R_WORDS];
    const bool key_ok = cv_verify_prep(aw, rw, sw, msg, mlen, hs, tab);
    ge_p2 R;
    cv_verify_straus(btab, hs, tab, R);
    fe_store(Rrec, R.X);
    fe_store(Rrec + 10, R.Y);
    fe_store(Rrec + 20, R.Z);
    uint32_t sigw[16];
#pragma unroll
    for (int q = 0; q < 8; q++) { sigw[q] = rw[q]; sigw[8 + q] = sw[q]; }
    const uint8_t okb = key_ok ? 1 : 0;
    *key_ok_out = key_ok;
    return cv_verify_finish(Rrec, sigw, &okb, 1) & 1u;
}

// ---------------------------------------------------------------- keyed verify (per-key comb)
// For keys that repeat across a batch (notary / party keys) the key work is
// done once per key: decode A (eddsa-0.1.0 rules) and the comb tables
//     T_j[k] = k * 2^(64 j) * (-A),   j = 0..3, k = 0..128 (entry 0 the identity)
// (affine precomp, CV_KTAB_WORDS words = 66 KB per key).  Then [h](-A) = sum_j [h_j] 2^(64 j)(-A) over
// the four 64-bit rows of h's signed radix-256 digits (digit 8 j + u uses row table j at window u of
// 8 bits), and [s]B from the radix-2^16 CV_BW16 rows k * 2^(64 j) * B (digit 4 j + u/2 of s at even
// windows u): 7 x 8 = 56 doublings instead of 252, 32 + 16 additions, all mixed (affine tables).  The
// sums are exact integer scalar multiples, so torsion components of A come out exactly as in the
// single-key schedule (and eddsa-0.1.0's slide-based one).  The W16 = false form of the comb (host
// harness, reference schedule) reads the same key rows with radix-16 digits (entries 0..8) and the
// radix-256 CV_BCOMB rows for B.

#define CV_COMB_ROWS 4
#define CV_KENT_WORDS 32                                      // one affine entry: 30 words + pad (128 B)
#define CV_KENT_ENTRIES 129                                   // k = 0..128 per row
#define CV_KROW_WORDS (CV_KENT_ENTRIES * CV_KENT_WORDS)
#define CV_KTAB_WORDS (CV_COMB_ROWS * CV_KROW_WORDS)          // 16,512 words = 66 KB per key

CV_HD void ge_p3_sel(ge_p3 &r, const ge_p3 &f, const ge_p3 &g, bool b) {
    fe_sel(r.X, f.X, g.X, b);
    fe_sel(r.Y, f.Y, g.Y, b);
    fe_sel(r.Z, f.Z, g.Z, b);
    fe_sel(r.T, f.T, g.T, b);
}

// Key precompute, ONE comb row j of one key (the GPU runs a key's four rows on four lanes):
//     ktab[j][k] = (y+x, y-x, 2dxy) of k * 2^(64 j) * (-A),   k = 0..128
// The 128 multiples go to `ext` (scratch, same layout) in extended coordinates and are normalised
// with one inversion per row (Montgomery's trick; the prefix products are parked in the not yet
// written xy2d words of ktab's entries).  Every lane runs the same 3 x 64 doublings and keeps its
// row's base point, so the four lanes never diverge.  Returns key_ok; invalid keys get identity
// tables (-A = identity).
__host__ __device__ __forceinline__ bool cv_key_prep_row(const uint32_t aw[8], int j, uint32_t *ext, uint32_t *ktab) {
    ge_p3 A, P, Pj;
    const bool key_ok = ge_decode_0_1_0<true>(A, aw);
    if (!key_ok) ge_p3_identity(A);
    ge_p3_neg(P, A);
    Pj = P;
#pragma unroll 1
    for (int r = 1; r < CV_COMB_ROWS; r++) {   // P <- 2^64 P
        ge_p2 q;
        ge_p1p1 t;
        ge_p3_to_p2(q, P);
#pragma unroll 1
        for (int d = 0; d < 63; d++) {
            ge_p2_dbl(t, q);
            ge_p1p1_to_p2(q, t);
        }
        ge_p2_dbl(t, q);
        ge_p1p1_to_p3(P, t);
        ge_p3_sel(Pj, Pj, P, r == j);
    }
    uint32_t *xrow = ext + (size_t)j * CV_KROW_WORDS, *trow = ktab + (size_t)j * CV_KROW_WORDS;
    {
        ge_cached c1;
        ge_p3 Q = Pj;
        ge_p1p1 t;
        ge_p3_to_cached(c1, Pj);
#pragma unroll 1
        for (int k = 1; k < CV_KENT_ENTRIES; k++) {
            if (k == 2) {
                ge_p3_dbl(t, Pj);
                ge_p1p1_to_p3(Q, t);
            } else if (k > 2) {
                ge_add(t, Q, c1);
                ge_p1p1_to_p3(Q, t);
            }
            fe_store(xrow + k * CV_KENT_WORDS, Q.X);
            fe_store(xrow + k * CV_KENT_WORDS + 10, Q.Y);
            fe_store(xrow + k * CV_KENT_WORDS + 20, Q.Z);
        }
    }
    fe acc, z;
    fe_load(acc, xrow + CV_KENT_WORDS + 20);
    fe_store(trow + CV_KENT_WORDS + 20, acc);
#pragma unroll 1
    for (int k = 2; k < CV_KENT_ENTRIES; k++) {
        fe_load(z, xrow + k * CV_KENT_WORDS + 20);
        fe_mul_m<true>(acc, acc, z);
        fe_store(trow + k * CV_KENT_WORDS + 20, acc);
    }
    fe inv, d2;
    fe_invert<true>(inv, acc);
    fe_const_d2(d2);
#pragma unroll 1
    for (int k = CV_KENT_ENTRIES - 1; k >= 1; k--) {
        fe zi, x, y, t;
        if (k > 1) {
            fe pre;
            fe_load(pre, trow + (k - 1) * CV_KENT_WORDS + 20);
            fe_mul_m<true>(zi, inv, pre);
            fe_load(z, xrow + k * CV_KENT_WORDS + 20);
            fe_mul_m<true>(inv, inv, z);
        } else {
            zi = inv;
        }
        fe_load(x, xrow + k * CV_KENT_WORDS);
        fe_load(y, xrow + k * CV_KENT_WORDS + 10);
        fe_mul_m<true>(x, x, zi);
        fe_mul_m<true>(y, y, zi);
        uint32_t *e = trow + k * CV_KENT_WORDS;
        fe_add(t, y, x);
        fe_carry(t, t);
        fe_store(e, t);                      // y + x
        fe_sub<2>(t, y, x);
        fe_carry(t, t);
        fe_store(e + 10, t);                 // y - x
        fe_mul_m<true>(t, x, y);
        fe_mul_m<true>(t, t, d2);
        fe_store(e + 20, t);                 // 2 d x y
        e[30] = e[31] = 0;
    }
    {   // entry 0: the identity (1, 1, 0)
        ge_precomp id;
        ge_precomp_identity(id);
        fe_store(trow, id.yplusx);
        fe_store(trow + 10, id.yminusx);
        fe_store(trow + 20, id.xy2d);
        trow[30] = trow[31] = 0;
    }
    return key_ok;
}

// The whole key's four rows (host harness).
__host__ __device__ __forceinline__ bool cv_key_prep(const uint32_t aw[8], uint32_t *ext, uint32_t *ktab) {
    bool ok = true;
    for (int j = 0; j < CV_COMB_ROWS; j++) ok = cv_key_prep_row(aw, j, ext, ktab);
    return ok;
}

// Keyed phase 1 for one signature: only the hash and scalar (the key work is in the table).
__host__ __device__ __forceinline__ void cv_keyed_hs(const uint32_t aw[8], const uint32_t rw[8], const uint32_t sw[8],
                                                     const uint8_t *msg, uint32_t mlen, uint32_t *hs) {
    uint32_t pre[16], dig[16], h[8], abyte[8], s[8];
    ge_abyte_from_key(abyte, aw);
#pragma unroll
    for (int q = 0; q < 8; q++) { pre[q] = rw[q]; pre[8 + q] = abyte[q]; }
    sha512_pre_msg(dig, pre, 64, msg, mlen);
    sc_reduce512(h, dig);
    sc_effective_s(s, sw);
#pragma unroll
    for (int q = 0; q < 8; q++) { hs[q] = h[q]; hs[8 + q] = s[q]; }
}

// affine entry |d| of one key row table (entry 0 = identity), negated for d < 0
CV_HD void krow_select(ge_precomp &e, const uint32_t *row, int d) {
    const int m = d < 0 ? -d : d;
    const uint4 *q = reinterpret_cast<const uint4 *>(row + m * CV_KENT_WORDS);
    uint32_t t[32];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint4 v = q[j];
        t[4 * j] = v.x; t[4 * j + 1] = v.y; t[4 * j + 2] = v.z; t[4 * j + 3] = v.w;
    }
    fe_load(e.yplusx, t);
    fe_load(e.yminusx, t + 10);
    fe_load(e.xy2d, t + 20);
    ge_precomp_cneg(e, d < 0);
}

// Keyed phase 2: R' = [h](-A) + [s]B by the 4-row comb.
//   W16 = true (the GPU): h as signed radix-256 digits (row j, 8-bit window u: digit 8 j + u, key
//     entries 0..128), s as its 16 carry-propagated radix-2^16 digits from the CV_BW16 rows
//     k * 2^(64 j) * B (bcomb; digit 4 j + u/2 at even windows): 7 x 8 = 56 doublings, 32 + 16 madds.
//   W16 = false (the host harness's reference schedule): h as radix-16 digits (key entries 0..8), s
//     as radix-256 digits from CV_BCOMB (bcomb): 15 x 4 = 60 doublings, 64 + 32 madds.
template <bool W16 = false>
__host__ __device__ __forceinline__ void cv_comb_straus(const uint32_t *bcomb, const uint32_t *hs, const uint32_t *ktab,
                                                        ge_p2 &out) {
    uint32_t h[8], s[8], sd[8];
#pragma unroll
    for (int q = 0; q < 8; q++) { h[q] = hs[q]; s[q] = hs[8 + q]; }
    if (W16) digits65536_pairs(sd, s);      // sd[j] = d_j | d_(j+8) << 16
    constexpr int NWIN = W16 ? 8 : 16, WBITS = W16 ? 8 : 4;
    ge_p2 R;
    ge_p2_identity(R);
#pragma unroll 1
    for (int u = NWIN - 1; u >= 0; u--) {
        ge_p1p1 t;
        ge_p3 R3;
        if (u != NWIN - 1) {
#pragma unroll 1
            for (int d = 0; d < WBITS - 1; d++) {
                ge_p2_dbl(t, R);
                ge_p1p1_to_p2(R, t);
            }
            ge_p2_dbl(t, R);
            ge_p1p1_to_p3(R3, t);
        } else {
            ge_p3_identity(R3);
        }
        const bool with_b = (u & 1) == 0;
#pragma unroll
        for (int j = 0; j < CV_COMB_ROWS; j++) {
            ge_precomp e;
            krow_select(e, ktab + j * CV_KROW_WORDS, W16 ? digit256_row(h, j, u) : digit16(h, 16 * j + u));
            ge_madd(t, R3, e);
            if (j + 1 < CV_COMB_ROWS || with_b) ge_p1p1_to_p3(R3, t);
        }
        if (with_b) {
#pragma unroll
            for (int j = 0; j < CV_COMB_ROWS; j++) {
                ge_precomp e;
                if (W16) {
                    // digit k = 4j + u/2 of s: the low half of sd[k] (k < 8) or the high half of sd[k - 8]
                    const int k = 4 * j + (u >> 1);
                    const uint32_t word = sel8(sd, k & 7);
                    const int d = k < 8 ? (int)(int16_t)(word & 0xffffu) : (int)word >> 16;
                    btab_select(e, bcomb + j * CV_BW16_ROW, d);
                } else {
                    btab_select(e, bcomb + j * CV_BTAB_ENTRIES * CV_BTAB_STRIDE, digit256(s, 8 * j + (u >> 1)));
                }
                ge_madd(t, R3, e);
                if (j + 1 < CV_COMB_ROWS) ge_p1p1_to_p3(R3, t);
            }
        }
        ge_p1p1_to_p2(R, t);
    }
    out = R;
}

// cv_comb_straus<true> with the scalars read from memory each window instead of held in VGPRs across the loop:
// rec[0..7] = h, rec[8..15] = s's radix-2^16 digit pairs (digits65536_pairs, written there by the caller).  Sixteen
// fewer registers live through the loop let cv_comb_kernel fit 3 waves/SIMD without spilling;
// the reloads are two 16-B loads per window plus one word per basepoint window, from the lane's own L2-hot record.
__host__ __device__ __forceinline__ void cv_comb_straus_rec(const uint32_t *bcomb, const uint32_t *rec,
                                                            const uint32_t *ktab, ge_p2 &out) {
    ge_p2 R;
    ge_p2_identity(R);
#pragma unroll 1
    for (int u = 7; u >= 0; u--) {
        ge_p1p1 t;
        ge_p3 R3;
        if (u != 7) {
#pragma unroll 1
            for (int d = 0; d < 7; d++) {
                ge_p2_dbl(t, R);
                ge_p1p1_to_p2(R, t);
            }
            ge_p2_dbl(t, R);
            ge_p1p1_to_p3(R3, t);
        } else {
            ge_p3_identity(R3);
        }
        const bool with_b = (u & 1) == 0;
#pragma unroll
        for (int j = 0; j < CV_COMB_ROWS; j++) {
            // the words of h this row's digit reads (2j - 1 .. 2j + 1), loaded where they are used
            uint32_t h[8] = {};
            if (j) h[2 * j - 1] = rec[2 * j - 1];
            h[2 * j] = rec[2 * j];
            h[2 * j + 1] = rec[2 * j + 1];
            ge_precomp e;
            krow_select(e, ktab + j * CV_KROW_WORDS, digit256_row(h, j, u));
            ge_madd(t, R3, e);
            if (j + 1 < CV_COMB_ROWS || with_b) ge_p1p1_to_p3(R3, t);
        }
        if (with_b) {
#pragma unroll
            for (int j = 0; j < CV_COMB_ROWS; j++) {
                ge_precomp e;
                // digit k = 4j + u/2 of s: the low half of pair word k (k < 8) or the high half of word k - 8
                const int k = 4 * j + (u >> 1);
                const uint32_t word = rec[8 + (k & 7)];
                const int d = k < 8 ? (int)(int16_t)(word & 0xffffu) : (int)word >> 16;
                btab_select(e, bcomb + j * CV_BW16_ROW, d);
                ge_madd(t, R3, e);
                if (j + 1 < CV_COMB_ROWS) ge_p1p1_to_p3(R3, t);
            }
        }
        ge_p1p1_to_p2(R, t);
    }
    out = R;
}

// ---------------------------------------------------------------- keygen + sign one message
// EdDSAPrivateKeySpec(seed) + EdDSAEngine.sign (RFC 8032): pk = [a]B, R = [r]B, S = r + k a.
__host__ __device__ __forceinline__ void cv_sign_one(const uint32_t *btab, const uint32_t seed[8], const uint8_t *msg,
                                            uint32_t mlen, uint32_t pk_out[8], uint32_t sig_out[16]) {
    uint32_t sd[16], hd[16];
#pragma unroll
    for (int q = 0; q < 8; q++) { sd[q] = seed[q]; sd[8 + q] = 0; }
    sha512_pre_msg(hd, sd, 32, msg, 0);               // h = SHA-512(seed)
    uint32_t a[8], prefix[16];
#pragma unroll
    for (int q = 0; q < 8; q++) { a[q] = hd[q]; prefix[q] = hd[8 + q]; prefix[8 + q] = 0; }
    a[0] &= 0xfffffff8u;                               // clamp: h[0] &= 248
    a[7] &= 0x3fffffffu;                               //        h[31] &= 63
    a[7] |= 0x40000000u;                               //        h[31] |= 64
    ge_p3 A;
    ge_scalarmult_base(A, a, btab);
    uint32_t abyte[8];
    ge_p3_encode(abyte, A);
    uint32_t r[8], rd[16];
    sha512_pre_msg(rd, prefix, 32, msg, mlen);         // r = SHA-512(prefix || M) mod L
    sc_reduce512(r, rd);
    ge_p3 Rp;
    ge_scalarmult_base(Rp, r, btab);
    uint32_t rb[8];
    ge_p3_encode(rb, Rp);
    uint32_t pre[16], kd[16], k[8], S[8];
#pragma unroll
    for (int q = 0; q < 8; q++) { pre[q] = rb[q]; pre[8 + q] = abyte[q]; }
    sha512_pre_msg(kd, pre, 64, msg, mlen);            // k = SHA-512(R || A || M) mod L
    sc_reduce512(k, kd);
    sc_muladd(S, k, a, r);                             // S = (r + k a) mod L
#pragma unroll
    for (int q = 0; q < 8; q++) { pk_out[q] = abyte[q]; sig_out[q] = rb[q]; sig_out[8 + q] = S[q]; }
}

// ---------------------------------------------------------------- Merkle root of one transaction
// MerkleTree.buildMerkleTree over cnt leaf digests (8 big-endian words each), in place.
// Returns false for an empty leaf list (MerkleTreeException).  root = 8 big-endian words.
__host__ __device__ __forceinline__ bool cv_merkle_root_inplace(uint32_t *lvl, uint32_t cnt, uint32_t root[8]) {
    if (cnt == 0) {
#pragma unroll
        for (int q = 0; q < 8; q++) root[q] = 0;
        return false;
    }
    while (cnt > 1) {
        const uint32_t m = (cnt + 1) >> 1;
        for (uint32_t j = 0; j < m; j++) {
            uint32_t l[8], r[8], o[8];
            const uint32_t li = 2 * j, ri = (2 * j + 1 < cnt) ? 2 * j + 1 : cnt - 1;
#pragma unroll
            for (int q = 0; q < 8; q++) { l[q] = lvl[li * 8 + q]; r[q] = lvl[ri * 8 + q]; }
            sha256_node(o, l, r);
#pragma unroll
            for (int q = 0; q < 8; q++) lvl[j * 8 + q] = o[q];
        }
        cnt = m;
    }
#pragma unroll
    for (int q = 0; q < 8; q++) root[q] = lvl[q];
    return true;
}

// ---------------------------------------------------------------- half-size verify (throughput path)
// Same verdict as phases 1-3 above with about half the doublings (sc_halfsize, cv_scalar.h):
//   accept  <=>  key_ok  AND  R's bytes are the canonical encoding of a curve point
//                        AND  [v]R + [u]A + [w]B == O
// R' = [s]B - [h]A always encodes canonically (toByteArray), so the reference's byte compare accepts
// exactly when R decodes canonically to the point R' (encoding is injective on points); the scaled
// equation is equivalent to R == R' because gcd(v, 8L) = 1.
//   hsprep : decode R (canonical), table k*R (k = 1..8, cached), (u, v, w) -> workspace
//   straus : ~33 windows of 4 doublings; R and A digits every window, B digits every other window
//            from two radix-256 tables (k*B and k*2^128*B: w's low and high 128 bits); the identity
//            test needs no inversion, so the verdict bit comes straight out of this kernel.
// hsprep leaves per window one packed digit word, window-major (dig[win * stride + i]: a wave reads
// 256 contiguous bytes per window), two's-complement fields:  bits 0-4 = digit of A in [-8, 8] (sign
// pre-flipped for the k*(-A) table), bits 5-9 = digit of R (sign of v folded in), bits 10-18 and
// 19-27 = radix-256 digits in [-128, 128] of w for k*B and k*2^128*B (even windows < 32 only).
// dig[64 * stride + i] = the lane's window count.
CV_HD int cv_sfield(uint32_t w, int off, int width) { return (int)(w << (32 - off - width)) >> (32 - width); }
// W16 digit format (the throughput group): the window words carry only the A and R digits; w's 16
// signed radix-2^16 digits live in 8 more words (digits65536_pairs), word j at dig[(CV_HS_BWORD + j) *
// stride], added at window 4j from the CV_BW16 rows k*B and k*2^128*B (16 basepoint madds per verify
// instead of 32 with the radix-256 rows).  The table has four rows, k * 2^(64 r) * B (r = 0..3): the
// half-size Straus uses rows 0 and 2, the keyed comb all four.
#define CV_HS_BWORD 65
#define CV_HS_DIGWORDS 73

// Canonical decode of R: true iff the 8 words are exactly GroupElement.toByteArray() of a point.
template <bool LAT = false> __host__ __device__ __forceinline__ bool ge_decode_canonical(ge_p3 &P, const uint32_t w[8]) {
    bool ok = ge_decode_0_1_0<LAT>(P, w);
    uint32_t enc[8], diff = 0;
    ge_abyte_from_key(enc, w);          // y mod p, sign bit cleared when x = 0
#pragma unroll
    for (int q = 0; q < 8; q++) diff |= enc[q] ^ w[q];
    return ok && diff == 0;
}

template <bool LAT = false, bool W16 = false>
__host__ __device__ __forceinline__ bool cv_hs_prep(const uint32_t rw[8], const uint32_t *hs, uint32_t *dig, size_t stride,
                                                    uint32_t *tabR, bool reduce = true) {
    {
        uint32_t h[8], s[8], u[8], v[8], w[8];
#pragma unroll
        for (int q = 0; q < 8; q++) { h[q] = hs[q]; s[q] = hs[8 + q]; }
        bool v_neg;
        int nwin;
        sc_halfsize(u, v, v_neg, nwin, w, h, s, reduce);
#pragma unroll
        for (int win = 0; win < 64; win++) {
            const int da = -digit16(u, win), dr = v_neg ? -digit16(v, win) : digit16(v, win);
            const bool bw = !W16 && (win & 1) == 0 && win < 32;
            const int dlo = bw ? digit256(w, win >> 1) : 0, dhi = bw ? digit256(w, 16 + (win >> 1)) : 0;
            dig[(size_t)win * stride] = ((uint32_t)da & 0x1fu) | (((uint32_t)dr & 0x1fu) << 5) |
                                        (((uint32_t)dlo & 0x1ffu) << 10) | (((uint32_t)dhi & 0x1ffu) << 19);
        }
        dig[64 * stride] = (uint32_t)nwin;
        if (W16) {
            uint32_t bw16[8];
            digits65536_pairs(bw16, w);
#pragma unroll
            for (int j = 0; j < 8; j++) dig[(size_t)(CV_HS_BWORD + j) * stride] = bw16[j];
        }
    }
    ge_p3 R;
    const bool r_ok = ge_decode_canonical<LAT>(R, rw);
    if (!r_ok) ge_p3_identity(R);
    ge_cached_multiples8(tabR, R);
    return r_ok;
}

// entry |d| of a cached k*P table (entry 0 = identity), negated for d < 0
CV_HD void tab_cached_select(ge_cached &e, const uint32_t *tab, int d) {
    const int m = d < 0 ? -d : d;
    ge_cached_load(e, tab + 40 * m);
    ge_cached_cneg(e, d < 0);
}

// E = [v]R + [u]A + [w]B from the packed digits (tabA = k*(-A), tabR = k*R); nw (>= 32, uniform
// over the wave on the GPU) windows; the basepoint rows blo / bhi are BSTRIDE words apart.
// W16 = false: radix-256 digits of w in the even window words, rows k*B / k*2^128*B for k = 0..128
// (CV_BCOMB); W16 = true: radix-2^16 digit pairs in their own words, added every fourth window from
// the CV_BW16 rows (k = 0..2^15).  Returns E == O.
template <int BSTRIDE = CV_BTAB_STRIDE, bool W16 = false>
__host__ __device__ __forceinline__ bool cv_hs_straus(const uint32_t *blo, const uint32_t *bhi, const uint32_t *dig,
                                                      size_t stride, const uint32_t *tabA, const uint32_t *tabR, int nw) {
    ge_p2 R;
    ge_p2_identity(R);
#pragma unroll 1
    for (int win = nw - 1; win >= 0; win--) {
        const uint32_t dw = dig[(size_t)win * stride];
        ge_p1p1 t;
        ge_p3 R3;
        if (win != nw - 1) {
            // the first three doublings as a rolled loop: one copy of the formula keeps the window
            // loop's code at 91 KB instead of 115 KB (same-box A/B: hs_straus -1.5 %)
#pragma unroll 1
            for (int d = 0; d < 3; d++) {
                ge_p2_dbl(t, R);
                ge_p1p1_to_p2(R, t);
            }
            ge_p2_dbl(t, R);
            ge_p1p1_to_p3(R3, t);
        } else {
            ge_p3_identity(R3);
        }
        {
            ge_cached e;
            tab_cached_select(e, tabR, cv_sfield(dw, 5, 5));
            ge_add(t, R3, e);
        }
        ge_p1p1_to_p3(R3, t);
        {
            ge_cached e;
            tab_cached_select(e, tabA, cv_sfield(dw, 0, 5));
            ge_add(t, R3, e);
        }
        if (W16 ? ((win & 3) == 0 && win < 32) : ((win & 1) == 0 && win < 32)) {
            int dlo, dhi;
            if (W16) {
                const uint32_t bw = dig[(size_t)(CV_HS_BWORD + (win >> 2)) * stride];
                dlo = (int)(int16_t)(bw & 0xffffu);
                dhi = (int)bw >> 16;
            } else {
                dlo = cv_sfield(dw, 10, 9);
                dhi = cv_sfield(dw, 19, 9);
            }
            ge_precomp e;
            ge_p1p1_to_p3(R3, t);
            btab_select<BSTRIDE>(e, blo, dlo);
            ge_madd(t, R3, e);
            ge_p1p1_to_p3(R3, t);
            btab_select<BSTRIDE>(e, bhi, dhi);
            ge_madd(t, R3, e);
        }
        ge_p1p1_to_p2(R, t);
    }
    // identity: X = 0 and Y = Z (Z != 0 for points of the complete formulas)
    fe d;
    fe_sub<2>(d, R.Y, R.Z);
    return fe_is_zero(R.X) && fe_is_zero(d);
}

// Single-signature convenience (host harness): prep + hsprep + straus.  dig_out: 65 words or null.
__host__ __device__ __forceinline__ bool cv_verify_one_hs(const uint32_t *bcomb, const uint32_t aw[8], const uint32_t rw[8],
                                                          const uint32_t sw[8], const uint8_t *msg, uint32_t mlen,
                                                          bool *key_ok_out, uint32_t *dig_out) {
    uint32_t hs[CV_HS_WORDS];
    alignas(16) uint32_t tab[CV_TAB_WORDS];
    alignas(16) uint32_t tabR[CV_TAB_WORDS];
    uint32_t dig[CV_HS_DIGWORDS];
    const bool key_ok = cv_verify_prep(aw, rw, sw, msg, mlen, hs, tab);
    const bool r_ok = cv_hs_prep(rw, hs, dig, 1, tabR);
    int nw = (int)dig[64];
    if (nw < 32) nw = 32;
    const bool eq = cv_hs_straus(bcomb, bcomb + 2 * CV_BTAB_ENTRIES * CV_BTAB_STRIDE, dig, 1, tab, tabR, nw);
    *key_ok_out = key_ok;
    if (dig_out)
        for (int q = 0; q < CV_HS_DIGWORDS; q++) dig_out[q] = dig[q];
    return key_ok && r_ok && eq;
}

// ---------------------------------------------------------------- partial Merkle tree verify (f3)
// PartialMerkleTree.verify (core/src/main/kotlin/net/corda/core/crypto/PartialMerkleTree.kt:117-144)
// over the flat encoding of include/cordaverify.h (cv_partial_merkle_verify): nodes [b, e) of one
// tree, kind 0 Leaf / 1 IncludedLeaf / 2 Node, children (absolute indices) before their parent,
// root = node e-1.  The root is recomputed bottom-up with hashConcat = SHA-256(left32 || right32);
// the included-leaf hashes must equal the check list as a multiset (the reference's groupBy
// compare); verdict = multiset equal AND root equal.  Workspace: dig (8 words per node), flag (one
// byte per node: bit 0 referenced as a child, bit 1 matched by a check hash).  Returns 0, or 2 when
// [b, e) is not a tree encoding (empty, unknown kind, child not before its parent or outside the
// tree, a node referenced twice or never): verdict false.
#define CV_PMT_LEAF 0
#define CV_PMT_INCLUDED 1
#define CV_PMT_NODE 2

CV_HD void cv_load_digest(uint32_t d[8], const uint8_t *p) {
#pragma unroll
    for (int q = 0; q < 8; q++)
        d[q] = ((uint32_t)p[4 * q] << 24) | ((uint32_t)p[4 * q + 1] << 16) | ((uint32_t)p[4 * q + 2] << 8) | p[4 * q + 3];
}

__host__ __device__ inline int cv_pmt_verify(uint32_t b, uint32_t e, const uint8_t *kind, const uint32_t *left,
                                             const uint32_t *right, const uint8_t *leaf_hash, const uint8_t *root,
                                             const uint8_t *check, uint32_t cb, uint32_t ce, uint32_t *dig,
                                             uint8_t *flag, bool &verdict) {
    verdict = false;
    if (e <= b) return 2;
    for (uint32_t k = b; k < e; k++) flag[k] = 0;
    uint32_t n_incl = 0;
    for (uint32_t k = b; k < e; k++) {
        const uint8_t kd = kind[k];
        uint32_t o[8];
        if (kd == CV_PMT_NODE) {
            const uint32_t l = left[k], r = right[k];
            if (l < b || l >= k || r < b || r >= k || l == r) return 2;
            if ((flag[l] | flag[r]) & 1u) return 2;
            flag[l] |= 1u;
            flag[r] |= 1u;
            uint32_t lw[8], rw[8];
#pragma unroll
            for (int q = 0; q < 8; q++) { lw[q] = dig[8 * (size_t)l + q]; rw[q] = dig[8 * (size_t)r + q]; }
            sha256_node(o, lw, rw);
        } else if (kd == CV_PMT_LEAF || kd == CV_PMT_INCLUDED) {
            cv_load_digest(o, leaf_hash + 32 * (size_t)k);
            n_incl += kd == CV_PMT_INCLUDED;
        } else {
            return 2;
        }
#pragma unroll
        for (int q = 0; q < 8; q++) dig[8 * (size_t)k + q] = o[q];
    }
    for (uint32_t k = b; k + 1 < e; k++)
        if (!(flag[k] & 1u)) return 2;                 // every node but the root has a parent
    if (ce - cb != n_incl) return 0;
    for (uint32_t j = cb; j < ce; j++) {
        uint32_t c[8];
        cv_load_digest(c, check + 32 * (size_t)j);
        bool found = false;
        for (uint32_t k = b; k < e && !found; k++) {
            if (kind[k] != CV_PMT_INCLUDED || (flag[k] & 2u)) continue;
            uint32_t diff = 0;
#pragma unroll
            for (int q = 0; q < 8; q++) diff |= dig[8 * (size_t)k + q] ^ c[q];
            if (diff == 0) {
                flag[k] |= 2u;
                found = true;
            }
        }
        if (!found) return 0;
    }
    uint32_t rt[8], diff = 0;
    cv_load_digest(rt, root);
#pragma unroll
    for (int q = 0; q < 8; q++) diff |= dig[8 * (size_t)(e - 1) + q] ^ rt[q];
    verdict = diff == 0;
    return 0;
}

// ---------------------------------------------------------------- half-size prep, in two parts
// scalars : h = SHA-512(R || Abyte || M) mod L (cv_keyed_hs), the lattice (u, v, w) and the packed
//           window digits -> dig (window-major, stride `stride`), dig[64 * stride] = window count
// points  : A and R decoded (eddsa-0.1.0 rules; R must also be canonical) and the odd-multiple tables
//           k*(-A), k*R; key_ok = A decodes (the status byte), verdict mask = key_ok AND r_ok
// The GPU runs them as separate kernels (cv_kernels.hip: cv_scalars_kernel at 4 waves per SIMD;
// cv_points_kernel with both decodes interleaved per lane for throughput, or cv_points_pair_kernel
// with one decode per lane of a lane pair for small latency-bound batches).
// B16 = false: w as signed radix-256 digits at the even windows (dlo, dhi: 9 bits at 10 and 19, the
// k*B / k*2^128*B rows of the single-chain forms); B16 = true: w as 64 signed radix-16 digits split in
// two 32-window halves (bits 10 and 15, 5 bits each: window t holds digit t and digit 32 + t), for the
// tri-chain form (cv_hsquad.h) whose two B quads each add one digit per window like the R / A quads.
// W16 = true (the throughput group): the window words carry only the A / R digits and w goes to
// the 8 radix-2^16 pair words (CV_HS_BWORD).
template <bool B16 = false, bool W16 = false>
__host__ __device__ __forceinline__ void cv_hs_scalars(const uint32_t hs[CV_HS_WORDS], uint32_t *dig, size_t stride) {
    uint32_t h[8], s[8], u[8], v[8], w[8];
#pragma unroll
    for (int q = 0; q < 8; q++) { h[q] = hs[q]; s[q] = hs[8 + q]; }
    bool v_neg;
    int nwin;
    sc_halfsize(u, v, v_neg, nwin, w, h, s);
    auto window_word = [&](int win) -> uint32_t {
        const int da = -digit16(u, win), dr = v_neg ? -digit16(v, win) : digit16(v, win);
        uint32_t bf;
        if (B16) {
            const int dlo = win < 32 ? digit16(w, win) : 0, dhi = win < 32 ? digit16(w, 32 + win) : 0;
            bf = (((uint32_t)dlo & 0x1fu) << 10) | (((uint32_t)dhi & 0x1fu) << 15);
        } else if (W16) {
            bf = 0;
        } else {
            const bool bw = (win & 1) == 0 && win < 32;
            const int dlo = bw ? digit256(w, win >> 1) : 0, dhi = bw ? digit256(w, 16 + (win >> 1)) : 0;
            bf = (((uint32_t)dlo & 0x1ffu) << 10) | (((uint32_t)dhi & 0x1ffu) << 19);
        }
        return ((uint32_t)da & 0x1fu) | (((uint32_t)dr & 0x1fu) << 5) | bf;
    };
    if constexpr (W16) {
        // fully unrolled: every digit's word and shift are compile-time constants (no runtime word
        // select per digit); same-box A/B: throughput scalars 0.88 -> 0.82 ms per 10^6
#pragma unroll
        for (int win = 0; win < 64; win++) dig[(size_t)win * stride] = window_word(win);
    } else if constexpr (B16) {
        // the tri form's lone wave: a rolled loop over the eight 32-bit words (straight-line code for all 64
        // windows was slower — a lone wave waits on its instruction fetches), eight windows per word with
        // constant shifts: digit = sign-extended nibble + the bit below it (digit16's recoding); the arrays
        // shift down one word per iteration so every index is a constant.  ~1.3 k instructions for the 64
        // words instead of ~6 k with digit16's word selects (in-lane 17.7 us, tools/microbench/lat_parts.hip).
        uint32_t pu = 0, pv = 0, pl = 0, ph = w[3] >> 31;     // the bit below each array's current word
        const uint32_t vneg = v_neg ? ~0u : 0u;
#pragma unroll 1
        for (int j = 0; j < 8; j++) {
            const uint32_t xu = u[0], xv = v[0], xl = j < 4 ? w[0] : 0u, xh = j < 4 ? w[4] : 0u;
#pragma unroll
            for (int t = 0; t < 8; t++) {
                auto dgt = [&](uint32_t x, uint32_t prev) -> int {
                    const int nib = (int)(x << (28 - 4 * t)) >> 28;                    // sign-extended nibble
                    return nib + (int)(t ? (x >> (4 * t - 1)) & 1u : prev);
                };
                const int du = dgt(xu, pu), dv = dgt(xv, pv), dl = dgt(xl, pl), dh = dgt(xh, ph);
                const uint32_t da = (uint32_t)(-du), dr = ((uint32_t)dv ^ vneg) - vneg;   // -u digit, +-v digit
                dig[(size_t)(8 * j + t) * stride] = (da & 0x1fu) | ((dr & 0x1fu) << 5) | (((uint32_t)dl & 0x1fu) << 10) |
                                                    (((uint32_t)dh & 0x1fu) << 15);
            }
            pu = xu >> 31;
            pv = xv >> 31;
            pl = j < 3 ? xl >> 31 : 0u;                       // w's halves end at window 32: no carry-in past it
            ph = j < 3 ? xh >> 31 : 0u;
#pragma unroll
            for (int k = 0; k < 7; k++) {
                u[k] = u[k + 1];
                v[k] = v[k + 1];
            }
            u[7] = v[7] = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) {
                w[k] = w[k + 1];
                w[4 + k] = w[5 + k];
            }
        }
    } else {
        // the tri form's lone-wave prep: the unrolled code was slower (0.089 -> 0.095 ms at 4,096)
#pragma unroll 4
        for (int win = 0; win < 64; win++) dig[(size_t)win * stride] = window_word(win);
    }
    dig[64 * stride] = (uint32_t)nwin;
    if (W16) {
        uint32_t bw16[8];
        digits65536_pairs(bw16, w);
#pragma unroll
        for (int j = 0; j < 8; j++) dig[(size_t)(CV_HS_BWORD + j) * stride] = bw16[j];
    }
}

// R's canonical-encoding check: its bytes re-encode to themselves (y < p; x = 0 only with sign 0)
CV_HD bool cv_r_canonical(const uint32_t rw[8]) {
    uint32_t enc[8], diff = 0;
    ge_abyte_from_key(enc, rw);
#pragma unroll
    for (int q = 0; q < 8; q++) diff |= enc[q] ^ rw[q];
    return diff == 0;
}

// points, both decodes interleaved in one lane (throughput form).  Returns key_ok; ok_out = key_ok
// AND r_ok.
template <bool LAT = false>
__host__ __device__ __forceinline__ bool cv_hs_points(const uint32_t aw[8], const uint32_t rw[8], uint32_t *tabA,
                                                      uint32_t *tabR, bool &ok_out) {
    ge_p3 P[2];
    bool ok[2];
    ge_decode2_0_1_0<LAT>(P, ok, aw, rw);
    const bool key_ok = ok[0], r_ok = ok[1] && cv_r_canonical(rw);
    if (!key_ok) ge_p3_identity(P[0]);
    if (!r_ok) ge_p3_identity(P[1]);
    ge_p3 nA;
    ge_p3_neg(nA, P[0]);
    ge_cached_multiples8(tabA, nA);
    ge_cached_multiples8(tabR, P[1]);
    ok_out = key_ok && r_ok;
    return key_ok;
}

// points, one encoding per lane (latency form: a lane pair per signature runs the two decodes side by
// side): is_r = false decodes the key A into k*(-A), true decodes R (canonical) into k*R.  Both lanes
// run the same instructions.  Returns the lane's decode verdict (key_ok or r_ok).
template <bool LAT = true>
__host__ __device__ __forceinline__ bool cv_hs_point_one(const uint32_t w[8], bool is_r, uint32_t *tab,
                                                         int half = -1) {
    ge_p3 P, nP;
    bool ok = ge_decode_0_1_0<LAT>(P, w);
    ok = ok && (!is_r || cv_r_canonical(w));
    if (!ok) ge_p3_identity(P);
    ge_p3_neg(nP, P);
    if (!is_r) P = nP;
    if (half < 0)
        ge_cached_multiples8(tab, P);
    else
        ge_cached_multiples8_half(tab, P, half == 1);   // two lanes per point, half of the table each
    return ok;
}

// hash + scalars + points in one pass (host harness, and the reference order of the GPU kernels)
template <bool LAT = false>
__host__ __device__ __forceinline__ bool cv_hs_prep_fused_hs(const uint32_t aw[8], const uint32_t rw[8],
                                                             const uint32_t hs[CV_HS_WORDS], uint32_t *dig,
                                                             size_t stride, uint32_t *tabA, uint32_t *tabR,
                                                             bool &ok_out) {
    cv_hs_scalars(hs, dig, stride);
    return cv_hs_points<LAT>(aw, rw, tabA, tabR, ok_out);
}
template <bool LAT = false>
__host__ __device__ __forceinline__ bool cv_hs_prep_fused(const uint32_t aw[8], const uint32_t rw[8], const uint32_t sw[8],
                                                          const uint8_t *msg, uint32_t mlen, uint32_t *dig, size_t stride,
                                                          uint32_t *tabA, uint32_t *tabR, bool &ok_out) {
    uint32_t hs[CV_HS_WORDS];
    cv_keyed_hs(aw, rw, sw, msg, mlen, hs);            // h = SHA-512(R || Abyte || M) mod L, effective s
    return cv_hs_prep_fused_hs<LAT>(aw, rw, hs, dig, stride, tabA, tabR, ok_out);
}

// Single-signature convenience of the fused schedule (host harness).
template <bool LAT = false>
__host__ __device__ __forceinline__ bool cv_verify_one_hs_fused(const uint32_t *bcomb, const uint32_t aw[8],
                                                                const uint32_t rw[8], const uint32_t sw[8],
                                                                const uint8_t *msg, uint32_t mlen, bool *key_ok_out) {
    alignas(16) uint32_t tab[CV_TAB_WORDS];
    alignas(16) uint32_t tabR[CV_TAB_WORDS];
    uint32_t dig[CV_HS_DIGWORDS];
    bool ok = false;
    *key_ok_out = cv_hs_prep_fused<LAT>(aw, rw, sw, msg, mlen, dig, 1, tab, tabR, ok);
    int nw = (int)dig[64];
    if (nw < 32) nw = 32;
    const bool eq = cv_hs_straus(bcomb, bcomb + 2 * CV_BTAB_ENTRIES * CV_BTAB_STRIDE, dig, 1, tab, tabR, nw);
    return ok && eq;
}

// ---------------------------------------------------------------- transactions (cv_verify_transactions)
// The transaction signature g belongs to: the largest t < nt with tsb[t] <= g (tsb[0] <= g < tsb[nt]), so
// transactions without signatures are passed over.  tsb: nt + 1 non-decreasing boundaries.
__host__ __device__ __forceinline__ uint32_t cv_tx_of_sig(uint32_t g, uint32_t nt, const uint32_t *tsb) {
    uint32_t lo = 0, hi = nt;   // tsb[lo] <= g < tsb[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tsb[mid] <= g) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Signatures [b, e) all valid in a verdict bitmap (bit j of word j / 64), and at least one of them: the "all
// signatures valid" half of verifySignatures (SignedTransaction.kt:83-87; a transaction has sigs, :28).
__host__ __device__ __forceinline__ bool cv_tx_all_valid(uint32_t b, uint32_t e, const uint64_t *bitmap) {
    bool ok = e > b;
    for (uint32_t w = b >> 6; ok && w <= (e - 1) >> 6; w++) {
        const uint32_t lo = w == (b >> 6) ? (b & 63) : 0, hi = w == ((e - 1) >> 6) ? ((e - 1) & 63) : 63;
        const uint64_t mask = (hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & ~((1ull << lo) - 1);
        ok = (bitmap[w] & mask) == mask;
    }
    return ok;
}
