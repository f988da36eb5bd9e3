// cv_field.h — GF(2^255-19) arithmetic for the gfx950 verify/sign kernels.
//
// Representation: 10 signed 32-bit limbs, alternating 26/25 bits (radix 2^25.5):
//   f = sum f[i] * 2^ceil(25.5*i),  limb offsets 0,26,51,77,102,128,153,179,204,230.
// Products are 32x32->64 (v_mad_i64_i32 on CDNA4); a full multiply is 100 of them accumulated in
// 64-bit, then one signed carry chain.  This is VALU integer work by design (no MFMA): see DESIGN.md.
//
// Bounds discipline (checked by tests/test_device_logic.py with random and extreme limbs):
//   "tight"  : |f[i]| <= 1.01 * 2^(w_i - 1), w_i = 26 (even i) / 25 (odd i) — output of fe_mul/fe_sq
//   "loose"  : |f[i]| <= 1.65 * 2^w_i, e.g. a sum/difference of at most three tight values —
//              legal input to fe_mul / fe_sq (keeps 38*f9 and 19*g_j inside int32, sums inside int64)
// fe_add / fe_sub do not carry; every group formula in cv_group.h keeps mul inputs loose.
//
// Every function is __host__ __device__ so that the same code is unit-tested on the CPU
// (tests/test_device_logic.py builds a host harness from these headers) and runs on the GPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CV_HD __host__ __device__ __forceinline__

struct fe { int32_t v[10]; };

CV_HD void fe_zero(fe &h) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = 0;
}
CV_HD void fe_one(fe &h) { fe_zero(h); h.v[0] = 1; }
CV_HD void fe_copy(fe &h, const fe &f) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = f.v[i];
}
CV_HD void fe_add(fe &h, const fe &f, const fe &g) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + g.v[i];
}
CV_HD void fe_sub(fe &h, const fe &f, const fe &g) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = f.v[i] - g.v[i];
}
CV_HD void fe_neg(fe &h, const fe &f) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = -f.v[i];
}
// h = b ? g : f  (branch-free select, per lane)
CV_HD void fe_sel(fe &h, const fe &f, const fe &g, bool b) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = b ? g.v[i] : f.v[i];
}

// Signed rounding carry from limb i (width w bits) into limb i+1.
#define CV_CARRY(h, i, w, nxt)                                   \
    {                                                            \
        int64_t c_ = (h[i] + ((int64_t)1 << ((w) - 1))) >> (w);  \
        nxt += c_;                                               \
        h[i] -= c_ * ((int64_t)1 << (w));                        \
    }

// Reduce ten 64-bit column sums to a tight field element.  The carry order interleaves two chains
// (0..4 and 4..9 then 9->0 via 19) so the dependency depth is ~6 instead of 11.
CV_HD void fe_reduce64(fe &out, int64_t h[10]) {
    CV_CARRY(h, 0, 26, h[1]);
    CV_CARRY(h, 4, 26, h[5]);
    CV_CARRY(h, 1, 25, h[2]);
    CV_CARRY(h, 5, 25, h[6]);
    CV_CARRY(h, 2, 26, h[3]);
    CV_CARRY(h, 6, 26, h[7]);
    CV_CARRY(h, 3, 25, h[4]);
    CV_CARRY(h, 7, 25, h[8]);
    CV_CARRY(h, 4, 26, h[5]);
    CV_CARRY(h, 8, 26, h[9]);
    {
        int64_t c = (h[9] + ((int64_t)1 << 24)) >> 25;
        h[0] += c * 19;
        h[9] -= c * ((int64_t)1 << 25);
    }
    CV_CARRY(h, 0, 26, h[1]);
#pragma unroll
    for (int i = 0; i < 10; i++) out.v[i] = (int32_t)h[i];
}

CV_HD int64_t m64(int32_t a, int32_t b) { return (int64_t)a * (int64_t)b; }

// h = f * g
CV_HD void fe_mul(fe &h, const fe &f, const fe &g) {
    const int32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
    const int32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
    const int32_t g0 = g.v[0], g1 = g.v[1], g2 = g.v[2], g3 = g.v[3], g4 = g.v[4];
    const int32_t g5 = g.v[5], g6 = g.v[6], g7 = g.v[7], g8 = g.v[8], g9 = g.v[9];
    // 19*g_j folds the 2^255 wrap; 2*f_i (odd i) pays the extra half bit of odd*odd offsets
    const int32_t g1_19 = 19 * g1, g2_19 = 19 * g2, g3_19 = 19 * g3, g4_19 = 19 * g4, g5_19 = 19 * g5;
    const int32_t g6_19 = 19 * g6, g7_19 = 19 * g7, g8_19 = 19 * g8, g9_19 = 19 * g9;
    const int32_t f1_2 = 2 * f1, f3_2 = 2 * f3, f5_2 = 2 * f5, f7_2 = 2 * f7, f9_2 = 2 * f9;
    int64_t h_[10];
    h_[0] = m64(f0, g0) + m64(f1_2, g9_19) + m64(f2, g8_19) + m64(f3_2, g7_19) + m64(f4, g6_19) +
            m64(f5_2, g5_19) + m64(f6, g4_19) + m64(f7_2, g3_19) + m64(f8, g2_19) + m64(f9_2, g1_19);
    h_[1] = m64(f0, g1) + m64(f1, g0) + m64(f2, g9_19) + m64(f3, g8_19) + m64(f4, g7_19) +
            m64(f5, g6_19) + m64(f6, g5_19) + m64(f7, g4_19) + m64(f8, g3_19) + m64(f9, g2_19);
    h_[2] = m64(f0, g2) + m64(f1_2, g1) + m64(f2, g0) + m64(f3_2, g9_19) + m64(f4, g8_19) +
            m64(f5_2, g7_19) + m64(f6, g6_19) + m64(f7_2, g5_19) + m64(f8, g4_19) + m64(f9_2, g3_19);
    h_[3] = m64(f0, g3) + m64(f1, g2) + m64(f2, g1) + m64(f3, g0) + m64(f4, g9_19) +
            m64(f5, g8_19) + m64(f6, g7_19) + m64(f7, g6_19) + m64(f8, g5_19) + m64(f9, g4_19);
    h_[4] = m64(f0, g4) + m64(f1_2, g3) + m64(f2, g2) + m64(f3_2, g1) + m64(f4, g0) +
            m64(f5_2, g9_19) + m64(f6, g8_19) + m64(f7_2, g7_19) + m64(f8, g6_19) + m64(f9_2, g5_19);
    h_[5] = m64(f0, g5) + m64(f1, g4) + m64(f2, g3) + m64(f3, g2) + m64(f4, g1) +
            m64(f5, g0) + m64(f6, g9_19) + m64(f7, g8_19) + m64(f8, g7_19) + m64(f9, g6_19);
    h_[6] = m64(f0, g6) + m64(f1_2, g5) + m64(f2, g4) + m64(f3_2, g3) + m64(f4, g2) +
            m64(f5_2, g1) + m64(f6, g0) + m64(f7_2, g9_19) + m64(f8, g8_19) + m64(f9_2, g7_19);
    h_[7] = m64(f0, g7) + m64(f1, g6) + m64(f2, g5) + m64(f3, g4) + m64(f4, g3) +
            m64(f5, g2) + m64(f6, g1) + m64(f7, g0) + m64(f8, g9_19) + m64(f9, g8_19);
    h_[8] = m64(f0, g8) + m64(f1_2, g7) + m64(f2, g6) + m64(f3_2, g5) + m64(f4, g4) +
            m64(f5_2, g3) + m64(f6, g2) + m64(f7_2, g1) + m64(f8, g0) + m64(f9_2, g9_19);
    h_[9] = m64(f0, g9) + m64(f1, g8) + m64(f2, g7) + m64(f3, g6) + m64(f4, g5) +
            m64(f5, g4) + m64(f6, g3) + m64(f7, g2) + m64(f8, g1) + m64(f9, g0);
    fe_reduce64(h, h_);
}

// h = f^2 (55 products); dbl != 0 gives h = 2 f^2
CV_HD void fe_sq_impl(fe &h, const fe &f, bool dbl) {
    const int32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
    const int32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
    const int32_t f0_2 = 2 * f0, f1_2 = 2 * f1, f2_2 = 2 * f2, f3_2 = 2 * f3, f4_2 = 2 * f4;
    const int32_t f5_2 = 2 * f5, f6_2 = 2 * f6, f7_2 = 2 * f7;
    const int32_t f5_38 = 38 * f5, f6_19 = 19 * f6, f7_38 = 38 * f7, f8_19 = 19 * f8, f9_38 = 38 * f9;
    int64_t h_[10];
    h_[0] = m64(f0, f0) + m64(f1_2, f9_38) + m64(f2_2, f8_19) + m64(f3_2, f7_38) + m64(f4_2, f6_19) +
            m64(f5, f5_38);
    h_[1] = m64(f0_2, f1) + m64(f2, f9_38) + m64(f3_2, f8_19) + m64(f4, f7_38) + m64(f5_2, f6_19);
    h_[2] = m64(f0_2, f2) + m64(f1_2, f1) + m64(f3_2, f9_38) + m64(f4_2, f8_19) + m64(f5_2, f7_38) +
            m64(f6, f6_19);
    h_[3] = m64(f0_2, f3) + m64(f1_2, f2) + m64(f4, f9_38) + m64(f5_2, f8_19) + m64(f6, f7_38);
    h_[4] = m64(f0_2, f4) + m64(f1_2, f3_2) + m64(f2, f2) + m64(f5_2, f9_38) + m64(f6_2, f8_19) +
            m64(f7, f7_38);
    h_[5] = m64(f0_2, f5) + m64(f1_2, f4) + m64(f2_2, f3) + m64(f6, f9_38) + m64(f7_2, f8_19);
    h_[6] = m64(f0_2, f6) + m64(f1_2, f5_2) + m64(f2_2, f4) + m64(f3_2, f3) + m64(f7_2, f9_38) +
            m64(f8, f8_19);
    h_[7] = m64(f0_2, f7) + m64(f1_2, f6) + m64(f2_2, f5) + m64(f3_2, f4) + m64(f8, f9_38);
    h_[8] = m64(f0_2, f8) + m64(f1_2, f7_2) + m64(f2_2, f6) + m64(f3_2, f5_2) + m64(f4, f4) +
            m64(f9, f9_38);
    h_[9] = m64(f0_2, f9) + m64(f1_2, f8) + m64(f2_2, f7) + m64(f3_2, f6) + m64(f4_2, f5);
    if (dbl) {
#pragma unroll
        for (int i = 0; i < 10; i++) h_[i] += h_[i];
    }
    fe_reduce64(h, h_);
}
CV_HD void fe_sq(fe &h, const fe &f) { fe_sq_impl(h, f, false); }
CV_HD void fe_sq2(fe &h, const fe &f) { fe_sq_impl(h, f, true); }

// h = f^(2^n) (n >= 1); a real loop keeps the code small (used only in exponentiation chains)
__host__ __device__ inline void fe_sqn(fe &h, const fe &f, int n) {
    fe_sq(h, f);
#pragma nounroll
    for (int i = 1; i < n; i++) fe_sq(h, h);
}

// h = f * 121666-style small constant is not needed; d and 2d come from constants below.

// Parse 32 little-endian bytes given as 8 uint32 words.  Bit 255 is ignored and the value is NOT
// reduced mod p (eddsa-0.1.0 Ed25519LittleEndianEncoding.decode semantics): y in [p, 2^255) is
// simply a non-canonical representative.
CV_HD void fe_from_words(fe &h, const uint32_t w[8]) {
    // limb i covers bits [off_i, off_i + width_i)
    const uint64_t lo0 = w[0] | ((uint64_t)w[1] << 32);
    const uint64_t lo1 = w[2] | ((uint64_t)w[3] << 32);
    const uint64_t lo2 = w[4] | ((uint64_t)w[5] << 32);
    const uint64_t lo3 = w[6] | ((uint64_t)(w[7] & 0x7fffffffu) << 32);
    // helper: bits [a, a+n) of the 256-bit value (n <= 26)
    auto bits = [&](int a, int n) -> int32_t {
        const int q = a >> 6, r = a & 63;
        const uint64_t W[4] = {lo0, lo1, lo2, lo3};
        uint64_t x = W[q] >> r;
        if (r + n > 64 && q < 3) x |= W[q + 1] << (64 - r);
        return (int32_t)(x & ((1ull << n) - 1));
    };
    h.v[0] = bits(0, 26);
    h.v[1] = bits(26, 25);
    h.v[2] = bits(51, 26);
    h.v[3] = bits(77, 25);
    h.v[4] = bits(102, 26);
    h.v[5] = bits(128, 25);
    h.v[6] = bits(153, 26);
    h.v[7] = bits(179, 25);
    h.v[8] = bits(204, 26);
    h.v[9] = bits(230, 25);
}

// Canonical encoding (value mod p in [0, p)) as 8 little-endian uint32 words.
// Input must be tight or loose (|limb| < 2^27).
CV_HD void fe_to_words(uint32_t w[8], const fe &f) {
    int64_t h[10];
#pragma unroll
    for (int i = 0; i < 10; i++) h[i] = f.v[i];
    // first make every limb non-negative and within width (value preserved mod p)
    fe t;
    fe_reduce64(t, h);
#pragma unroll
    for (int i = 0; i < 10; i++) h[i] = t.v[i];
    // q = floor(value / p) in {0, 1} after the tight carry; computed as in a constant-time
    // "subtract p if >= p": q = carry out of (value + 19) at bit 255.
    int64_t q = (19 * h[9] + ((int64_t)1 << 24)) >> 25;
    q = (h[0] + q) >> 26;
    q = (h[1] + q) >> 25;
    q = (h[2] + q) >> 26;
    q = (h[3] + q) >> 25;
    q = (h[4] + q) >> 26;
    q = (h[5] + q) >> 25;
    q = (h[6] + q) >> 26;
    q = (h[7] + q) >> 25;
    q = (h[8] + q) >> 26;
    q = (h[9] + q) >> 25;
    h[0] += 19 * q;
    // exact (floor) carries; the final carry out of limb 9 is 2^255*q and is discarded
    int64_t c;
    c = h[0] >> 26; h[1] += c; h[0] -= c * ((int64_t)1 << 26);
    c = h[1] >> 25; h[2] += c; h[1] -= c * ((int64_t)1 << 25);
    c = h[2] >> 26; h[3] += c; h[2] -= c * ((int64_t)1 << 26);
    c = h[3] >> 25; h[4] += c; h[3] -= c * ((int64_t)1 << 25);
    c = h[4] >> 26; h[5] += c; h[4] -= c * ((int64_t)1 << 26);
    c = h[5] >> 25; h[6] += c; h[5] -= c * ((int64_t)1 << 25);
    c = h[6] >> 26; h[7] += c; h[6] -= c * ((int64_t)1 << 26);
    c = h[7] >> 25; h[8] += c; h[7] -= c * ((int64_t)1 << 25);
    c = h[8] >> 26; h[9] += c; h[8] -= c * ((int64_t)1 << 26);
    c = h[9] >> 25; h[9] -= c * ((int64_t)1 << 25);
    const uint32_t l0 = (uint32_t)h[0], l1 = (uint32_t)h[1], l2 = (uint32_t)h[2], l3 = (uint32_t)h[3];
    const uint32_t l4 = (uint32_t)h[4], l5 = (uint32_t)h[5], l6 = (uint32_t)h[6], l7 = (uint32_t)h[7];
    const uint32_t l8 = (uint32_t)h[8], l9 = (uint32_t)h[9];
    w[0] = l0 | (l1 << 26);
    w[1] = (l1 >> 6) | (l2 << 19);
    w[2] = (l2 >> 13) | (l3 << 13);
    w[3] = (l3 >> 19) | (l4 << 6);
    w[4] = l5 | (l6 << 25);
    w[5] = (l6 >> 7) | (l7 << 19);
    w[6] = (l7 >> 13) | (l8 << 12);
    w[7] = (l8 >> 20) | (l9 << 6);
}

CV_HD bool fe_is_zero(const fe &f) {
    uint32_t w[8];
    fe_to_words(w, f);
    return (w[0] | w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7]) == 0;
}
CV_HD int fe_is_negative(const fe &f) {
    uint32_t w[8];
    fe_to_words(w, f);
    return (int)(w[0] & 1);
}

// z^(2^252 - 3)
__host__ __device__ inline void fe_pow22523(fe &out, const fe &z) {
    fe t0, t1, t2;
    fe_sq(t0, z);            // z^2
    fe_sqn(t1, t0, 2);       // z^8
    fe_mul(t1, z, t1);       // z^9
    fe_mul(t0, t0, t1);      // z^11
    fe_sq(t0, t0);           // z^22
    fe_mul(t0, t1, t0);      // z^31 = z^(2^5-1)
    fe_sqn(t1, t0, 5);
    fe_mul(t0, t1, t0);      // z^(2^10-1)
    fe_sqn(t1, t0, 10);
    fe_mul(t1, t1, t0);      // z^(2^20-1)
    fe_sqn(t2, t1, 20);
    fe_mul(t1, t2, t1);      // z^(2^40-1)
    fe_sqn(t1, t1, 10);
    fe_mul(t0, t1, t0);      // z^(2^50-1)
    fe_sqn(t1, t0, 50);
    fe_mul(t1, t1, t0);      // z^(2^100-1)
    fe_sqn(t2, t1, 100);
    fe_mul(t1, t2, t1);      // z^(2^200-1)
    fe_sqn(t1, t1, 50);
    fe_mul(t0, t1, t0);      // z^(2^250-1)
    fe_sqn(t0, t0, 2);       // z^(2^252-4)
    fe_mul(out, t0, z);      // z^(2^252-3)
}

// z^(p-2) = z^(2^255 - 21)
__host__ __device__ inline void fe_invert(fe &out, const fe &z) {
    fe t0, t1, t2, t3;
    fe_sq(t0, z);            // z^2
    fe_sqn(t1, t0, 2);       // z^8
    fe_mul(t1, z, t1);       // z^9
    fe_mul(t0, t0, t1);      // z^11
    fe_sq(t2, t0);           // z^22
    fe_mul(t1, t1, t2);      // z^31
    fe_sqn(t2, t1, 5);
    fe_mul(t1, t2, t1);      // 2^10-1
    fe_sqn(t2, t1, 10);
    fe_mul(t2, t2, t1);      // 2^20-1
    fe_sqn(t3, t2, 20);
    fe_mul(t2, t3, t2);      // 2^40-1
    fe_sqn(t2, t2, 10);
    fe_mul(t1, t2, t1);      // 2^50-1
    fe_sqn(t2, t1, 50);
    fe_mul(t2, t2, t1);      // 2^100-1
    fe_sqn(t3, t2, 100);
    fe_mul(t2, t3, t2);      // 2^200-1
    fe_sqn(t2, t2, 50);
    fe_mul(t1, t2, t1);      // 2^250-1
    fe_sqn(t1, t1, 5);       // 2^255-32
    fe_mul(out, t1, t0);     // 2^255-21
}
