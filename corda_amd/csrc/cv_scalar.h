// cv_scalar.h — arithmetic modulo L = 2^252 + 27742317777372353535851937790883648493 and the
// scalar recodings used by the gfx950 verify/sign kernels.
//
//   sc_reduce512   : 512-bit little-endian value -> value mod L   (h = SHA-512(...) mod L,
//                    eddsa-0.1.0 Ed25519ScalarOps.reduce)
//   slide_drops_carry : exact replay of ref10/eddsa-0.1.0 GroupElement.slide() on S, reporting
//                    whether the carry out of bit 255 is dropped (effective scalar S - 2^256)
//   digit16 / digit256 : signed radix-16 / radix-256 digits read straight from the scalar bits
//                    (d_k = n_k - 2^w * top(n_k) + top(n_{k-1})), so no recoded copy is stored.
#pragma once
#include "cv_field.h"

// ---------------------------------------------------------------- mod L
// 2^252 == mu (mod L) with mu = -(L - 2^252) written in signed 21-bit digits.
#define CV_MU0 666643
#define CV_MU1 470296
#define CV_MU2 654183
#define CV_MU3 (-997805)
#define CV_MU4 136657
#define CV_MU5 (-683901)

#define CV_FOLD(a, k)                    \
    {                                    \
        const int64_t s_ = a[k];         \
        a[(k)-12] += s_ * CV_MU0;        \
        a[(k)-11] += s_ * CV_MU1;        \
        a[(k)-10] += s_ * CV_MU2;        \
        a[(k)-9] += s_ * CV_MU3;         \
        a[(k)-8] += s_ * CV_MU4;         \
        a[(k)-7] += s_ * CV_MU5;         \
        a[k] = 0;                        \
    }
#define CV_SCARRY(a, i)                                         \
    {                                                           \
        const int64_t c_ = (a[i] + ((int64_t)1 << 20)) >> 21;   \
        a[(i) + 1] += c_;                                       \
        a[i] -= c_ * ((int64_t)1 << 21);                        \
    }

// out = (x mod L), x given as 16 little-endian uint32 words (512 bits).
__host__ __device__ __forceinline__ void sc_reduce512(uint32_t out[8], const uint32_t x[16]) {
    int64_t a[25];
    // 21-bit limbs; limb 24 holds the top 8 bits
#pragma unroll
    for (int i = 0; i < 25; i++) {
        const int bit = 21 * i;
        const int w = bit >> 5, r = bit & 31;
        uint64_t v = x[w] >> r;
        if (w + 1 < 16) v |= (uint64_t)x[w + 1] << (32 - r);
        a[i] = (int64_t)(v & 0x1fffff);
    }
    // fold limbs 24..18 into 12..6 (targets never exceed limb 17)
    CV_FOLD(a, 24); CV_FOLD(a, 23); CV_FOLD(a, 22); CV_FOLD(a, 21);
    CV_FOLD(a, 20); CV_FOLD(a, 19); CV_FOLD(a, 18);
#pragma unroll
    for (int i = 6; i < 18; i++) CV_SCARRY(a, i);
    // limb 18 now holds the carry out of 17
    CV_FOLD(a, 18); CV_FOLD(a, 17); CV_FOLD(a, 16); CV_FOLD(a, 15);
    CV_FOLD(a, 14); CV_FOLD(a, 13); CV_FOLD(a, 12);
#pragma unroll
    for (int i = 0; i < 12; i++) CV_SCARRY(a, i);
    CV_FOLD(a, 12);
#pragma unroll
    for (int i = 0; i < 12; i++) CV_SCARRY(a, i);
    CV_FOLD(a, 12);
    // floor carries 0..10: limbs 0..10 in [0, 2^21), limb 11 keeps the (signed) rest
#pragma unroll
    for (int i = 0; i < 11; i++) {
        const int64_t c = a[i] >> 21;
        a[i + 1] += c;
        a[i] -= c * ((int64_t)1 << 21);
    }
    // pack into a signed 288-bit two's-complement value v = sum a_i 2^(21 i)
    uint32_t v[9];
#pragma unroll
    for (int i = 0; i < 9; i++) v[i] = 0;
    uint64_t acc = 0;
    int accbits = 0, wi = 0;
#pragma unroll
    for (int i = 0; i < 11; i++) {
        acc |= (uint64_t)a[i] << accbits;
        accbits += 21;
        while (accbits >= 32) {
            v[wi++] = (uint32_t)acc;
            acc >>= 32;
            accbits -= 32;
        }
    }
    // a[11] is signed: add a[11] * 2^231 (231 = 7*32 + 7) to the words, sign-extending
    {
        const int64_t top = a[11];
        // current words v[0..6] complete, acc holds bits 224.. (accbits = 7)
        const int64_t t = (int64_t)acc + top * 128;   // bits 224.. : acc + top * 2^7
        v[7] = (uint32_t)t;
        v[8] = (uint32_t)(t >> 32);                   // sign-extended high part (value < 2^264 in size)
    }
    const uint32_t Lw[8] = {0x5cf5d3ed, 0x5812631a, 0xa2f79cd6, 0x14def9de, 0, 0, 0, 0x10000000};
    // if negative: add L (at most twice)
#pragma unroll
    for (int rep = 0; rep < 2; rep++) {
        if ((int32_t)v[8] < 0) {
            uint64_t c = 0;
#pragma unroll
            for (int i = 0; i < 9; i++) {
                c += (uint64_t)v[i] + (i < 8 ? Lw[i] : 0);
                v[i] = (uint32_t)c;
                c >>= 32;
            }
        }
    }
    // while v >= L: v -= L (at most a few times; value < 2^254 here)
#pragma unroll
    for (int rep = 0; rep < 4; rep++) {
        uint32_t t[9];
        int64_t br = 0;
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const int64_t d = (int64_t)v[i] - (int64_t)(i < 8 ? Lw[i] : 0) + br;
            t[i] = (uint32_t)d;
            br = d >> 32;   // 0 or -1
        }
        const bool ge = br == 0;
#pragma unroll
        for (int i = 0; i < 9; i++) v[i] = ge ? t[i] : v[i];
    }
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = v[i];
}

// (a * b + c) mod L for 256-bit a, b, c (signing only)
__host__ __device__ __forceinline__ void sc_muladd(uint32_t out[8], const uint32_t a[8], const uint32_t b[8],
                                          const uint32_t c[8]) {
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = 0;
    for (int i = 0; i < 8; i++) {
        uint64_t carry = 0;
        for (int j = 0; j < 8; j++) {
            const uint64_t t = (uint64_t)a[i] * b[j] + x[i + j] + carry;
            x[i + j] = (uint32_t)t;
            carry = t >> 32;
        }
        x[i + 8] = (uint32_t)carry;
    }
    uint64_t carry = 0;
    for (int i = 0; i < 16; i++) {
        carry += (uint64_t)x[i] + (i < 8 ? c[i] : 0);
        x[i] = (uint32_t)carry;
        carry >>= 32;
    }
    sc_reduce512(out, x);
}

// ---------------------------------------------------------------- slide() carry loss

// Exact replay of GroupElement.slide(S) reduced to what decides the dropped carry.  Facts about the
// Java loop (window start i = a set bit, r[i] = 1, then b = 1..6 over r[i+b]):
//   b <= 3: r[i] + 2^b <= 1 + 2 + 4 + 8 = 15, so a set bit is always ADDED (no carry);
//   b == 4: r[i] + 16 > 15 and r[i] - 16 >= -15, so a set bit is always SUBTRACTED: r[i+4] cleared
//           and +2^(i+5) carried into the bits above (the loop that zeroes a run of ones and sets
//           the next zero);  b = 5, 6: neither fits (|r[i]| <= 15 < 17), a set bit only breaks.
// So the scan is a two-state machine over the ORIGINAL bits: with no carry pending the next window
// starts at the next set bit; with a carry pending the run of ones above is cleared and the window
// starts at the first zero (which the carry turns into a one).  A window at j leaves a carry iff
// j + 4 < 256 and bit j+4 is set, and the next scan resumes at j + 5.  A carry reaching bit 256 is
// the drop.  Runs are skipped with count-trailing-zeros on 64-bit windows of S, so a scalar costs
// its ~45 windows, not its 256 bits (the bit-by-bit replay held a 4,096-signature notary batch with
// 1/16 adversarial items for +0.1 ms, tools/lat_scaling.py).  Fast path: with bit 255 clear no
// carry can leave the top (checked by tests/test_oracle.py::test_slide_drop_needs_bit255); the
// replay is pinned against the literal oracle by tests/test_device_logic.py::test_slide_replay_*.
// The 256-bit value lives in four 64-bit registers read through select trees (never a dynamically
// indexed array, which the GPU would keep in scratch memory).
CV_HD uint64_t cv_sel4(const uint64_t u[4], int q) { return (q & 2) ? ((q & 1) ? u[3] : u[2]) : ((q & 1) ? u[1] : u[0]); }
__host__ __device__ __forceinline__ bool slide_drops_carry(const uint32_t s[8]) {
    if (!(s[7] >> 31)) return false;
    uint64_t u[4];
#pragma unroll
    for (int k = 0; k < 4; k++) u[k] = s[2 * k] | ((uint64_t)s[2 * k + 1] << 32);
    // the scan position is base + p, with w = bits [base, base + 64) of S (base a multiple of 64, so a
    // word of u, no shifts): a window step costs one ctz and a shift, and w is re-read only when the scan
    // crosses into the next word — about 5 times per scalar instead of twice per window (round 3: the
    // C4 mix's slide replays set the notary prep's critical path at 4,096)
    int base = 0, p = 0;
    uint64_t w = u[0];
    bool carry = false;
    for (;;) {
        // carry pending: first zero bit (the carry's landing place); none: first set bit
        const uint64_t look = (carry ? ~w : w) >> p;
        if (look == 0) {                               // none in [base + p, base + 64): next word
            base += 64;                                // (a carry whose run of ones reaches bit 256
            if (base >= 256) return carry;             //  is dropped)
            w = cv_sel4(u, base >> 6);
            p = 0;
            continue;
        }
        const int t = __builtin_ctzll(look);
        const int q = base + p + t + 4;                // the window starts at q - 4 (< 256)
        carry = q < 256 && ((p + t + 4 < 64) ? ((w >> (p + t + 4)) & 1u) : ((cv_sel4(u, q >> 6) >> (q & 63)) & 1u));
        p += t + 5;
        if (p >= 64) {
            base += 64;
            p -= 64;
            if (base >= 256) return carry;
            w = cv_sel4(u, base >> 6);
        }
    }
}

// Effective [S]B scalar of eddsa-0.1.0, reduced mod L: (S - 2^256 * drop) mod L.
__host__ __device__ __forceinline__ void sc_effective_s(uint32_t out[8], const uint32_t s[8]) {
    const bool drop = slide_drops_carry(s);
    // -2^256 mod L = 16 (L - 2^252)
    const uint32_t K[5] = {0xcf5d3ed0u, 0x812631a5u, 0x2f79cd65u, 0x4def9deau, 0x1u};
    uint32_t x[16];
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        c += (uint64_t)s[i] + (drop && i < 5 ? K[i] : 0);
        x[i] = (uint32_t)c;
        c >>= 32;
    }
    x[8] = (uint32_t)c;
#pragma unroll
    for (int i = 9; i < 16; i++) x[i] = 0;
    sc_reduce512(out, x);
}

// ---------------------------------------------------------------- digits
// Word q (runtime, 0..7) of an 8-word register array through a select tree: keeps the array in
// VGPRs (a dynamically indexed private array would be demoted to scratch memory).
CV_HD uint32_t sel8(const uint32_t n[8], int q) {
    const uint32_t a0 = (q & 1) ? n[1] : n[0], a1 = (q & 1) ? n[3] : n[2];
    const uint32_t a2 = (q & 1) ? n[5] : n[4], a3 = (q & 1) ? n[7] : n[6];
    const uint32_t b0 = (q & 2) ? a1 : a0, b1 = (q & 2) ? a3 : a2;
    return (q & 4) ? b1 : b0;
}
// bit i (runtime, 0..255) of an 8-word scalar
CV_HD int bit_of_sel(const uint32_t n[8], int i) { return (int)((sel8(n, i >> 5) >> (i & 31)) & 1u); }

// Signed radix-16 digit k (0..63) of a scalar n < 2^255:  d_k in [-8, 8],  sum d_k 16^k = n.
CV_HD int digit16(const uint32_t n[8], int k) {
    const uint32_t nib = (sel8(n, k >> 3) >> ((k & 7) * 4)) & 15u;
    const int top = (int)(nib >> 3);
    const int prev = k ? bit_of_sel(n, 4 * k - 1) : 0;
    return (int)nib - 16 * top + prev;
}
// Signed radix-256 digit k (0..31) of a scalar n < 2^255:  d_k in [-128, 128].
CV_HD int digit256(const uint32_t n[8], int k) {
    const uint32_t byte = (sel8(n, k >> 2) >> ((k & 3) * 8)) & 255u;
    const int top = (int)(byte >> 7);
    const int prev = k ? bit_of_sel(n, 8 * k - 1) : 0;
    return (int)byte - 256 * top + prev;
}

// digit256(n, 8 j + u) for a compile-time j and a run-time u (0..7): the keyed comb's row digits, read with
// static indices and two value selects only — a run-time index into n (digit256 / sel8 there) was turned into a
// dynamically indexed private array, i.e. scratch memory, in cv_comb_kernel.
CV_HD int digit256_row(const uint32_t n[8], int j, int u) {
    const bool hi = (u >> 2) != 0;
    const uint32_t w = hi ? n[2 * j + 1] : n[2 * j];
    const int sh = 8 * (u & 3);
    const uint32_t byte = (w >> sh) & 255u;
    const int top = (int)(byte >> 7);
    // the bit below the digit: bit sh - 1 of w, or (sh == 0) bit 31 of the word before it
    const uint32_t below = hi ? n[2 * j] : (j ? n[2 * j - 1] : 0u);
    const int prev = sh ? (int)((w >> (sh - 1)) & 1u) : (int)(below >> 31);
    return (int)byte - 256 * top + prev;
}

// Signed radix-2^16 digits of a scalar n < 2^253 with the carry propagated (x = raw_k + carry;
// x >= 2^15 -> d_k = x - 2^16, carry 1), d_k in [-2^15, 2^15), sum d_k 2^(16k) = n; packed two per
// word as 16-bit two's complement: out[j] = d_j | d_(j+8) << 16 (j = 0..7), i.e. the digit of the
// k*B row and the digit of the k*2^128*B row that the Straus loop adds at the same window.
CV_HD void digits65536_pairs(uint32_t out[8], const uint32_t n[8]) {
    int d[16];
    uint32_t carry = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t x = ((n[k >> 1] >> (16 * (k & 1))) & 0xffffu) + carry;
        carry = x >= 0x8000u ? 1u : 0u;
        d[k] = (int)x - (int)(carry << 16);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) out[j] = ((uint32_t)d[j] & 0xffffu) | ((uint32_t)d[j + 8] << 16);
}

// ---------------------------------------------------------------- half-size scalars
// For the verify equation R = [s]B - [h]A (eddsa-0.1.0, cofactorless) find u, v with
//     u = v * h  (mod 8L),   v odd,   |u|, |v| ~ 2^128
// by the extended Euclidean algorithm on (8L, h) stopped half-way (the lattice
// {(u, v) : u = v h mod 8L} of determinant 8L, Lagrange/Gauss reduction in dimension 2).  Then
//     [v] (R - [s]B + [h]A) = [v]R + [u]A + [w]B,    w = (-v s) mod L
// because A's order divides 8L and B's is L; and since gcd(v, 8L) = 1 (v odd, 0 < |v| < L),
// [v] is a bijection on E(F_p) (order 8L), so  R == [s]B - [h]A  <=>  [v]R + [u]A + [w]B == O.
// The double-scalar multiplication then needs ~128 doublings instead of ~252.  Modulus 8L (not
// L) keeps the identity exact for keys with a torsion component; v odd keeps it exact for R.
// When no short odd-v vector turns up (rare), (u, v) = (h, 1) is returned with the full window count.

#ifndef CV_STAT
#define CV_STAT(x)
#endif
#define CV_HS_MAXWIN 36                 // |u|, |v| < 2^140 -> at most 36 signed radix-16 windows
#define CV_HS_MAXIT 200                 // Euclid steps (the Fibonacci worst case is ~185)

// a / b for the lattice's quotient estimates, b > 0: on the GPU one v_rcp_f64 refined by two Newton
// steps (relative error ~2^-52, against the IEEE division's ~15-instruction scale/fma/fixup sequence);
// every use tolerates it — the Lehmer loop re-checks each quotient (0 <= remainder < divisor, else it
// stops early and the exact loop continues), the exact loop scales its estimate by 1 - 2^-44
// Host builds (the test harness): a nonzero cv_rcp_emulation replaces the exact division by the device's
// sequence — an initial reciprocal with that relative error (v_rcp_f64's estimate; tests use errors up to
// 2^-12, far worse) refined by the same two Newton steps — so the CPU tests run the quotients the GPU runs.
// (A host variable: device code never reads it.)
inline double cv_rcp_emulation = 0.0;
CV_HD double cv_qdiv(double a, double b) {
#ifdef __HIP_DEVICE_COMPILE__
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    r = fma(fma(-b, r, 1.0), r, r);
    return a * r;
#else
    if (cv_rcp_emulation != 0.0) {
        double r = (1.0 / b) * (1.0 + cv_rcp_emulation);
        r = fma(fma(-b, r, 1.0), r, r);
        r = fma(fma(-b, r, 1.0), r, r);
        return a * r;
    }
    return a / b;
#endif
}
CV_HD double cv_words_to_double(const uint32_t a[8]) {
    double d = (double)a[7];
#pragma unroll
    for (int i = 6; i >= 0; i--) d = d * 4294967296.0 + (double)a[i];
    return d;
}
// two's-complement 5-word signed value -> |value| as double
CV_HD double cv_sw5_abs_double(const uint32_t t[5]) {
    const bool neg = (int32_t)t[4] < 0;
    double d = 0;
#pragma unroll
    for (int i = 4; i >= 0; i--) d = d * 4294967296.0 + (double)(neg ? ~t[i] : t[i]);
    return neg ? d + 1.0 : d;
}
// The exact loop's quotient (r0 >= r1 >= 2^128): an estimate never above floor(r0 / r1) — the doubles carry
// < 2^-49 relative error (word conversions 2^-53 each, the reciprocal and product a few ulp), scaled down by
// 1 - 2^-44 — clamped to [1, 2^32 - 1]; an underestimate leaves r0 - q r1 >= r1 for the next step.
CV_HD uint32_t cv_exact_quotient(const uint32_t r0[8], const uint32_t r1[8]) {
    double q = cv_qdiv(cv_words_to_double(r0), cv_words_to_double(r1)) * (1.0 - 0x1p-44);
    q = q < 1.0 ? 1.0 : (q > 4294967295.0 ? 4294967295.0 : q);
    return (uint32_t)q;
}
// a -= q * b (8 words, no underflow by construction)
CV_HD void cv_submul8(uint32_t a[8], const uint32_t b[8], uint32_t q) {
    uint64_t carry = 0;
    int64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t p = (uint64_t)b[i] * q + carry;
        carry = p >> 32;
        const int64_t d = (int64_t)a[i] - (int64_t)(uint32_t)p + borrow;
        a[i] = (uint32_t)d;
        borrow = d >> 32;
    }
}
// a -= q * b modulo 2^160 (two's complement: works for signed a, b)
CV_HD void cv_submul5(uint32_t a[5], const uint32_t b[5], uint32_t q) {
    uint64_t carry = 0;
    int64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const uint64_t p = (uint64_t)b[i] * q + carry;
        carry = p >> 32;
        const int64_t d = (int64_t)a[i] - (int64_t)(uint32_t)p + borrow;
        a[i] = (uint32_t)d;
        borrow = d >> 32;
    }
}
CV_HD bool cv_lt8(const uint32_t a[8], const uint32_t b[8]) {
    int64_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) borrow = ((int64_t)a[i] - (int64_t)b[i] + borrow) >> 32;
    return borrow != 0;
}
// bits [sh, sh + 53) of an 8-word value below 2^(sh + 53), as an exact double (0 <= sh <= 203)
CV_HD double cv_top53(const uint32_t a[8], int sh) {
    const int ws = sh >> 5, bs = sh & 31;
    const uint32_t w0 = sel8(a, ws), w1 = sel8(a, ws + 1), w2 = ws + 2 < 8 ? sel8(a, ws + 2) : 0u;
    const uint32_t lo = (uint32_t)((((uint64_t)w1 << 32) | w0) >> bs);
    const uint32_t hi = (uint32_t)((((uint64_t)w2 << 32) | w1) >> bs);
    return (double)hi * 4294967296.0 + (double)lo;
}
// out = m0 a + m1 b over NW words (|m0|, |m1| < 2^30), two's complement, word NW (if kept) = sign
template <int NW> CV_HD void cv_lincomb(uint32_t *out, const uint32_t *a, int64_t m0, const uint32_t *b, int64_t m1) {
    int64_t carry = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        const int64_t acc = (int64_t)a[i] * m0 + (int64_t)b[i] * m1 + carry;
        out[i] = (uint32_t)acc;
        carry = acc >> 32;
    }
    out[NW] = (uint32_t)carry;
}
// two's-complement negation of n words when neg
template <int N> CV_HD void cv_cneg_words(uint32_t *x, bool neg) {
    uint64_t c = neg ? 1 : 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
        c += (uint64_t)(neg ? ~x[i] : x[i]);
        x[i] = (uint32_t)c;
        c >>= 32;
    }
}

CV_HD int cv_bitlen8(const uint32_t a[8]) {
    int b = 0;
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (a[i]) b = 32 * i + 32 - __builtin_clz(a[i]);
    return b;
}

// Outputs: u (8 words, u >= 0), v = |v| (8 words), v_neg, nwin = signed radix-16 windows that cover
// both (digit16 k < nwin), w = (-v s) mod L.  Returns false when it fell back to (h, 1).
__host__ __device__ __forceinline__ bool sc_halfsize(uint32_t u[8], uint32_t v[8], bool &v_neg, int &nwin,
                                                     uint32_t w[8], const uint32_t h[8], const uint32_t s[8],
                                                     bool reduce = true) {
    uint32_t r0[8] = {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0, 0, 0, 0x80000000u};   // 8L
    uint32_t r1[8], t0[5] = {0, 0, 0, 0, 0}, t1[5] = {1, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 8; i++) r1[i] = h[i];
    bool done = false;
    // Lehmer phase: Euclid on the leading 53 bits in double precision (cosequence entries < 2^30),
    // one exact multi-word application per ~26 bits.  Every applied matrix is unimodular, so the
    // invariant r_i = t_i h (mod 8L) holds whatever the quotients; a quotient the truncation got
    // wrong only shows up as a negative or out-of-order pair, normalised below.  The exact loop
    // then finishes at the first remainder below 2^128.
#pragma nounroll
    for (int outer = 0; outer < (reduce ? 6 : 0); outer++) {
        if ((r1[4] | r1[5] | r1[6] | r1[7]) == 0) break;
        const int sh = cv_bitlen8(r0) - 53;           // >= 76: r0 >= r1 >= 2^128
        double x0 = cv_top53(r0, sh), x1 = cv_top53(r1, sh);
        double a00 = 1, a01 = 0, a10 = 0, a11 = 1;
        const double lim = sh >= 128 ? 1.0 : (double)(1ull << (128 - sh));   // full r1 stays >= 2^128
        int steps = 0;
#pragma nounroll
        for (int k = 0; k < 40; k++) {
            if (!(x1 >= 0x1p27)) break;
            const double q = floor(cv_qdiv(x0, x1));
            const double nx = fma(-q, x1, x0);
            const double n0 = fma(-q, a10, a00), n1 = fma(-q, a11, a01);
            const double e = fabs(n0) + fabs(n1);
            if (!(nx >= 0 && nx < x1 && e < 0x1p30 && nx >= lim)) break;
            if (!(nx >= e + 1 && x1 - nx >= e + fabs(a10) + fabs(a11) + 1)) break;   // truncation-safe quotient
            x0 = x1; x1 = nx;
            a00 = a10; a01 = a11; a10 = n0; a11 = n1;
            steps++;
        }
        CV_STAT(g_outer++; g_inner += steps;)
        if (steps == 0) break;
        uint32_t nr0[9], nr1[9], nt0[6], nt1[6];
        const int64_t m00 = (int64_t)a00, m01 = (int64_t)a01, m10 = (int64_t)a10, m11 = (int64_t)a11;
        cv_lincomb<8>(nr0, r0, m00, r1, m01);
        cv_lincomb<8>(nr1, r0, m10, r1, m11);
        cv_lincomb<5>(nt0, t0, m00, t1, m01);
        cv_lincomb<5>(nt1, t0, m10, t1, m11);
        const bool n0neg = (int32_t)nr0[8] < 0, n1neg = (int32_t)nr1[8] < 0;
        cv_cneg_words<8>(nr0, n0neg);
        cv_cneg_words<5>(nt0, n0neg);
        cv_cneg_words<8>(nr1, n1neg);
        cv_cneg_words<5>(nt1, n1neg);
#pragma unroll
        for (int i = 0; i < 8; i++) { r0[i] = nr0[i]; r1[i] = nr1[i]; }
#pragma unroll
        for (int i = 0; i < 5; i++) { t0[i] = nt0[i]; t1[i] = nt1[i]; }
    }
#pragma nounroll
    for (int it = 0; it < (reduce ? CV_HS_MAXIT : 0); it++) {
        // keep r0 >= r1 (a quotient underestimate leaves r0 >= r1: the next step continues it)
        const bool lt = cv_lt8(r0, r1);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t a = r0[i], b = r1[i];
            r0[i] = lt ? b : a;
            r1[i] = lt ? a : b;
        }
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const uint32_t a = t0[i], b = t1[i];
            t0[i] = lt ? b : a;
            t1[i] = lt ? a : b;
        }
        if ((r1[4] | r1[5] | r1[6] | r1[7]) == 0) {   // r1 < 2^128 <= r0: stop
            done = true;
            break;
        }
        CV_STAT(g_exact++;)
        const uint32_t qi = cv_exact_quotient(r0, r1);
        cv_submul8(r0, r1, qi);
        cv_submul5(t0, t1, qi);
    }
    // candidate: (r1, t1) if t1 is odd, else (r0 - k r1, t0 - k t1) balanced (t0 is then odd, and
    // t0, t1 have opposite signs so |t0 - k t1| = |t0| + k |t1|)
    bool ok = done;
    uint32_t vt[5];
    if ((t1[0] & 1u) != 0) {
#pragma unroll
        for (int i = 0; i < 8; i++) u[i] = r1[i];
#pragma unroll
        for (int i = 0; i < 5; i++) vt[i] = t1[i];
    } else {
        double k = (cv_words_to_double(r0) - cv_sw5_abs_double(t0)) /
                   (cv_words_to_double(r1) + cv_sw5_abs_double(t1)) * (1.0 - 0x1p-40);
        if (!(k < 4294967295.0)) ok = false;
        k = k < 0.0 ? 0.0 : (k > 4294967295.0 ? 4294967295.0 : k);
        const uint32_t ki = (uint32_t)k;
#pragma unroll
        for (int i = 0; i < 8; i++) u[i] = r0[i];
#pragma unroll
        for (int i = 0; i < 5; i++) vt[i] = t0[i];
        cv_submul8(u, r1, ki);
        cv_submul5(vt, t1, ki);
    }
    v_neg = (int32_t)vt[4] < 0;
    {
        uint64_t c = v_neg ? 1 : 0;                            // |vt| = v_neg ? ~vt + 1 : vt
#pragma unroll
        for (int i = 0; i < 5; i++) {
            c += (uint64_t)(v_neg ? ~vt[i] : vt[i]);
            v[i] = (uint32_t)c;
            c >>= 32;
        }
    }
    v[5] = v[6] = v[7] = 0;
    // bit length of max(u, |v|) -> windows (digit16 of an x < 2^b needs floor(b/4) + 1 digits)
    uint32_t m[8];
#pragma unroll
    for (int i = 0; i < 8; i++) m[i] = u[i] | v[i];
    nwin = cv_bitlen8(m) / 4 + 1;
    if (nwin > CV_HS_MAXWIN) ok = false;
    if (!ok) {
#pragma unroll
        for (int i = 0; i < 8; i++) { u[i] = h[i]; v[i] = i == 0; }
        v_neg = false;
        nwin = 64;
    }
    // w = (-v s) mod L
    {
        uint32_t x[16];
#pragma unroll
        for (int i = 0; i < 16; i++) x[i] = 0;
#pragma unroll
        for (int i = 0; i < 5; i++) {
            uint64_t carry = 0;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint64_t t = (uint64_t)v[i] * s[j] + x[i + j] + carry;
                x[i + j] = (uint32_t)t;
                carry = t >> 32;
            }
            x[i + 8] = (uint32_t)carry;
        }
        uint32_t mm[8];
        sc_reduce512(mm, x);                                   // |v| s mod L
        const uint32_t Lw[8] = {0x5cf5d3ed, 0x5812631a, 0xa2f79cd6, 0x14def9de, 0, 0, 0, 0x10000000};
        uint32_t nz = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) nz |= mm[i];
        int64_t br = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int64_t d = (int64_t)Lw[i] - (int64_t)mm[i] + br;
            const uint32_t neg_i = nz ? (uint32_t)d : 0u;      // (L - m) mod L
            br = d >> 32;
            w[i] = v_neg ? mm[i] : neg_i;                      // v < 0: -v s = |v| s
        }
    }
    return ok;
}
