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
CV_HD int bit_of(const uint32_t u[8], int i) { return (int)((u[i >> 5] >> (i & 31)) & 1u); }

// Exact replay of GroupElement.slide(S) tracking only what decides the dropped carry: the scan
// keeps the not-yet-absorbed bits as a 256-bit integer U; a "subtract" step adds 2^(i+b) to U
// (the Java loop that zeroes a run of ones and sets the next zero); a carry out of bit 255 is the
// drop.  Fast path: with bit 255 clear no carry can leave the top (checked exhaustively on the top
// bits and on 10^5 random scalars by tests/test_oracle.py::test_slide_drop_needs_bit255).
__host__ __device__ __forceinline__ bool slide_drops_carry(const uint32_t s[8]) {
    if (!(s[7] >> 31)) return false;
    uint32_t u[8];
#pragma unroll
    for (int i = 0; i < 8; i++) u[i] = s[i];
    for (int i = 0; i < 256; i++) {
        if (!bit_of(u, i)) continue;
        int d = 1;
        for (int b = 1; b <= 6 && i + b < 256; b++) {
            if (!bit_of(u, i + b)) continue;
            if (d + (1 << b) <= 15) {
                d += 1 << b;
                u[(i + b) >> 5] &= ~(1u << ((i + b) & 31));
            } else if (d - (1 << b) >= -15) {
                d -= 1 << b;
                // U += 2^(i+b)
                int w = (i + b) >> 5;
                uint64_t c = (uint64_t)u[w] + (1ull << ((i + b) & 31));
                u[w] = (uint32_t)c;
                c >>= 32;
                for (w = w + 1; w < 8 && c; w++) {
                    c += u[w];
                    u[w] = (uint32_t)c;
                    c >>= 32;
                }
                if (c) return true;
            } else {
                break;
            }
        }
    }
    return false;
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
