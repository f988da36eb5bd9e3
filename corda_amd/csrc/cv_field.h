// cv_field.h — GF(2^255-19) arithmetic for the gfx950 verify/sign kernels.
//
// Representation: 10 UNSIGNED 32-bit limbs, alternating 26/25 bits (radix 2^25.5):
//   f = sum f[i] * 2^off_i,  off = 0,26,51,77,102,128,153,179,204,230,  M_i = 2^w_i (w = 26,25,26,...)
// A multiply is 100 32x32->64 products accumulated in 64-bit columns — `v_mad_u64_u32`, which issues
// ~12 % faster than the signed `v_mad_i64_i32` on gfx950 (tools/microbench/instr_rates.hip) — then
// one floor-carry chain (logical shifts + masks: no rounding constants, no signed fix-ups).
// This is VALU integer work by design (no MFMA): see DESIGN.md.
//
// Bounds (in units of M_i per limb; checked on the host by CV_BOUNDS_CHECK):
//   T  "tight"  : output of fe_mul / fe_sq / fe_sq2 / fe_carry            <= 1.01
//   fe_mul(h, f, g): g <= 3.3 (19*g_j must fit 32 bits), f <= 8 (column sums stay < 2^64)
//   fe_sq(h, f) / fe_sq2: f <= 3.3 (38*f_odd, 19*f_even fit 32 bits; doubled columns < 2^64)
//   fe_sub<k>(h, f, g) = f + k*p - g : needs g <= k - 0.01 (no limb underflow), result <= f + k
// Every group formula in cv_group.h is written against these rules (the host harness asserts them
// on every call while it replays the whole golden corpus).
//
// Every function is __host__ __device__: the same code runs in the GPU kernels and in the CPU test
// harness (tests/host_harness.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "cv_madc.h"

#define CV_HD __host__ __device__ __forceinline__

#if defined(CV_BOUNDS_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
#include <cstdio>
#include <cstdlib>
#define CV_ASSERT(c, msg)                                                  \
    do {                                                                   \
        if (!(c)) {                                                        \
            fprintf(stderr, "cv_field bound violated: %s (%s:%d)\n", msg, __FILE__, __LINE__); \
            abort();                                                       \
        }                                                                  \
    } while (0)
#define CV_CHECKING 1
#else
#define CV_ASSERT(c, msg) ((void)0)
#define CV_CHECKING 0
#endif

struct fe { uint32_t v[10]; };

// limb widths / masks
#define CV_W(i) (((i) & 1) ? 25 : 26)
#define CV_MASK(i) (((i) & 1) ? 0x1ffffffu : 0x3ffffffu)

// k*p in limb form (k = 2, 3, 4): limb 0 = k(2^26 - 19), odd = k(2^25 - 1), even = k(2^26 - 1)
#define CV_KP0(k) ((uint32_t)(k) * 0x3ffffedu)
#define CV_KPO(k) ((uint32_t)(k) * 0x1ffffffu)
#define CV_KPE(k) ((uint32_t)(k) * 0x3ffffffu)
CV_HD uint32_t cv_kp(int k, int i) { return i == 0 ? CV_KP0(k) : ((i & 1) ? CV_KPO(k) : CV_KPE(k)); }

CV_HD void fe_zero(fe &h) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = 0;
}
CV_HD void fe_one(fe &h) { fe_zero(h); h.v[0] = 1; }
CV_HD void fe_add(fe &h, const fe &f, const fe &g) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = f.v[i] + g.v[i];
}
// h = f + k*p - g   (k = 2, 3 or 4; see the bounds table above).  Written as |k*p_i - g_i| + f_i, which equals
// it because g_i <= k*p_i (the asserted bound): LLVM selects ONE v_sad_u32 per limb (absolute difference plus
// addend, the k*p limb from an SGPR) instead of an add and a subtract — 10 VALU per subtraction instead of 20.
template <int K> CV_HD void fe_sub(fe &h, const fe &f, const fe &g) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        CV_ASSERT(g.v[i] <= cv_kp(K, i), "fe_sub: subtrahend limb exceeds k*p");
        uint32_t k = cv_kp(K, i);
        const uint32_t x = g.v[i];
#ifdef __HIP_DEVICE_COMPILE__
        asm("" : "+s"(k));   // an opaque k: x's known range would otherwise fold the select back into add + subtract
#endif
        h.v[i] = (k > x ? k - x : x - k) + f.v[i];
    }
}
// h = f + k*p - g with its even limbs carried (fe_sub then fe_carry_even, in one pass): each odd limb's
// v_sad_u32 takes the even limb's carry in its addend (f_odd + c), so LLVM does not merge the carry add into a
// v_add3 that would leave the absolute difference as min / max / subtract.
template <int K> CV_HD void fe_sub_carry_even(fe &h, const fe &f, const fe &g) {
#pragma unroll
    for (int i = 0; i < 10; i += 2) {
        uint32_t k0 = cv_kp(K, i), k1 = cv_kp(K, i + 1);
        CV_ASSERT(g.v[i] <= k0 && g.v[i + 1] <= k1, "fe_sub: subtrahend limb exceeds k*p");
#ifdef __HIP_DEVICE_COMPILE__
        asm("" : "+s"(k0), "+s"(k1));
#endif
        const uint32_t x0 = g.v[i], x1 = g.v[i + 1];
        const uint32_t e = (k0 > x0 ? k0 - x0 : x0 - k0) + f.v[i];
        uint32_t a1 = f.v[i + 1] + (e >> 26);
#ifdef __HIP_DEVICE_COMPILE__
        asm("" : "+v"(a1));   // keeps the add out of a v_add3 with the absolute difference
#endif
        h.v[i] = e & 0x3ffffffu;
        h.v[i + 1] = (k1 > x1 ? k1 - x1 : x1 - k1) + a1;
    }
}

// h = -f = 2p - f  (f tight)
CV_HD void fe_neg(fe &h, const fe &f) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        CV_ASSERT(f.v[i] <= cv_kp(2, i), "fe_neg: limb exceeds 2p");
        h.v[i] = cv_kp(2, i) - f.v[i];
    }
}
// h = b ? g : f  (branch-free select, per lane)
CV_HD void fe_sel(fe &h, const fe &f, const fe &g, bool b) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = b ? g.v[i] : f.v[i];
}

// Renormalise an element whose limbs are < 2^31 to tight, with 32-bit ops only.
CV_HD void fe_carry(fe &h, const fe &f) {
    uint32_t t[10];
#pragma unroll
    for (int i = 0; i < 10; i++) t[i] = f.v[i];
#pragma unroll
    for (int i = 0; i < 9; i++) {
        t[i + 1] += t[i] >> CV_W(i);
        t[i] &= CV_MASK(i);
    }
    const uint32_t c = t[9] >> 25;
    t[9] &= 0x1ffffffu;
    t[0] += c * 19;
    t[1] += t[0] >> 26;
    t[0] &= 0x3ffffffu;
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = t[i];
}

// Carry of the even limbs only: even limbs < 2^26, odd limbs grow by at most 2^6.  Half the instructions
// of fe_carry; enough for a multiplication's g operand whose limbs are a few units (19 g_j < 2^32 for odd
// limbs up to 6.7 units and even limbs up to 3.3) when fe_check_mul_in's column rule holds.
CV_HD void fe_carry_even(fe &h) {
#pragma unroll
    for (int i = 0; i < 10; i += 2) {
        h.v[i + 1] += h.v[i] >> 26;
        h.v[i] &= 0x3ffffffu;
    }
}

CV_HD uint64_t mu64(uint32_t a, uint32_t b) { return (uint64_t)a * (uint64_t)b; }

// The operand rules of fe_mul, checked exactly on the host build: 2 f_i (odd i) and 19 g_j fit 32 bits,
// and every column sum (x2 for odd x odd limbs, x19 past 2^255) stays below 2^63.9, which leaves room
// for the sequential carry-in (< 2^40).  The documented bounds (f <= 8, g <= 3.3 units) satisfy them;
// so do the refined ones some formulas use (g's odd limbs up to 6.7 units with a smaller f or even g).
CV_HD void fe_check_mul_in(const fe &f, const fe &g) {
#if CV_CHECKING
    for (int i = 0; i < 10; i++) {
        CV_ASSERT((uint64_t)f.v[i] * 2 < ((uint64_t)1 << 32), "fe_mul: 2*f overflows");
        CV_ASSERT(i == 0 || (uint64_t)g.v[i] * 19 < ((uint64_t)1 << 32), "fe_mul: 19*g overflows");
    }
    for (int k = 0; k < 10; k++) {
        unsigned __int128 sum = 0;
        for (int i = 0; i < 10; i++) {
            const int j = (k - i + 10) % 10;
            const uint64_t a = ((i & 1) && (j & 1)) ? 2ull * f.v[i] : f.v[i];
            const uint64_t b = i + j >= 10 ? 19ull * g.v[j] : g.v[j];
            sum += (unsigned __int128)a * b;
        }
        CV_ASSERT(sum < ((unsigned __int128)15 << 60), "fe_mul: column sum >= 2^63.9");
    }
#else
    (void)f; (void)g;
#endif
}

// Sequential-carry column accumulation: column k is accumulated on top of the carry out of column
// k-1, so a carry costs only its shift (the first v_mad_u64_u32 of the next column adds it for
// free) instead of shift + 64-bit add.  CV_MADC(acc, a, b): acc = a*b + acc as ONE v_mad_u64_u32,
// written in asm so the compiler cannot reassociate the carry to the end of the column sum.
// The mad's carry-out goes to VCC, declared as a clobber (round 1 bound it to an "=s" output).  The
// hardware needs no padding between dependent mads: distance 1, 2, 3 and 4 are exact
// (tools/microbench/mad_hazard.hip: 0 mismatches in 10^7 chained mads on MI355X).  LLVM, however,
// pads with "s_nop 0" any instruction that reads a VGPR written by the inline-asm statement
// IMMEDIATELY before it (it cannot see whether the asm used dst_sel forwarding) — 1,414 such nops in
// round 1's hs_straus.  So every mad is its own asm statement and the N independent chains of
// fe_mul_n / fe_sq_n are issued round-robin: chain m's next product is N statements later and never
// directly follows the statement that wrote its accumulator (N >= 2).
#ifdef __HIP_DEVICE_COMPILE__
#define CV_MADC(acc, a, b) asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b) : "vcc")
#else
#define CV_MADC(acc, a, b) ((acc) += (uint64_t)(a) * (uint64_t)(b))
#endif

template <int N> CV_HD void cv_madc_n(uint64_t (&t)[N], const uint32_t (&a)[N], const uint32_t (&b)[N]) {
#pragma unroll
    for (int m = 0; m < N; m++) CV_MADC(t[m], a[m], b[m]);
}

// Closing the sequential chain: the carry out of limb 9 (< 2^40) wraps into limb 0 as 19*c, and one
// more carry takes limb 0 back under 2^26 (limb 1 stays < M_1 + 2^19: tight).
CV_HD void fe_wrap_carry(fe &out, uint64_t c, uint32_t r[10]) {
    c = c * 19 + r[0];
    r[0] = (uint32_t)c & 0x3ffffffu;
    r[1] += (uint32_t)(c >> 26);
#pragma unroll
    for (int i = 0; i < 10; i++) out.v[i] = r[i];
}

// h[m] = f[m] * g[m] for m < N, interleaved (g[m] is the operand multiplied by 19: g <= 3.3, f <= 8).
// Column k holds f_i g_j for i + j = k (mod 10): x2 when i and j are both odd (half-bit offsets),
// x19 when i + j >= 10 (2^255 = 19).  Column sums stay < 2^63.7.
template <int N> CV_HD void fe_mul_n(fe (&h)[N], const fe (&f)[N], const fe (&g)[N]) {
    uint32_t fd[N][10], g19[N][10];
#pragma unroll
    for (int m = 0; m < N; m++) {
        fe_check_mul_in(f[m], g[m]);
#pragma unroll
        for (int i = 0; i < 10; i++) {
            fd[m][i] = (i & 1) ? 2 * f[m].v[i] : f[m].v[i];
            g19[m][i] = 19 * g[m].v[i];
        }
    }
    uint64_t t[N];
    uint32_t r[N][10];
#pragma unroll
    for (int m = 0; m < N; m++) t[m] = 0;
#pragma unroll
    for (int k = 0; k < 10; k++) {
        uint32_t a[10][N], b[10][N];
#pragma unroll
        for (int i = 0; i < 10; i++) {
            const int j = (k - i + 10) % 10;
            const bool dbl = (i & 1) && (j & 1);
            const bool wrap = i + j >= 10;
#pragma unroll
            for (int m = 0; m < N; m++) {
                a[i][m] = dbl ? fd[m][i] : f[m].v[i];
                b[i][m] = wrap ? g19[m][j] : g[m].v[j];
            }
        }
        cv_madc_col<N, 10>(t, a, b);
#pragma unroll
        for (int m = 0; m < N; m++) {
            r[m][k] = (uint32_t)t[m] & CV_MASK(k);
            t[m] >>= CV_W(k);
        }
    }
#pragma unroll
    for (int m = 0; m < N; m++) fe_wrap_carry(h[m], t[m], r[m]);
}

// Squaring: 55 products, column k as (left limb, left x1|x2, right limb, right x1|x2|x19|x38).
// DBL bit m set: h[m] = 2 f[m]^2 (every left factor doubled; left factors stay < 2^29.7).
// compile-time schedule (indices fold to constants inside the unrolled loops)
CV_HD constexpr int cv_sq_cols(int k, int q, int field) {
    // {l, lm, r, rm} of term q of column k; l = -1 marks an unused slot
    constexpr int8_t T[10][6][4] = {
        {{0, 1, 0, 1}, {1, 2, 9, 38}, {2, 2, 8, 19}, {3, 2, 7, 38}, {4, 2, 6, 19}, {5, 1, 5, 38}},
        {{0, 2, 1, 1}, {2, 1, 9, 38}, {3, 2, 8, 19}, {4, 1, 7, 38}, {5, 2, 6, 19}, {-1, 0, 0, 0}},
        {{0, 2, 2, 1}, {1, 2, 1, 1}, {3, 2, 9, 38}, {4, 2, 8, 19}, {5, 2, 7, 38}, {6, 1, 6, 19}},
        {{0, 2, 3, 1}, {1, 2, 2, 1}, {4, 1, 9, 38}, {5, 2, 8, 19}, {6, 1, 7, 38}, {-1, 0, 0, 0}},
        {{0, 2, 4, 1}, {1, 2, 3, 2}, {2, 1, 2, 1}, {5, 2, 9, 38}, {6, 2, 8, 19}, {7, 1, 7, 38}},
        {{0, 2, 5, 1}, {1, 2, 4, 1}, {2, 2, 3, 1}, {6, 1, 9, 38}, {7, 2, 8, 19}, {-1, 0, 0, 0}},
        {{0, 2, 6, 1}, {1, 2, 5, 2}, {2, 2, 4, 1}, {3, 2, 3, 1}, {7, 2, 9, 38}, {8, 1, 8, 19}},
        {{0, 2, 7, 1}, {1, 2, 6, 1}, {2, 2, 5, 1}, {3, 2, 4, 1}, {8, 1, 9, 38}, {-1, 0, 0, 0}},
        {{0, 2, 8, 1}, {1, 2, 7, 2}, {2, 2, 6, 1}, {3, 2, 5, 2}, {4, 1, 4, 1}, {9, 1, 9, 38}},
        {{0, 2, 9, 1}, {1, 2, 8, 1}, {2, 2, 7, 1}, {3, 2, 6, 1}, {4, 2, 5, 1}, {-1, 0, 0, 0}},
    };
    return T[k][q][field];
}

// rtk (0 or 1, run time): every chain additionally doubled (h = 2 f^2) — the per-lane doubling flag of
// the quad formulas; a literal 0 folds away.
template <int N, unsigned DBL = 0> CV_HD void fe_sq_n(fe (&h)[N], const fe (&f)[N], uint32_t rtk = 0) {
    // operand variants: left x1 / x2 (times 2 again for DBL chains), right x1 / x2 / x19 / x38
    uint32_t l1[N][10], l2[N][10], r2[N][10], r19[N][10], r38[N][10];
#pragma unroll
    for (int m = 0; m < N; m++) {
#if CV_CHECKING
        for (int i = 0; i < 10; i++)
            CV_ASSERT((uint64_t)f[m].v[i] * 10 < ((uint64_t)33 << CV_W(i)), "fe_sq: limb > 3.3M");
#endif
        const uint32_t k = ((DBL >> m) & 1u) + rtk;
#pragma unroll
        for (int i = 0; i < 10; i++) {
            l1[m][i] = f[m].v[i] << k;
            l2[m][i] = f[m].v[i] << (k + 1);
            r2[m][i] = 2 * f[m].v[i];
            r19[m][i] = 19 * f[m].v[i];
            r38[m][i] = 38 * f[m].v[i];
        }
    }
    uint64_t t[N];
    uint32_t r[N][10];
#pragma unroll
    for (int m = 0; m < N; m++) t[m] = 0;
#pragma unroll
    for (int k = 0; k < 10; k++) {
        constexpr int P0 = 6;
        uint32_t a[P0][N], b[P0][N];
#pragma unroll
        for (int q = 0; q < P0; q++) {
            const int li = cv_sq_cols(k, q, 0), lm = cv_sq_cols(k, q, 1);
            const int ri = cv_sq_cols(k, q, 2), rm = cv_sq_cols(k, q, 3);
#pragma unroll
            for (int m = 0; m < N; m++) {
                a[q][m] = li < 0 ? 0u : lm == 2 ? l2[m][li] : l1[m][li];
                b[q][m] = li < 0 ? 0u : rm == 1 ? f[m].v[ri] : rm == 2 ? r2[m][ri] : rm == 19 ? r19[m][ri] : r38[m][ri];
            }
        }
        // odd columns have 5 products (slot 5 unused), even columns 6
        if (k & 1) {
            const uint32_t(&a5)[5][N] = *reinterpret_cast<const uint32_t(*)[5][N]>(&a);
            const uint32_t(&b5)[5][N] = *reinterpret_cast<const uint32_t(*)[5][N]>(&b);
            cv_madc_col<N, 5>(t, a5, b5);
        } else {
            cv_madc_col<N, 6>(t, a, b);
        }
#pragma unroll
        for (int m = 0; m < N; m++) {
            r[m][k] = (uint32_t)t[m] & CV_MASK(k);
            t[m] >>= CV_W(k);
        }
    }
#pragma unroll
    for (int m = 0; m < N; m++) fe_wrap_carry(h[m], t[m], r[m]);
}

// single-operation forms
CV_HD void fe_mul(fe &h, const fe &f, const fe &g) {
    fe hh[1];
    const fe ff[1] = {f}, gg[1] = {g};
    fe_mul_n<1>(hh, ff, gg);
    h = hh[0];
}
CV_HD void fe_sq(fe &h, const fe &f) {
    fe hh[1];
    const fe ff[1] = {f};
    fe_sq_n<1, 0>(hh, ff);
    h = hh[0];
}
CV_HD void fe_sq2(fe &h, const fe &f) {
    fe hh[1];
    const fe ff[1] = {f};
    fe_sq_n<1, 1>(hh, ff);
    h = hh[0];
}

// Latency forms (the quad kernels, cv_quad.h, which run where the chip is under-occupied): ten
// independent column chains, then the carry chain with 64-bit adds — more instructions than the
// sequential-carry forms but no long dependent chain, which is what a lone wave per SIMD waits on.
// Floor carry of ten 64-bit column sums (each < 2^64) into a tight element.  Order: two
// interleaved chains (0..4, 4..9) and the 2^255 = 19 wrap, as in the classic 25.5-bit schedule.
#define CV_FCARRY(h, i, nxt)              \
    {                                     \
        nxt += h[i] >> CV_W(i);           \
        h[i] &= (uint64_t)CV_MASK(i);     \
    }
CV_HD void fe_reduce64(fe &out, uint64_t h[10]) {
    CV_FCARRY(h, 0, h[1]);
    CV_FCARRY(h, 4, h[5]);
    CV_FCARRY(h, 1, h[2]);
    CV_FCARRY(h, 5, h[6]);
    CV_FCARRY(h, 2, h[3]);
    CV_FCARRY(h, 6, h[7]);
    CV_FCARRY(h, 3, h[4]);
    CV_FCARRY(h, 7, h[8]);
    CV_FCARRY(h, 4, h[5]);
    CV_FCARRY(h, 8, h[9]);
    {
        const uint64_t c = h[9] >> 25;
        h[9] &= 0x1ffffffu;
        h[0] += c * 19;
    }
    CV_FCARRY(h, 0, h[1]);
#pragma unroll
    for (int i = 0; i < 10; i++) out.v[i] = (uint32_t)h[i];
}

CV_HD void fe_mul_ilp(fe &h, const fe &f, const fe &g) {
    fe_check_mul_in(f, g);
    const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
    const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
    const uint32_t g0 = g.v[0], g1 = g.v[1], g2 = g.v[2], g3 = g.v[3], g4 = g.v[4];
    const uint32_t g5 = g.v[5], g6 = g.v[6], g7 = g.v[7], g8 = g.v[8], g9 = g.v[9];
    // 19*g_j folds the 2^255 wrap; 2*f_i (odd i) pays the extra half bit of odd*odd offsets
    const uint32_t g1_19 = 19 * g1, g2_19 = 19 * g2, g3_19 = 19 * g3, g4_19 = 19 * g4, g5_19 = 19 * g5;
    const uint32_t g6_19 = 19 * g6, g7_19 = 19 * g7, g8_19 = 19 * g8, g9_19 = 19 * g9;
    const uint32_t f1_2 = 2 * f1, f3_2 = 2 * f3, f5_2 = 2 * f5, f7_2 = 2 * f7, f9_2 = 2 * f9;
    uint64_t h_[10];
    h_[0] = mu64(f0, g0) + mu64(f1_2, g9_19) + mu64(f2, g8_19) + mu64(f3_2, g7_19) + mu64(f4, g6_19) +
            mu64(f5_2, g5_19) + mu64(f6, g4_19) + mu64(f7_2, g3_19) + mu64(f8, g2_19) + mu64(f9_2, g1_19);
    h_[1] = mu64(f0, g1) + mu64(f1, g0) + mu64(f2, g9_19) + mu64(f3, g8_19) + mu64(f4, g7_19) +
            mu64(f5, g6_19) + mu64(f6, g5_19) + mu64(f7, g4_19) + mu64(f8, g3_19) + mu64(f9, g2_19);
    h_[2] = mu64(f0, g2) + mu64(f1_2, g1) + mu64(f2, g0) + mu64(f3_2, g9_19) + mu64(f4, g8_19) +
            mu64(f5_2, g7_19) + mu64(f6, g6_19) + mu64(f7_2, g5_19) + mu64(f8, g4_19) + mu64(f9_2, g3_19);
    h_[3] = mu64(f0, g3) + mu64(f1, g2) + mu64(f2, g1) + mu64(f3, g0) + mu64(f4, g9_19) +
            mu64(f5, g8_19) + mu64(f6, g7_19) + mu64(f7, g6_19) + mu64(f8, g5_19) + mu64(f9, g4_19);
    h_[4] = mu64(f0, g4) + mu64(f1_2, g3) + mu64(f2, g2) + mu64(f3_2, g1) + mu64(f4, g0) +
            mu64(f5_2, g9_19) + mu64(f6, g8_19) + mu64(f7_2, g7_19) + mu64(f8, g6_19) + mu64(f9_2, g5_19);
    h_[5] = mu64(f0, g5) + mu64(f1, g4) + mu64(f2, g3) + mu64(f3, g2) + mu64(f4, g1) +
            mu64(f5, g0) + mu64(f6, g9_19) + mu64(f7, g8_19) + mu64(f8, g7_19) + mu64(f9, g6_19);
    h_[6] = mu64(f0, g6) + mu64(f1_2, g5) + mu64(f2, g4) + mu64(f3_2, g3) + mu64(f4, g2) +
            mu64(f5_2, g1) + mu64(f6, g0) + mu64(f7_2, g9_19) + mu64(f8, g8_19) + mu64(f9_2, g7_19);
    h_[7] = mu64(f0, g7) + mu64(f1, g6) + mu64(f2, g5) + mu64(f3, g4) + mu64(f4, g3) +
            mu64(f5, g2) + mu64(f6, g1) + mu64(f7, g0) + mu64(f8, g9_19) + mu64(f9, g8_19);
    h_[8] = mu64(f0, g8) + mu64(f1_2, g7) + mu64(f2, g6) + mu64(f3_2, g5) + mu64(f4, g4) +
            mu64(f5_2, g3) + mu64(f6, g2) + mu64(f7_2, g1) + mu64(f8, g0) + mu64(f9_2, g9_19);
    h_[9] = mu64(f0, g9) + mu64(f1, g8) + mu64(f2, g7) + mu64(f3, g6) + mu64(f4, g5) +
            mu64(f5, g4) + mu64(f6, g3) + mu64(f7, g2) + mu64(f8, g1) + mu64(f9, g0);
    fe_reduce64(h, h_);
}

CV_HD void fe_sq_ilp(fe &h, const fe &f, bool dbl) {
#if CV_CHECKING
    for (int i = 0; i < 10; i++) CV_ASSERT((uint64_t)f.v[i] * 10 < ((uint64_t)33 << CV_W(i)), "fe_sq: limb > 3.3M");
#endif
    const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
    const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
    const uint32_t f0_2 = 2 * f0, f1_2 = 2 * f1, f2_2 = 2 * f2, f3_2 = 2 * f3, f4_2 = 2 * f4;
    const uint32_t f5_2 = 2 * f5, f6_2 = 2 * f6, f7_2 = 2 * f7;
    const uint32_t f5_38 = 38 * f5, f6_19 = 19 * f6, f7_38 = 38 * f7, f8_19 = 19 * f8, f9_38 = 38 * f9;
    uint64_t h_[10];
    h_[0] = mu64(f0, f0) + mu64(f1_2, f9_38) + mu64(f2_2, f8_19) + mu64(f3_2, f7_38) + mu64(f4_2, f6_19) +
            mu64(f5, f5_38);
    h_[1] = mu64(f0_2, f1) + mu64(f2, f9_38) + mu64(f3_2, f8_19) + mu64(f4, f7_38) + mu64(f5_2, f6_19);
    h_[2] = mu64(f0_2, f2) + mu64(f1_2, f1) + mu64(f3_2, f9_38) + mu64(f4_2, f8_19) + mu64(f5_2, f7_38) +
            mu64(f6, f6_19);
    h_[3] = mu64(f0_2, f3) + mu64(f1_2, f2) + mu64(f4, f9_38) + mu64(f5_2, f8_19) + mu64(f6, f7_38);
    h_[4] = mu64(f0_2, f4) + mu64(f1_2, f3_2) + mu64(f2, f2) + mu64(f5_2, f9_38) + mu64(f6_2, f8_19) +
            mu64(f7, f7_38);
    h_[5] = mu64(f0_2, f5) + mu64(f1_2, f4) + mu64(f2_2, f3) + mu64(f6, f9_38) + mu64(f7_2, f8_19);
    h_[6] = mu64(f0_2, f6) + mu64(f1_2, f5_2) + mu64(f2_2, f4) + mu64(f3_2, f3) + mu64(f7_2, f9_38) +
            mu64(f8, f8_19);
    h_[7] = mu64(f0_2, f7) + mu64(f1_2, f6) + mu64(f2_2, f5) + mu64(f3_2, f4) + mu64(f8, f9_38);
    h_[8] = mu64(f0_2, f8) + mu64(f1_2, f7_2) + mu64(f2_2, f6) + mu64(f3_2, f5_2) + mu64(f4, f4) +
            mu64(f9, f9_38);
    h_[9] = mu64(f0_2, f9) + mu64(f1_2, f8) + mu64(f2_2, f7) + mu64(f3_2, f6) + mu64(f4_2, f5);
    if (dbl) {
#pragma unroll
        for (int i = 0; i < 10; i++) h_[i] += h_[i];
    }
    fe_reduce64(h, h_);
}
// h = f^2 (dbl = false) or 2 f^2 (dbl = true), sequential-carry form with a run-time doubling flag
CV_HD void fe_sq_rt(fe &h, const fe &f, bool dbl) {
    fe hh[1];
    const fe ff[1] = {f};
    fe_sq_n<1, 0>(hh, ff, dbl ? 1u : 0u);
    h = hh[0];
}
// Field forms of the quad / tri latency kernels: SEQ = false the ILP forms (ten independent column
// chains + a 64-bit carry tree), true the sequential-carry forms (fewer instructions, one dependent
// chain per product)
template <bool SEQ> CV_HD void fe_mul_q(fe &h, const fe &f, const fe &g) {
    if constexpr (SEQ) fe_mul(h, f, g); else fe_mul_ilp(h, f, g);
}
template <bool SEQ> CV_HD void fe_sq_q(fe &h, const fe &f, bool dbl) {
    if constexpr (SEQ) fe_sq_rt(h, f, dbl); else fe_sq_ilp(h, f, dbl);
}
// Mode dispatch for the long single chains (key decoding, inversion): LAT = true selects the latency
// forms above (small batches, a lone wave per SIMD), false the sequential-carry forms (throughput).
template <bool LAT> CV_HD void fe_mul_m(fe &h, const fe &f, const fe &g) {
    if constexpr (LAT) fe_mul_ilp(h, f, g); else fe_mul(h, f, g);
}
template <bool LAT> CV_HD void fe_sq_m(fe &h, const fe &f) {
    if constexpr (LAT) fe_sq_ilp(h, f, false); else fe_sq(h, f);
}

// h = f^(2^n) (n >= 1).  A real loop keeps the code small; the trip count is hidden from the
// optimiser so it cannot unroll the short chains into long straight-line blocks that the machine
// scheduler then interleaves into VGPR spills.
template <bool LAT = false> __host__ __device__ __forceinline__ void fe_sqn(fe &h, const fe &f, int n) {
#ifdef __HIP_DEVICE_COMPILE__
    asm volatile("" : "+s"(n));
#endif
    fe_sq_m<LAT>(h, f);
#pragma nounroll
    for (int i = 1; i < n; i++) fe_sq_m<LAT>(h, h);
}

// Parse 32 little-endian bytes given as 8 uint32 words.  Bit 255 is ignored and the value is NOT
// reduced mod p (eddsa-0.1.0 Ed25519LittleEndianEncoding.decode semantics): y in [p, 2^255) is
// simply a non-canonical representative.  Output limbs are < M_i (tight).
CV_HD void fe_from_words(fe &h, const uint32_t w[8]) {
    const uint64_t W[4] = {w[0] | ((uint64_t)w[1] << 32), w[2] | ((uint64_t)w[3] << 32),
                           w[4] | ((uint64_t)w[5] << 32), w[6] | ((uint64_t)(w[7] & 0x7fffffffu) << 32)};
    auto bits = [&](int a, int n) -> uint32_t {
        const int q = a >> 6, r = a & 63;
        uint64_t x = W[q] >> r;
        if (r + n > 64 && q < 3) x |= W[q + 1] << (64 - r);
        return (uint32_t)(x & ((1ull << n) - 1));
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

// Canonical encoding (value mod p in [0, p)) as 8 little-endian uint32 words.  Input limbs < 2^31.
CV_HD void fe_to_words(uint32_t w[8], const fe &f) {
    fe t;
    fe_carry(t, f);
    uint32_t h[10];
#pragma unroll
    for (int i = 0; i < 10; i++) h[i] = t.v[i];
    // value < 2^255 + 2^26 here; q = 1 iff value >= p, i.e. iff value + 19 carries out of bit 255
    uint32_t q = (h[0] + 19) >> 26;
#pragma unroll
    for (int i = 1; i < 10; i++) q = (h[i] + q) >> CV_W(i);
    h[0] += 19 * q;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        h[i + 1] += h[i] >> CV_W(i);
        h[i] &= CV_MASK(i);
    }
    h[9] &= 0x1ffffffu;   // drop 2^255 * q
    w[0] = h[0] | (h[1] << 26);
    w[1] = (h[1] >> 6) | (h[2] << 19);
    w[2] = (h[2] >> 13) | (h[3] << 13);
    w[3] = (h[3] >> 19) | (h[4] << 6);
    w[4] = h[5] | (h[6] << 25);
    w[5] = (h[6] >> 7) | (h[7] << 19);
    w[6] = (h[7] >> 13) | (h[8] << 12);
    w[7] = (h[8] >> 20) | (h[9] << 6);
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
template <bool LAT = false> __host__ __device__ __forceinline__ void fe_pow22523(fe &out, const fe &z) {
    fe t0, t1, t2;
    fe_sq_m<LAT>(t0, z);            // z^2
    fe_sqn<LAT>(t1, t0, 2);       // z^8
    fe_mul_m<LAT>(t1, z, t1);       // z^9
    fe_mul_m<LAT>(t0, t0, t1);      // z^11
    fe_sq_m<LAT>(t0, t0);           // z^22
    fe_mul_m<LAT>(t0, t1, t0);      // z^31 = z^(2^5-1)
    fe_sqn<LAT>(t1, t0, 5);
    fe_mul_m<LAT>(t0, t1, t0);      // z^(2^10-1)
    fe_sqn<LAT>(t1, t0, 10);
    fe_mul_m<LAT>(t1, t1, t0);      // z^(2^20-1)
    fe_sqn<LAT>(t2, t1, 20);
    fe_mul_m<LAT>(t1, t2, t1);      // z^(2^40-1)
    fe_sqn<LAT>(t1, t1, 10);
    fe_mul_m<LAT>(t0, t1, t0);      // z^(2^50-1)
    fe_sqn<LAT>(t1, t0, 50);
    fe_mul_m<LAT>(t1, t1, t0);      // z^(2^100-1)
    fe_sqn<LAT>(t2, t1, 100);
    fe_mul_m<LAT>(t1, t2, t1);      // z^(2^200-1)
    fe_sqn<LAT>(t1, t1, 50);
    fe_mul_m<LAT>(t0, t1, t0);      // z^(2^250-1)
    fe_sqn<LAT>(t0, t0, 2);       // z^(2^252-4)
    fe_mul_m<LAT>(out, t0, z);      // z^(2^252-3)
}

// z^(p-2) = z^(2^255 - 21)
template <bool LAT = false> __host__ __device__ __forceinline__ void fe_invert(fe &out, const fe &z) {
    fe t0, t1, t2, t3;
    fe_sq_m<LAT>(t0, z);            // z^2
    fe_sqn<LAT>(t1, t0, 2);       // z^8
    fe_mul_m<LAT>(t1, z, t1);       // z^9
    fe_mul_m<LAT>(t0, t0, t1);      // z^11
    fe_sq_m<LAT>(t2, t0);           // z^22
    fe_mul_m<LAT>(t1, t1, t2);      // z^31
    fe_sqn<LAT>(t2, t1, 5);
    fe_mul_m<LAT>(t1, t2, t1);      // 2^10-1
    fe_sqn<LAT>(t2, t1, 10);
    fe_mul_m<LAT>(t2, t2, t1);      // 2^20-1
    fe_sqn<LAT>(t3, t2, 20);
    fe_mul_m<LAT>(t2, t3, t2);      // 2^40-1
    fe_sqn<LAT>(t2, t2, 10);
    fe_mul_m<LAT>(t1, t2, t1);      // 2^50-1
    fe_sqn<LAT>(t2, t1, 50);
    fe_mul_m<LAT>(t2, t2, t1);      // 2^100-1
    fe_sqn<LAT>(t3, t2, 100);
    fe_mul_m<LAT>(t2, t3, t2);      // 2^200-1
    fe_sqn<LAT>(t2, t2, 50);
    fe_mul_m<LAT>(t1, t2, t1);      // 2^250-1
    fe_sqn<LAT>(t1, t1, 5);       // 2^255-32
    fe_mul_m<LAT>(out, t1, t0);     // 2^255-21
}
