// cv_quad.h — latency form of the double-scalar multiplication: FOUR lanes per signature.
//
// For batches too small to fill the chip (a notary batch of 4096 signatures is 64 wave64s on 1024
// SIMDs) the time of a batch is the time of one signature's dependent chain.  The extended-
// coordinate formulas are 4-way parallel (Hisil-Wong-Carter-Dawson §4): lane r of a quad holds
// coordinate r of the point (X, Y, Z, T); a doubling is one squaring + one multiplication per lane
// (4S + 4M over the quad), an addition two multiplications per lane (8M), and the operands are
// exchanged inside the quad with DPP quad_perm moves.  Same group law, same points, hence the same
// verdicts; ~2.5x shorter chain per signature for ~1.5x the lane work (so it is only used where
// lanes are idle anyway — cvk_verify picks it by batch size).
//
// Device-only (DPP).  Limb bounds as in cv_field.h / cv_group.h; every exchanged operand is carried
// to tight before it feeds a multiplication.
#pragma once
#include "cv_verify.h"

#define CV_QP(a, b, c, d) ((a) | ((b) << 2) | ((c) << 4) | ((d) << 6))

template <int CTRL> __device__ __forceinline__ void fe_qp(fe &h, const fe &f) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)f.v[i], CTRL, 0xF, 0xF, true);
}

// the second half of both formulas: R1 = (F, H, G, E) on lanes 0..3 (even limbs carried, fe_carry_even) ->
// own coordinate of (X, Y, Z, T) = (E F, G H, F G, E H): each lane multiplies its own value by the one
// the quad_perm (3, 2, 0, 1) brings (one move per limb; the own operand needs none)
template <bool SEQ = false>
__device__ __forceinline__ void quad_finish_products(fe &P, const fe &R1) {
    fe op2;
    fe_qp<CV_QP(3, 2, 0, 1)>(op2, R1);   // E, G, F, H
    fe_mul_q<SEQ>(P, R1, op2);
}

// One limb moved inside the quad.  Written so that every moved value feeds only VOP2 operations (add,
// and, xor) with VGPR operands: LLVM's DPP combiner then folds the move into each of them (v_add_u32_dpp,
// v_xor_b32_dpp, ...) and no v_mov_b32_dpp is issued.  Lane-dependent signs use the identity
// (x XOR m) + (m AND (k p_i + 1)) = k p_i - x on the lanes where m is all ones, x on the others — two
// instructions instead of a subtraction on every lane plus a select.
template <int CTRL> __device__ __forceinline__ uint32_t qpv(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, true);
}
// all ones on the lanes where c holds.  Opaque to the optimiser: seen as a select, x AND mask became a
// v_cndmask (VOP3), which takes no DPP operand, and the move stayed.
__device__ __forceinline__ uint32_t lane_mask(bool c) {
    uint32_t m = c ? ~0u : 0u;
    asm volatile("" : "+v"(m));
    return m;
}

// P <- 2P.  P: own coordinate of an extended point (T is not read).  Squares on lanes 0..3: C = 2 Z^2,
// A = X^2, B = Y^2, S = (X + Y)^2; then lane 0 F' = C - G = C + A - B, lane 1 H' = A + B, lane 2 G = B - A,
// lane 3 E = S - H' (the negated-(F, H) doubling: (E F', G H', F' G, E H') is 2P).
template <bool SEQ = false>
__device__ __forceinline__ void quad_dbl(fe &P, int r) {
    const uint32_t m3 = lane_mask(r == 3);
    const uint32_t ma = lane_mask(r != 1), na = lane_mask(r >= 2);     // A: +, 0, -, -
    const uint32_t mb = lane_mask(r != 2), nb = lane_mask(r == 0 || r == 3);   // B: -, +, 0, -
    fe u, sq, R1;
    // lane 0 Z, lane 1 X, lane 2 Y, lane 3 X + Y (<= 2.02)
#pragma unroll
    for (int i = 0; i < 10; i++) u.v[i] = qpv<CV_QP(2, 0, 1, 1)>(P.v[i]) + (qpv<CV_QP(0, 0, 0, 0)>(P.v[i]) & m3);
    fe_sq_q<SEQ>(sq, u, r == 0);         // C, A, B, S (tight)
#pragma unroll
    for (int i = 0; i < 10; i++) {
        // own + (+-A or 0) + (+-B or 0), each negation x -> (x XOR ~0) + kp_i + 1:
        // F' = C + A + 2p - B (<= 4.02), H' = A + B (<= 2.02), G = B + 2p - A (<= 3.01), E = S + 4p - A - B (<= 5.01)
        const uint32_t ta = (qpv<CV_QP(1, 1, 1, 1)>(sq.v[i]) & ma) ^ na;
        const uint32_t tb = (qpv<CV_QP(2, 2, 2, 2)>(sq.v[i]) & mb) ^ nb;
        const uint32_t k = r == 1 ? 0u : r == 3 ? 2u * (cv_kp(2, i) + 1u) : cv_kp(2, i) + 1u;
        R1.v[i] = sq.v[i] + ta + tb + k;
    }
    fe_carry_even(R1);
    quad_finish_products<SEQ>(P, R1);
}

// P <- P + Q, q = this lane's coordinate of Q in cached form (Y+X, Y-X, Z, 2dT); for an affine
// "precomp" Q (y+x, y-x, 1, 2dxy) lane 2 passes the constant 1.  Products on lanes 0..3: a = (Y1+X1)(Y2+X2),
// b = (Y1-X1)(Y2-X2), dd = Z1 Z2, c = T1 2d T2; then lane 0 F = 2dd - c, lane 1 H = a + b, lane 2 G = 2dd + c,
// lane 3 E = a - b.
template <bool SEQ = false>
__device__ __forceinline__ void quad_add(fe &P, const fe &q, int r) {
    const uint32_t m01 = lane_mask(r < 2), m1 = lane_mask(r == 1);
    const uint32_t m02 = lane_mask(r == 0 || r == 2), n03 = lane_mask(r == 0 || r == 3);
    fe L, m, R1;
    // lane 0 Y + X (<= 2.02), lane 1 Y + 2p - X (<= 3.01), lanes 2, 3 their own Z, T
#pragma unroll
    for (int i = 0; i < 10; i++)
        L.v[i] = qpv<CV_QP(1, 1, 2, 3)>(P.v[i]) + ((qpv<CV_QP(0, 0, 0, 0)>(P.v[i]) & m01) ^ m1) +
                 (m1 & (cv_kp(2, i) + 1u));
    fe_mul_q<SEQ>(m, L, q);              // a, b, dd, c
#pragma unroll
    for (int i = 0; i < 10; i++) {
        // x = dd, a, dd, a (doubled on lanes 0, 2);  y = c, b, c, b (negated on lanes 0, 3)
        const uint32_t x = qpv<CV_QP(2, 0, 2, 0)>(m.v[i]) + (qpv<CV_QP(2, 0, 2, 0)>(m.v[i]) & m02);
        // F = 2dd + 2p - c (<= 4.02), H = a + b, G = 2dd + c (<= 3.03), E = a + 2p - b (<= 3.01)
        R1.v[i] = x + (qpv<CV_QP(3, 1, 3, 1)>(m.v[i]) ^ n03) + (n03 & (cv_kp(2, i) + 1u));
    }
    fe_carry_even(R1);
    quad_finish_products<SEQ>(P, R1);
}

// this lane's coordinate of +-k*(-A) from a per-signature cached table (40 words per entry, entry k = kP)
__device__ __forceinline__ void quad_cached_coord(fe &q, const uint32_t *tab, int a, int r) {
    const int m = a < 0 ? -a : a;
    const bool neg = a < 0;
    const int c = (r < 2 && neg) ? 1 - r : r;        // -(Y+X, Y-X, Z, T2d) = (Y-X, Y+X, Z, -T2d)
    const uint32_t *p = tab + 40 * m + 10 * c;           // entry 0 = identity (1, 1, 1, 0)
    const uint2 *p2 = reinterpret_cast<const uint2 *>(p);
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint2 v = p2[j];
        q.v[2 * j] = v.x;
        q.v[2 * j + 1] = v.y;
    }
    fe nq;
    fe_neg(nq, q);
    fe_sel(q, q, nq, neg && r == 3);
}

// this lane's coordinate of +-|d| * P from an affine table (entries `stride` words apart: y+x at 0,
// y-x at 10, 2dxy at 20); lane 2 gets the constant Z = 1.  ident_row: row 0 of the table is the
// identity (the basepoint tables); otherwise entry k-1 holds k * P and d = 0 yields the identity.
__device__ __forceinline__ void quad_precomp_coord(fe &q, const uint32_t *tab, int stride, int a, int r,
                                                   bool ident_row) {
    const int m = a < 0 ? -a : a;
    const bool neg = a < 0;
    const int c = (r < 2) ? (neg ? 1 - r : r) : 2;   // lane 3 reads 2dxy; lane 2's word is unused
    const int row = ident_row ? m : (m ? m - 1 : 0);
    const uint32_t *p = tab + stride * row + 10 * c;
    const uint2 *p2 = reinterpret_cast<const uint2 *>(p);
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint2 v = p2[j];
        q.v[2 * j] = v.x;
        q.v[2 * j + 1] = v.y;
    }
    fe nq, one, zero;
    fe_neg(nq, q);
    fe_sel(q, q, nq, neg && r == 3);
    fe_one(one);
    fe_sel(q, q, one, r == 2);
    if (!ident_row) {
        fe_zero(zero);
        fe_sel(q, q, r == 3 ? zero : one, m == 0);
    }
}

// Quad version of cv_comb_straus (keyed path, reference schedule): affine key rows (entry k =
// k * 2^(64 j)(-A), entry 0 the identity), radix-16 digits of h, radix-256 CV_BCOMB rows for s.
__device__ __forceinline__ void cv_quad_comb(const uint32_t *bcomb, const uint32_t *hs, const uint32_t *ktab, int r,
                                             fe &P) {
    uint32_t h[8], s[8];
#pragma unroll
    for (int q = 0; q < 8; q++) { h[q] = hs[q]; s[q] = hs[8 + q]; }
    fe_zero(P);
    if (r == 1 || r == 2) P.v[0] = 1;
#pragma unroll 1
    for (int u = 15; u >= 0; u--) {
        if (u != 15) {
            quad_dbl(P, r);
            quad_dbl(P, r);
            quad_dbl(P, r);
            quad_dbl(P, r);
        }
#pragma unroll
        for (int j = 0; j < CV_COMB_ROWS; j++) {
            fe q;
            quad_precomp_coord(q, ktab + j * CV_KROW_WORDS, CV_KENT_WORDS, digit16(h, 16 * j + u), r, true);
            quad_add(P, q, r);
        }
        if ((u & 1) == 0) {
#pragma unroll
            for (int j = 0; j < CV_COMB_ROWS; j++) {
                fe q;
                quad_precomp_coord(q, bcomb + j * CV_BTAB_ENTRIES * CV_BTAB_STRIDE, CV_BTAB_STRIDE,
                                   digit256(s, 8 * j + (u >> 1)), r, true);
                quad_add(P, q, r);
            }
        }
    }
}
