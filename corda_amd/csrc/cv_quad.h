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

// the second half of both formulas: R1 = (H, G, F, E) on lanes 0..3 (tight) ->
// own coordinate of (X, Y, Z, T) = (E F, G H, F G, E H)
template <bool SEQ = false>
__device__ __forceinline__ void quad_finish_products(fe &P, const fe &R1) {
    fe op1, op2;
    fe_qp<CV_QP(3, 1, 2, 3)>(op1, R1);   // E, G, F, E
    fe_qp<CV_QP(2, 0, 1, 0)>(op2, R1);   // F, H, G, H
    fe_mul_q<SEQ>(P, op1, op2);
}

// P <- 2P.  P: own coordinate of an extended point (T is not read).
template <bool SEQ = false>
__device__ __forceinline__ void quad_dbl(fe &P, int r) {
    fe w, x, u, sq;
    fe_qp<CV_QP(0, 1, 2, 1)>(w, P);      // X, Y, Z, Y
    fe_qp<CV_QP(0, 0, 0, 0)>(x, P);      // X everywhere
#pragma unroll
    for (int i = 0; i < 10; i++) u.v[i] = w.v[i] + (r == 3 ? x.v[i] : 0u);   // lane 3: X + Y (<= 2.02)
    fe_sq_q<SEQ>(sq, u, r == 2);         // A = X^2, B = Y^2, C = 2 Z^2, S = (X + Y)^2   (tight)
    fe a, b, hp, g, t, d, R1;
    fe_qp<CV_QP(0, 0, 0, 0)>(a, sq);
    fe_qp<CV_QP(1, 1, 1, 1)>(b, sq);
    fe_add(hp, a, b);                    // H' = A + B          <= 2.02
    fe_sub<2>(g, b, a);                  // G  = B - A          <= 3.01
    fe_sel(t, g, hp, r == 0 || r == 3);
    fe_sub<4>(d, sq, t);                 // lane 2: F' = C - G, lane 3: E = S - H'   (<= 6.03)
    fe_sel(R1, t, d, r >= 2);
    fe_carry(R1, R1);
    quad_finish_products<SEQ>(P, R1);    // (E F', G H', F' G, E H') — the negated-(F, H) doubling, same point
}

// P <- P + Q, q = this lane's coordinate of Q in cached form (Y+X, Y-X, Z, 2dT); for an affine
// "precomp" Q (y+x, y-x, 1, 2dxy) lane 2 passes the constant 1.
template <bool SEQ = false>
__device__ __forceinline__ void quad_add(fe &P, const fe &q, int r) {
    fe y, x, s, d, L, m;
    fe_qp<CV_QP(1, 1, 2, 3)>(y, P);      // Y, Y, Z, T
    fe_qp<CV_QP(0, 0, 2, 3)>(x, P);      // X, X, Z, T
    fe_add(s, y, x);                     // lane 0: Y + X      <= 2.02
    fe_sub<2>(d, y, x);                  // lane 1: Y - X      <= 3.01
    fe_sel(L, y, d, r == 1);
    fe_sel(L, L, s, r == 0);             // lanes 2, 3: Z, T
    fe_mul_q<SEQ>(m, L, q);              // a, b, dd = Z1 Z2, c = T1 2d T2
    fe o1, o2, sum, diff, R1;
    fe_qp<CV_QP(0, 2, 2, 0)>(o1, m);     // a, dd, dd, a
    const uint32_t sh = (r == 1 || r == 2) ? 1u : 0u;
#pragma unroll
    for (int i = 0; i < 10; i++) o1.v[i] <<= sh;   // 2 dd on lanes 1, 2 (<= 2.02)
    fe_qp<CV_QP(1, 3, 3, 1)>(o2, m);     // b, c, c, b
    fe_add(sum, o1, o2);                 // lane 0: H = a + b, lane 1: G = 2dd + c
    fe_sub<2>(diff, o1, o2);             // lane 2: F = 2dd - c, lane 3: E = a - b
    fe_sel(R1, diff, sum, r < 2);
    fe_carry(R1, R1);
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

// Quad version of cv_verify_straus: R' = [h](-A) + [s]B; lanes 0..2 return X, Y, Z.
__device__ __forceinline__ void cv_quad_straus(const uint32_t *btab, const uint32_t *hs, const uint32_t *tab, int r,
                                               fe &P) {
    uint32_t h[8], s[8];
#pragma unroll
    for (int q = 0; q < 8; q++) { h[q] = hs[q]; s[q] = hs[8 + q]; }
    fe_zero(P);
    if (r == 1 || r == 2) P.v[0] = 1;          // identity (0, 1, 1, 0)
#pragma unroll 1
    for (int w = 63; w >= 0; w--) {
        if (w != 63) {
            quad_dbl(P, r);
            quad_dbl(P, r);
            quad_dbl(P, r);
            quad_dbl(P, r);
        }
        fe q;
        quad_cached_coord(q, tab, digit16(h, w), r);
        quad_add(P, q, r);
        if ((w & 1) == 0) {
            // B table rows: k*B for k = 0..128 (row 0 = identity), stride CV_BTAB_STRIDE
            quad_precomp_coord(q, btab, CV_BTAB_STRIDE, digit256(s, w >> 1), r, true);
            quad_add(P, q, r);
        }
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
