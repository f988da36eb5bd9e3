// cv_hsquad.h — the half-size-scalar schedule (cv_verify.h "half-size verify") in the quad latency
// form (cv_quad.h): four lanes per signature hold the four extended coordinates, so a notary-sized
// batch (a few thousand signatures: far fewer waves than the chip has SIMDs) runs ~128 doublings of
// 4-way parallel formulas per signature instead of the full-width ~252.
//
// Device-only (DPP quad_perm).  Same group law, same points, same identity test, hence the same
// verdicts as cv_hs_straus; tests/test_gpu_parity.py checks both forms against the oracle.
#pragma once
#include "cv_quad.h"

// E = [v]R + [u]A + [w]B from the packed window digits (cv_verify.h), nw windows (uniform over the
// wave); blo / bhi = k*B and k*2^128*B rows (row 0 = identity), tabA = k*(-A), tabR = k*R (cached).
// W16: w's radix-2^16 digit pairs every fourth window from the CV_BW16 rows (as cv_hs_straus<.., true>),
// else radix-256 digits every other window from CV_BCOMB.  Returns E == O on every lane of the quad.
template <bool W16 = false, bool SEQ = false>
__device__ __forceinline__ bool cv_quad_hs_straus(const uint32_t *blo, const uint32_t *bhi, const uint32_t *dig,
                                                  size_t stride, const uint32_t *tabA, const uint32_t *tabR, int nw,
                                                  int r) {
    fe P;
    fe_zero(P);
    if (r == 1 || r == 2) P.v[0] = 1;          // identity (0, 1, 1, 0)
#pragma unroll 1
    for (int win = nw - 1; win >= 0; win--) {
        const uint32_t dw = dig[(size_t)win * stride];
        if (win != nw - 1) {
            quad_dbl<SEQ>(P, r);
            quad_dbl<SEQ>(P, r);
            quad_dbl<SEQ>(P, r);
            quad_dbl<SEQ>(P, r);
        }
        fe q;
        quad_cached_coord(q, tabR, cv_sfield(dw, 5, 5), r);
        quad_add<SEQ>(P, q, r);
        quad_cached_coord(q, tabA, cv_sfield(dw, 0, 5), r);
        quad_add<SEQ>(P, q, r);
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
            quad_precomp_coord(q, blo, CV_BTAB_STRIDE, dlo, r, true);
            quad_add<SEQ>(P, q, r);
            quad_precomp_coord(q, bhi, CV_BTAB_STRIDE, dhi, r, true);
            quad_add<SEQ>(P, q, r);
        }
    }
    fe X, Y, Z, d;
    fe_qp<CV_QP(0, 0, 0, 0)>(X, P);
    fe_qp<CV_QP(1, 1, 1, 1)>(Y, P);
    fe_qp<CV_QP(2, 2, 2, 2)>(Z, P);
    fe_sub<2>(d, Y, Z);
    return fe_is_zero(X) && fe_is_zero(d);
}

// ---------------------------------------------------------------- tri-chain form (smallest batches)
// Sixteen lanes per signature, four quads running four INDEPENDENT chains in lockstep — quad 0
// [v]R, quad 1 [u](-A), quad 2 [w_lo]B, quad 3 [w_hi] 2^128 B (w = w_lo + 2^128 w_hi, radix-16
// digits: cv_hs_scalars<true>) — each one add per window after four doublings, then summed by a
// two-step rotation tree inside the 16-lane DPP row.  The per-signature chain is 4 doublings + 1
// add per window instead of 4 + 2 (+2 every other window): ~0.67x the serial work of the quad
// form, for 4x its lanes (4 signatures per wave).  Only for batches whose waves leave SIMDs idle.

// this lane's coordinate of d * P, cached form, from either table format: the per-signature cached
// tables (precomp = false: 40 words per entry, entry k = k P, entry 0 = identity) or the CV_BCOMB affine rows
// (precomp = true: stride CV_BTAB_STRIDE, row k = k P, row 0 = identity; Z = 1).  Same instructions
// on every lane (only addresses and selects differ), so the four quads never diverge.
__device__ __forceinline__ void quad_any_coord(fe &q, const uint32_t *tab, bool precomp, int a, int r) {
    const int m = a < 0 ? -a : a;
    const bool neg = a < 0;
    const int c = (r < 2 && neg) ? 1 - r : r;            // -(Y+X, Y-X, Z, T2d) = (Y-X, Y+X, Z, -T2d)
    const int stride = precomp ? CV_BTAB_STRIDE : 40;
    const int row = m;                                   // row 0 = identity in both formats
    const int offc = (precomp && r == 3) ? 20 : 10 * c;  // affine rows: 2dxy at word 20
    const uint2 *p2 = reinterpret_cast<const uint2 *>(tab + stride * row + offc);
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint2 v = p2[j];
        q.v[2 * j] = v.x;
        q.v[2 * j + 1] = v.y;
    }
    fe nq, one;
    fe_neg(nq, q);
    fe_sel(q, q, nq, neg && r == 3);
    fe_one(one);
    fe_sel(q, q, one, precomp && r == 2);
}

// this lane's coordinate of a full extended point in cached form (Y+X, Y-X, Z, 2dT), from each
// lane's own coordinate of (X, Y, Z, T)
template <bool SEQ = false>
__device__ __forceinline__ void quad_to_cached(fe &q, const fe &P, int r) {
    fe x, y, s, d, t, d2;
    fe_const_d2(d2);
    fe_qp<CV_QP(0, 0, 0, 0)>(x, P);
    fe_qp<CV_QP(1, 1, 1, 1)>(y, P);
    fe_add(s, y, x);
    fe_sub<2>(d, y, x);
    fe_mul_q<SEQ>(t, P, d2);                // lane 3: 2d T (other lanes discard it)
    fe_sel(q, P, t, r == 3);
    fe_sel(q, q, d, r == 1);
    fe_sel(q, q, s, r == 0);
    fe_carry(q, q);
}

template <int CTRL> __device__ __forceinline__ void fe_dpp_row(fe &h, const fe &f) {
#pragma unroll
    for (int i = 0; i < 10; i++) h.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)f.v[i], CTRL, 0xF, 0xF, false);
}

// E = [v]R + [u]A + [w]B by four chains (quad c of the 16-lane group, coordinate r); returns E == O
// on every lane.  tab / precomp / field: this quad's table and digit field (5 bits at `field`).
// (Loading each window's entry one window ahead, behind the four doublings, measured 2-4 us SLOWER at 256,
// 1,024, 2,048 and 4,096 signatures on one box and 2.7 us faster at 4,096 on another: not kept,
// tools/microbench/lat_parts.hip, profiles/r04_tri_quad_formulas.log.)
template <bool SEQ = false>
__device__ __forceinline__ bool cv_tri_hs_straus(const uint32_t *dig, size_t stride, const uint32_t *tab, bool precomp,
                                                 int field, int nw, int r) {
    fe P, q;
    fe_zero(P);
    if (r == 1 || r == 2) P.v[0] = 1;                    // identity (0, 1, 1, 0)
#pragma unroll 1
    for (int win = nw - 1; win >= 0; win--) {
        const uint32_t dw = dig[(size_t)win * stride];
        if (win != nw - 1) {
            quad_dbl<SEQ>(P, r);
            quad_dbl<SEQ>(P, r);
            quad_dbl<SEQ>(P, r);
            quad_dbl<SEQ>(P, r);
        }
        quad_any_coord(q, tab, precomp, cv_sfield(dw, field, 5), r);
        quad_add<SEQ>(P, q, r);
    }
    // every quad adds the quad 4 lanes away, then the quad 8 lanes away (row rotations): each quad
    // ends with the sum of all four chains
    fe Q;
    fe_dpp_row<0x124>(Q, P);                             // row_ror:4
    quad_to_cached<SEQ>(q, Q, r);
    quad_add<SEQ>(P, q, r);
    fe_dpp_row<0x128>(Q, P);                             // row_ror:8
    quad_to_cached<SEQ>(q, Q, r);
    quad_add<SEQ>(P, q, r);
    fe X, Y, Z, d;
    fe_qp<CV_QP(0, 0, 0, 0)>(X, P);
    fe_qp<CV_QP(1, 1, 1, 1)>(Y, P);
    fe_qp<CV_QP(2, 2, 2, 2)>(Z, P);
    fe_sub<2>(d, Y, Z);
    return fe_is_zero(X) && fe_is_zero(d);
}

// 16 signatures per wave: the quad-lane-0 bits of a ballot (lanes 0, 4, ..., 60) -> 16 bits
__device__ __forceinline__ uint32_t cv_quad_ballot_bits(uint64_t b) {
    b &= 0x1111111111111111ull;
    b = (b | (b >> 3)) & 0x0303030303030303ull;
    b = (b | (b >> 6)) & 0x000f000f000f000full;
    b = (b | (b >> 12)) & 0x000000ff000000ffull;
    b = (b | (b >> 24)) & 0xffffull;
    return (uint32_t)b;
}
