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
// Returns E == O on every lane of the quad.
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
            quad_dbl(P, r);
            quad_dbl(P, r);
            quad_dbl(P, r);
            quad_dbl(P, r);
        }
        fe q;
        quad_cached_coord(q, tabR, cv_sfield(dw, 5, 5), r);
        quad_add(P, q, r);
        quad_cached_coord(q, tabA, cv_sfield(dw, 0, 5), r);
        quad_add(P, q, r);
        if ((win & 1) == 0 && win < 32) {
            quad_precomp_coord(q, blo, CV_BTAB_STRIDE, cv_sfield(dw, 10, 9), r, true);
            quad_add(P, q, r);
            quad_precomp_coord(q, bhi, CV_BTAB_STRIDE, cv_sfield(dw, 19, 9), r, true);
            quad_add(P, q, r);
        }
    }
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
