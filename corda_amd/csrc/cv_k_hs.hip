// cv_k_hs.hip — half-size throughput group: scalars -> points -> hs_straus (the C2 / C3 / C5 hot path).
// Shared helpers and every kernel declaration: cv_kcommon.h; launchers: cv_kernels.hip.
#include "cv_kcommon.h"

// (WAVES: the waves per SIMD its register budget is built for; 3 spills ~64 VGPRs of the SHA-512 state)
template <int WAVES>
__global__ __launch_bounds__(CV_BLOCK, WAVES) void cv_scalars_kernel(uint32_t n, uint32_t cap, const uint8_t *__restrict__ pk,
                                                                 const uint8_t *__restrict__ sig,
                                                                 const uint8_t *__restrict__ arena,
                                                                 const uint64_t *__restrict__ off,
                                                                 const uint32_t *__restrict__ len,
                                                                 uint32_t *__restrict__ ws_dig) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i < n) cv_scalars_lane(i, cap, pk, sig, arena, off, len, ws_dig);
}

// points of the half-size group (throughput form): A and R decoded as one interleaved pair per lane,
// both odd-multiple tables (cv_hs_points); ws_ok = key_ok AND r_ok, status = key status.
template <bool SUB>
__global__ __launch_bounds__(CV_BLOCK, 2) void cv_points_kernel(uint32_t n, const uint8_t *__restrict__ pk,
                                                                const uint8_t *__restrict__ sig,
                                                                uint32_t *__restrict__ ws_tab,
                                                                uint32_t *__restrict__ ws_tabR,
                                                                uint8_t *__restrict__ ws_ok,
                                                                uint8_t *__restrict__ status) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t aw[8], rw[8];
    load_words8(aw, pk + (size_t)i * 32);
    load_words8(rw, sig + (size_t)i * 64);
    bool ok = false;
    const bool key_ok = cv_hs_points<false>(aw, rw, ws_tab + (size_t)i * CV_TAB_WORDS, ws_tabR + (size_t)i * CV_TAB_WORDS,
                                            ok);
    ws_ok[i] = ok ? 1 : 0;
    if (status) status[i] = key_ok ? 0 : 1;
}

// points of the half-size group, lane-pair throughput form: the even lane decodes A into k*(-A), the
// odd lane R into k*R (cv_hs_point_one with the sequential-carry field forms), so a lane holds one
// decode's state instead of two and the kernel fits WAVES waves per SIMD.  Grid 2n lanes.
template <int WAVES, bool SUB>
__global__ __launch_bounds__(CV_BLOCK, WAVES) void cv_points_one_kernel(uint32_t n, const uint8_t *__restrict__ pk,
                                                                        const uint8_t *__restrict__ sig,
                                                                        uint32_t *__restrict__ ws_tab,
                                                                        uint32_t *__restrict__ ws_tabR,
                                                                        uint8_t *__restrict__ ws_ok,
                                                                        uint8_t *__restrict__ status) {
    cv_points_one_lane(blockIdx.x * CV_BLOCK + threadIdx.x, n, pk, sig, ws_tab, ws_tabR, ws_ok, status);
}

// scalars and points of the half-size group in ONE launch (throughput form): blocks [0, nbp) run the
// point lane pairs, blocks [nbp, grid) the scalars.  The two roles are independent (both read only
// the inputs), so the short scalar waves, dispatched last, fill the partial last round of the point
// waves instead of paying a kernel boundary (drain + launch) of their own.  Both roles fit 3 waves
// per SIMD; every wave is one role (blocks are role-uniform), so the lane-pair shuffle stays valid.
template <bool SUB>
__global__ __launch_bounds__(CV_BLOCK, 3) void cv_prep_tp_kernel(uint32_t n, uint32_t cap, uint32_t nbp,
                                                                 const uint8_t *__restrict__ pk,
                                                                 const uint8_t *__restrict__ sig,
                                                                 const uint8_t *__restrict__ arena,
                                                                 const uint64_t *__restrict__ off,
                                                                 const uint32_t *__restrict__ len,
                                                                 uint32_t *__restrict__ ws_dig,
                                                                 uint32_t *__restrict__ ws_tab,
                                                                 uint32_t *__restrict__ ws_tabR,
                                                                 uint8_t *__restrict__ ws_ok,
                                                                 uint8_t *__restrict__ status) {
    if (blockIdx.x < nbp) {
        cv_points_one_lane(blockIdx.x * CV_BLOCK + threadIdx.x, n, pk, sig, ws_tab, ws_tabR, ws_ok, status);
    } else {
        const uint32_t i = (blockIdx.x - nbp) * CV_BLOCK + threadIdx.x;
        if (i < n) cv_scalars_lane(i, cap, pk, sig, arena, off, len, ws_dig);
    }
}

// hs_straus: E = [v]R + [u]A + [w]B per lane over the wave's largest window count, the identity
// test, and the verdict word by wave ballot (bit i of word i/64 = signature i).  Lanes past n
// replay signature n-1 so the whole wave takes part in the window-count reduction.
template <int WAVES, bool SUB>
__global__ __launch_bounds__(CV_BLOCK, WAVES) void cv_hs_straus_kernel(uint32_t n, uint32_t cap,
                                                                       const uint32_t *__restrict__ ws_dig,
                                                                       const uint32_t *__restrict__ ws_tab,
                                                                       const uint32_t *__restrict__ ws_tabR,
                                                                       const uint8_t *__restrict__ ws_ok,
                                                                       uint64_t *__restrict__ bitmap) {
    // LDS rows padded to CV_BTAB_LDS_STRIDE words: the 64 lanes of a wave gather data-dependent rows,
    // and with 128-B rows every row started in one of two 4-bank groups (32-way conflicts); with
    // 144-B rows consecutive row indices start 36 words apart and spread over 16 groups
    __shared__ __attribute__((aligned(16))) uint32_t btab[2 * CV_BTAB_ENTRIES * CV_BTAB_LDS_STRIDE];
    constexpr int ROW = CV_BTAB_ENTRIES * CV_BTAB_STRIDE, LROW = CV_BTAB_ENTRIES * CV_BTAB_LDS_STRIDE;
    for (int k = threadIdx.x; k < ROW; k += blockDim.x) {
        const int at = (k / CV_BTAB_STRIDE) * CV_BTAB_LDS_STRIDE + k % CV_BTAB_STRIDE;
        btab[at] = CV_BCOMB[k];                  // k * B
        btab[LROW + at] = CV_BCOMB[2 * ROW + k]; // k * 2^128 * B
    }
    __syncthreads();
    const uint32_t wave0 = blockIdx.x * CV_BLOCK + (threadIdx.x & ~63u);
    if (wave0 >= n) return;                    // whole waves past the end leave together
    const uint32_t i0 = wave0 + (threadIdx.x & 63u);
    const uint32_t i = i0 < n ? i0 : n - 1;
    int nw = (int)ws_dig[(size_t)64 * cap + i];
    nw = nw < 32 ? 32 : nw;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const int x = __shfl_xor(nw, o);
        nw = x > nw ? x : nw;
    }
    nw = __builtin_amdgcn_readfirstlane(nw);
    const bool eq = cv_hs_straus<CV_BTAB_LDS_STRIDE>(btab, btab + LROW, ws_dig + i, cap, ws_tab + (size_t)i * CV_TAB_WORDS,
                                 ws_tabR + (size_t)i * CV_TAB_WORDS, nw);
    const bool acc = eq && ws_ok[i] && i0 < n;
    const uint64_t bits = __ballot(acc);
    if ((threadIdx.x & 63u) == 0) bitmap[wave0 >> 6] = bits;
}
template __global__ void cv_hs_straus_kernel<2>(uint32_t, uint32_t, const uint32_t *, const uint32_t *,
                                                const uint32_t *, const uint8_t *, uint64_t *);
template __global__ void cv_hs_straus_kernel<3>(uint32_t, uint32_t, const uint32_t *, const uint32_t *,
                                                const uint32_t *, const uint8_t *, uint64_t *);
template __global__ void cv_hs_straus_kernel<2, true>(uint32_t, uint32_t, const uint32_t *, const uint32_t *,
                                                      const uint32_t *, const uint8_t *, uint64_t *);
template __global__ void cv_hs_straus_kernel<3, true>(uint32_t, uint32_t, const uint32_t *, const uint32_t *,
                                                      const uint32_t *, const uint8_t *, uint64_t *);

template __global__ void cv_points_kernel<false>(uint32_t n, const uint8_t *pk, const uint8_t *sig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status);
template __global__ void cv_points_kernel<true>(uint32_t n, const uint8_t *pk, const uint8_t *sig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status);
template __global__ void cv_points_one_kernel<2, false>(uint32_t n, const uint8_t *pk, const uint8_t *sig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status);
template __global__ void cv_points_one_kernel<2, true>(uint32_t n, const uint8_t *pk, const uint8_t *sig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status);
template __global__ void cv_points_one_kernel<3, false>(uint32_t n, const uint8_t *pk, const uint8_t *sig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status);
template __global__ void cv_points_one_kernel<3, true>(uint32_t n, const uint8_t *pk, const uint8_t *sig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status);
template __global__ void cv_prep_tp_kernel<false>(uint32_t n, uint32_t cap, uint32_t nbp, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *ws_dig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status);
template __global__ void cv_prep_tp_kernel<true>(uint32_t n, uint32_t cap, uint32_t nbp, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *ws_dig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status);
template __global__ void cv_scalars_kernel<2>(uint32_t n, uint32_t cap, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *ws_dig);
template __global__ void cv_scalars_kernel<3>(uint32_t n, uint32_t cap, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *ws_dig);
