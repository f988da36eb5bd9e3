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
    if (i < n) cv_scalars_lane<false, true>(i, cap, pk, sig, arena, off, len, ws_dig);
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

// The CV_BW16 table: row r (0..3), entry k (0 .. 2^15) = k * 2^(64 r) * B as an affine precomp
// (y+x, y-x, 2dxy), canonical limbs, CV_BTAB_STRIDE words per entry (30 used).  Built once per device
// (cv_kernels.hip: bw16_table) by one lane per entry: [k 2^(128 r)]B from the radix-256 basepoint
// table in LDS, then Z^-1.
__global__ __launch_bounds__(CV_BLOCK) void cv_bw16_init_kernel(uint32_t *__restrict__ tab) {
    __shared__ __attribute__((aligned(16))) uint32_t btab[CV_BTAB_ENTRIES * CV_BTAB_STRIDE];
    stage_btab(btab);
    const uint32_t t = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (t >= CV_BW16_ROWS * CV_BW16_ENTRIES) return;
    const uint32_t row = t / CV_BW16_ENTRIES, k = t % CV_BW16_ENTRIES;
    uint32_t sc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; q++) sc[2 * q] = (uint32_t)q == row ? k : 0u;   // k * 2^(64 row)
    ge_p3 P;
    ge_scalarmult_base(P, sc, btab);
    fe zi, x, y, xy, d2, f[3];
    fe_invert(zi, P.Z);
    fe_mul(x, P.X, zi);
    fe_mul(y, P.Y, zi);
    fe_add(f[0], y, x);
    fe_sub<2>(f[1], y, x);
    fe_mul(xy, x, y);
    fe_const_d2(d2);
    fe_mul(f[2], xy, d2);
    uint32_t *o = tab + (size_t)t * CV_BTAB_STRIDE;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        uint32_t w[8];
        fe_to_words(w, f[c]);                  // canonical (< p): limbs < M_i after the re-split
        fe canon;
        fe_from_words(canon, w);
        fe_store(o + 10 * c, canon);
    }
    o[30] = o[31] = 0;
}
template __global__ void cv_points_one_kernel<3, false>(uint32_t n, const uint8_t *pk, const uint8_t *sig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status);
template __global__ void cv_points_one_kernel<3, true>(uint32_t n, const uint8_t *pk, const uint8_t *sig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status);
template __global__ void cv_scalars_kernel<3>(uint32_t n, uint32_t cap, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *ws_dig);
