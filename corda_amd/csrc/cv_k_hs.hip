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

// The scalars in two launches (cvk_set_scalars_split): the SHA-512 challenge hash (+ effective S) and
// the lattice + window digits each at the occupancy its own registers allow — inside one kernel the
// hash's live state and the lattice's multi-word remainders shared one 168-VGPR budget and spilled.
// h || s go through ws_hs as four 16-B planes (plane p at word (p * cap + i) * 4), so each store and
// load of a wave is one contiguous 1-KB stretch.
template <int WAVES>
__global__ __launch_bounds__(CV_BLOCK, WAVES) void cv_hash_kernel(uint32_t n, uint32_t cap, const uint8_t *__restrict__ pk,
                                                              const uint8_t *__restrict__ sig,
                                                              const uint8_t *__restrict__ arena,
                                                              const uint64_t *__restrict__ off,
                                                              const uint32_t *__restrict__ len,
                                                              uint32_t *__restrict__ ws_hs) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t aw[8], rw[8], sw[8], hs[CV_HS_WORDS];
    load_words8(aw, pk + (size_t)i * 32);
    load_words8(rw, sig + (size_t)i * 64);
    load_words8(sw, sig + (size_t)i * 64 + 32);
    cv_keyed_hs(aw, rw, sw, arena + off[i], len[i], hs);
    uint4 *d = reinterpret_cast<uint4 *>(ws_hs);
#pragma unroll
    for (int q = 0; q < CV_HS_WORDS / 4; q++)
        d[(size_t)q * cap + i] = make_uint4(hs[4 * q], hs[4 * q + 1], hs[4 * q + 2], hs[4 * q + 3]);
}

template <int WAVES>
__global__ __launch_bounds__(CV_BLOCK, WAVES) void cv_lattice_kernel(uint32_t n, uint32_t cap,
                                                                 const uint32_t *__restrict__ ws_hs,
                                                                 uint32_t *__restrict__ ws_dig) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t hs[CV_HS_WORDS];
    const uint4 *src = reinterpret_cast<const uint4 *>(ws_hs);
#pragma unroll
    for (int q = 0; q < CV_HS_WORDS / 4; q++) {
        const uint4 v = src[(size_t)q * cap + i];
        hs[4 * q] = v.x; hs[4 * q + 1] = v.y; hs[4 * q + 2] = v.z; hs[4 * q + 3] = v.w;
    }
    cv_hs_scalars<false, true>(hs, ws_dig + i, cap);
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
        if (i < n) cv_scalars_lane<false, true>(i, cap, pk, sig, arena, off, len, ws_dig);
    }
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
template __global__ void cv_hash_kernel<3>(uint32_t n, uint32_t cap, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *ws_hs);
template __global__ void cv_hash_kernel<4>(uint32_t n, uint32_t cap, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *ws_hs);
template __global__ void cv_lattice_kernel<2>(uint32_t n, uint32_t cap, const uint32_t *ws_hs, uint32_t *ws_dig);
template __global__ void cv_lattice_kernel<3>(uint32_t n, uint32_t cap, const uint32_t *ws_hs, uint32_t *ws_dig);
template __global__ void cv_lattice_kernel<4>(uint32_t n, uint32_t cap, const uint32_t *ws_hs, uint32_t *ws_dig);
