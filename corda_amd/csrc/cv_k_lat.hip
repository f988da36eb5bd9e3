// cv_k_lat.hip — latency forms for notary-sized batches: fused scalars + point pairs, quad and tri-chain Straus.
// Shared helpers and every kernel declaration: cv_kcommon.h; launchers: cv_kernels.hip.
#include "cv_kcommon.h"

// Small (latency) batches: the scalars and the point pairs of a signature are independent (both
// read only the inputs), so one launch runs them side by side on otherwise idle SIMDs — blocks
// [0, nbp) decode point pairs, blocks [nbp, grid) derive the scalars — and the batch pays
// max(scalars, points) instead of their sum.  One wave per 64-thread block, the whole register
// file for it (no spills in either role).
template <bool B16, bool LAT>
__global__ __launch_bounds__(64, 1) void cv_prep_lat_kernel(uint32_t n, uint32_t cap, uint32_t nbp, uint32_t pts4,
                                                            const uint8_t *__restrict__ pk,
                                                            const uint8_t *__restrict__ sig,
                                                            const uint8_t *__restrict__ arena,
                                                            const uint64_t *__restrict__ off,
                                                            const uint32_t *__restrict__ len,
                                                            uint32_t *__restrict__ ws_dig,
                                                            uint32_t *__restrict__ ws_tab,
                                                            uint32_t *__restrict__ ws_tabR,
                                                            uint8_t *__restrict__ ws_ok,
                                                            uint8_t *__restrict__ status,
                                                            uint64_t *__restrict__ bitmap) {
    if (blockIdx.x < nbp) {
        // pts4 (kernel argument, uniform): four lanes per signature (split tables), else lane pairs
        if (pts4)
            cv_points_quad_lane<LAT>(blockIdx.x * 64 + threadIdx.x, n, pk, sig, ws_tab, ws_tabR, ws_ok, status);
        else
            cv_points_pair_lane<LAT>(blockIdx.x * 64 + threadIdx.x, n, pk, sig, ws_tab, ws_tabR, ws_ok, status);
    } else {
        const uint32_t i = (blockIdx.x - nbp) * 64 + threadIdx.x;
        // the chunk's verdict words start at zero for the Straus kernel's atomicOr (it runs after this
        // launch on the same stream): one lane per word, instead of a separate memset launch
        if (bitmap && i < n && (i & 63u) == 0) bitmap[i >> 6] = 0;
        // tri (B16): radix-16 halves of w; quad: the radix-2^16 pairs of the throughput group
        if (i < n) cv_scalars_lane<B16, !B16>(i, cap, pk, sig, arena, off, len, ws_dig);
    }
}

// Half-size quad kernel (cv_hsquad.h): grid 4n lanes.  The chunk's bitmap words must be zero on
// entry (the launcher clears them): each wave ORs its 16 verdict bits into its word.  Quads past n
// replay signature n-1 (whole waves take part in the window-count reduction) and add no bits.
template <bool SEQ>
__global__ __launch_bounds__(CV_BLOCK) void cv_hs_straus_quad_kernel(uint32_t n, uint32_t cap,
                                                                     const uint32_t *__restrict__ ws_dig,
                                                                     const uint32_t *__restrict__ ws_tab,
                                                                     const uint32_t *__restrict__ ws_tabR,
                                                                     const uint8_t *__restrict__ ws_ok,
                                                                     uint64_t *__restrict__ bitmap,
                                                                     const uint32_t *__restrict__ bw16) {
    const uint32_t lane0 = blockIdx.x * CV_BLOCK + (threadIdx.x & ~63u);
    const uint32_t sig0 = lane0 >> 2;                        // first signature of this wave
    if (sig0 >= n) return;                                   // whole waves leave together
    const uint32_t i0 = (blockIdx.x * CV_BLOCK + threadIdx.x) >> 2;
    const int r = threadIdx.x & 3;
    const uint32_t i = i0 < n ? i0 : n - 1;
    int nw = (int)ws_dig[(size_t)64 * cap + i];
    nw = nw < 32 ? 32 : nw;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const int x = __shfl_xor(nw, o);
        nw = x > nw ? x : nw;
    }
    nw = __builtin_amdgcn_readfirstlane(nw);
    // w's radix-2^16 pairs against the CV_BW16 rows k*B (row 0) and k*2^128*B (row 2)
    const bool eq = cv_quad_hs_straus<true, SEQ>(bw16, bw16 + 2 * CV_BW16_ROW, ws_dig + i, cap,
                                            ws_tab + (size_t)i * CV_TAB_WORDS, ws_tabR + (size_t)i * CV_TAB_WORDS, nw, r);
    const bool acc = eq && ws_ok[i] && i0 < n;
    const uint32_t bits = cv_quad_ballot_bits(__ballot(acc));
    if ((threadIdx.x & 63u) == 0 && bits)
        atomicOr(reinterpret_cast<unsigned long long *>(bitmap + (sig0 >> 6)), (unsigned long long)bits << (sig0 & 63u));
}

// Tri-chain kernel (cv_hsquad.h): grid 16n lanes, 4 signatures per wave; digits from
// cv_hs_scalars<true>.  Bitmap words zero on entry, as for the quad kernel — or, with nib set (the
// zero-copy host path, cvk_verify_tri_zc), each wave stores its 4 verdict bits as one byte nib[wave]
// (a plain store into pinned host memory: no atomics over PCIe, no bitmap to clear).
template <bool SEQ>
__global__ __launch_bounds__(CV_BLOCK) void cv_hs_straus_tri_kernel(uint32_t n, uint32_t cap,
                                                                    const uint32_t *__restrict__ ws_dig,
                                                                    const uint32_t *__restrict__ ws_tab,
                                                                    const uint32_t *__restrict__ ws_tabR,
                                                                    const uint8_t *__restrict__ ws_ok,
                                                                    uint64_t *__restrict__ bitmap,
                                                                    uint8_t *__restrict__ nib) {
    constexpr int ROW = CV_BTAB_ENTRIES * CV_BTAB_STRIDE;
    const uint32_t lane0 = blockIdx.x * CV_BLOCK + (threadIdx.x & ~63u);
    const uint32_t sig0 = lane0 >> 4;                        // first signature of this wave
    if (sig0 >= n) return;                                   // whole waves leave together
    const uint32_t i0 = (blockIdx.x * CV_BLOCK + threadIdx.x) >> 4;
    const int r = threadIdx.x & 3, c = (threadIdx.x >> 2) & 3;
    const uint32_t i = i0 < n ? i0 : n - 1;
    int nw = (int)ws_dig[(size_t)64 * cap + i];
    nw = nw < 32 ? 32 : nw;                                  // the B halves need 32 windows
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const int x = __shfl_xor(nw, o);
        nw = x > nw ? x : nw;
    }
    nw = __builtin_amdgcn_readfirstlane(nw);
    // quad 0: v digits over k*R, 1: -u digits over k*(-A), 2: w_lo over k*B, 3: w_hi over k*2^128*B
    const uint32_t *tab = c == 0 ? ws_tabR + (size_t)i * CV_TAB_WORDS
                        : c == 1 ? ws_tab + (size_t)i * CV_TAB_WORDS
                                 : CV_BCOMB + (c == 2 ? 0 : 2 * ROW);
    const int field = c == 0 ? 5 : c == 1 ? 0 : c == 2 ? 10 : 15;
    const bool eq = cv_tri_hs_straus<SEQ>(ws_dig + i, cap, tab, c >= 2, field, nw, r);
    const bool acc = eq && ws_ok[i] && i0 < n && (threadIdx.x & 15u) == 0;
    uint64_t b = __ballot(acc) & 0x0001000100010001ull;      // lanes 0, 16, 32, 48
    b = (b | (b >> 15)) & 0x0000000300000003ull;
    b = (b | (b >> 30)) & 0xfull;
    if ((threadIdx.x & 63u) == 0) {
        if (nib)
            nib[sig0 >> 2] = (uint8_t)b;
        else if (b)
            atomicOr((unsigned long long *)(bitmap + sig0 / 64), (unsigned long long)b << (sig0 & 63));
    }
}

// Host -> device gather of q 16-byte pieces (the zero-copy notary path's records, cvk_verify_tri_zc):
// grid-stride, one 16-B load per lane per pass, so a batch's whole staging is in flight over PCIe at once.
__global__ __launch_bounds__(256) void cv_gather16_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst,
                                                          size_t q) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < q; i += stride) dst[i] = src[i];
}

// the sequential-carry field forms everywhere (round 3: tri Straus 160 -> 151 us at 4,096 against the ILP
// forms, quad 216 -> 203 us at 16,384; profiles/r03b_notary_probe_seq_pool.log)
template __global__ void cv_prep_lat_kernel<true, false>(uint32_t n, uint32_t cap, uint32_t nbp, uint32_t pts4, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *ws_dig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status, uint64_t *bitmap);
template __global__ void cv_prep_lat_kernel<false, false>(uint32_t n, uint32_t cap, uint32_t nbp, uint32_t pts4, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *ws_dig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status, uint64_t *bitmap);
template __global__ void cv_hs_straus_quad_kernel<true>(uint32_t n, uint32_t cap, const uint32_t *ws_dig, const uint32_t *ws_tab, const uint32_t *ws_tabR, const uint8_t *ws_ok, uint64_t *bitmap, const uint32_t *bw16);
template __global__ void cv_hs_straus_tri_kernel<true>(uint32_t n, uint32_t cap, const uint32_t *ws_dig, const uint32_t *ws_tab, const uint32_t *ws_tabR, const uint8_t *ws_ok, uint64_t *bitmap, uint8_t *nib);
