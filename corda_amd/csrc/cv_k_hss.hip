// cv_k_hss.hip — the half-size Straus kernel (the throughput hot path), in a translation unit of its own so
// it can take its own compiler scheduling flags (corda_amd/build.py SRC_FLAGS).  Shared helpers and every
// kernel declaration: cv_kcommon.h; launchers: cv_kernels.hip.
#include "cv_kcommon.h"

// hs_straus: E = [v]R + [u]A + [w]B per lane over the wave's largest window count, the identity
// test, and the verdict word by wave ballot (bit i of word i/64 = signature i).  Lanes past n
// replay signature n-1 so the whole wave takes part in the window-count reduction.  The basepoint
// digits are the W16 pairs (radix 2^16, one pair every fourth window) against the CV_BW16 rows in
// global memory (bw16: rows 0 and 2 of 4 x 32,769 entries, 16.8 MB, L2 / Infinity-Cache resident; the lanes' gathers
// are data-dependent, as they were from LDS).
template <int WAVES, bool SUB>
__global__ __launch_bounds__(CV_BLOCK, WAVES) void cv_hs_straus_kernel(uint32_t n, uint32_t cap,
                                                                       const uint32_t *__restrict__ ws_dig,
                                                                       const uint32_t *__restrict__ ws_tab,
                                                                       const uint32_t *__restrict__ ws_tabR,
                                                                       const uint8_t *__restrict__ ws_ok,
                                                                       uint64_t *__restrict__ bitmap,
                                                                       const uint32_t *__restrict__ bw16) {
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
    const bool eq = cv_hs_straus<CV_BTAB_STRIDE, true>(bw16, bw16 + 2 * CV_BW16_ROW, ws_dig + i, cap,
                                                       ws_tab + (size_t)i * CV_TAB_WORDS,
                                                       ws_tabR + (size_t)i * CV_TAB_WORDS, nw);
    const bool acc = eq && ws_ok[i] && i0 < n;
    const uint64_t bits = __ballot(acc);
    if ((threadIdx.x & 63u) == 0) bitmap[wave0 >> 6] = bits;
}

template __global__ void cv_hs_straus_kernel<CV_HSS_WAVES>(uint32_t, uint32_t, const uint32_t *, const uint32_t *,
                                                const uint32_t *, const uint8_t *, uint64_t *, const uint32_t *);
template __global__ void cv_hs_straus_kernel<CV_HSS_WAVES, true>(uint32_t, uint32_t, const uint32_t *, const uint32_t *,
                                                const uint32_t *, const uint8_t *, uint64_t *, const uint32_t *);
