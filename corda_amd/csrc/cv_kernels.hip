// cv_kernels.hip — gfx950 kernels of the batched signature-verification engine.
//
//   cv_verify_kernel  : eddsa-0.1.0-exact Ed25519 verify, one signature per lane, verdict bitmap by
//                       wave ballot (replaces EdDSAEngine.verify behind PublicKey.verifyWithECDSA,
//                       reference core/src/main/kotlin/net/corda/core/crypto/CryptoUtilities.kt:90-96)
//   cv_sign_kernel    : deterministic RFC 8032 keygen + sign (EdDSAEngine.sign / entropyToKeyPair,
//                       CryptoUtilities.kt:63-73,123-130) — synthetic-input generation only
//   cv_leaf_hash_kernel / cv_merkle_tree_kernel : WireTransaction.id = Merkle root of SHA-256 leaf
//                       hashes (reference core/.../transactions/MerkleTransaction.kt:26-38,66-99)
//
// Verify schedule (per lane, data-independent so all 64 lanes of a wave run in lockstep):
//   decode A (eddsa-0.1.0 rules) -> Abyte -> h = SHA-512(R||Abyte||M) mod L
//   s = (S - 2^256*[slide drops carry]) mod L                         (exact 0.1.0 scalar)
//   R' = [h](-A) + [s]B by joint fixed-window Straus: 64 windows of 4 bits,
//        -A digits in [-8,8] from a per-lane 9-entry table (private scratch),
//        B digits in [-128,128] every other window from a 129-entry table staged in LDS
//   accept iff encode(R') == R (canonical y + sign bit) — the same byte compare as the reference.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "cv_verify.h"
#include "cv_quad.h"
#include "cv_hsquad.h"

#define CV_BLOCK 256

__device__ __forceinline__ void stage_btab(uint32_t *lds) {
    for (int i = threadIdx.x; i < CV_BTAB_ENTRIES * CV_BTAB_STRIDE; i += blockDim.x) lds[i] = CV_BTAB[i];
    __syncthreads();
}

__device__ __forceinline__ void load_words8(uint32_t w[8], const uint8_t *p) {
    const uint4 a = reinterpret_cast<const uint4 *>(p)[0];
    const uint4 b = reinterpret_cast<const uint4 *>(p)[1];
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// ---------------------------------------------------------------- verify (three kernels)
// SoA records: pk[n][32], sig[n][64]; message i = arena[off[i] .. off[i]+len[i]).
// Workspace per signature: hs (16 words), tab (320 words, per-lane contiguous so each table
// lookup is ten 16-B loads of one lane's own entry), R record (32 words), ok byte.

__device__ __forceinline__ void store_words(uint32_t *dst, const uint32_t *src, int nwords4) {
    uint4 *d = reinterpret_cast<uint4 *>(dst);
#pragma unroll
    for (int q = 0; q < nwords4; q++) d[q] = make_uint4(src[4 * q], src[4 * q + 1], src[4 * q + 2], src[4 * q + 3]);
}

template <bool LAT>
__global__ __launch_bounds__(CV_BLOCK, 2) void cv_prep_kernel(
    uint32_t n, const uint8_t *__restrict__ pk, const uint8_t *__restrict__ sig, const uint8_t *__restrict__ arena,
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ len, uint32_t *__restrict__ ws_hs,
    uint32_t *__restrict__ ws_tab, uint8_t *__restrict__ ws_ok, uint8_t *__restrict__ status) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t aw[8], rw[8], sw[8];
    load_words8(aw, pk + (size_t)i * 32);
    load_words8(rw, sig + (size_t)i * 64);
    load_words8(sw, sig + (size_t)i * 64 + 32);
    uint32_t hs[CV_HS_WORDS];
    const bool ok = cv_verify_prep<LAT>(aw, rw, sw, arena + off[i], len[i], hs, ws_tab + (size_t)i * CV_TAB_WORDS);
    store_words(ws_hs + (size_t)i * CV_HS_WORDS, hs, CV_HS_WORDS / 4);
    ws_ok[i] = ok ? 1 : 0;
    if (status) status[i] = ok ? 0 : 1;
}

template <int WAVES>
__global__ __launch_bounds__(CV_BLOCK, WAVES) void cv_straus_kernel(uint32_t n, const uint32_t *__restrict__ ws_hs,
                                                                    const uint32_t *__restrict__ ws_tab,
                                                                    uint32_t *__restrict__ ws_R) {
    __shared__ __attribute__((aligned(16))) uint32_t btab[CV_BTAB_ENTRIES * CV_BTAB_STRIDE];
    stage_btab(btab);
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i >= n) return;
    ge_p2 R;
    cv_verify_straus(btab, ws_hs + (size_t)i * CV_HS_WORDS, ws_tab + (size_t)i * CV_TAB_WORDS, R);
    uint32_t rec[CV_R_WORDS];
    fe_store(rec, R.X);
    fe_store(rec + 10, R.Y);
    fe_store(rec + 20, R.Z);
    rec[30] = rec[31] = 0;
    store_words(ws_R + (size_t)i * CV_R_WORDS, rec, CV_R_WORDS / 4);
}
template __global__ void cv_straus_kernel<2>(uint32_t, const uint32_t *, const uint32_t *, uint32_t *);
template __global__ void cv_straus_kernel<3>(uint32_t, const uint32_t *, const uint32_t *, uint32_t *);
template __global__ void cv_straus_kernel<4>(uint32_t, const uint32_t *, const uint32_t *, uint32_t *);

// occupancy variant of the Straus kernel (waves per SIMD the register budget is built for);
// tuned on the box with tools/ab_straus.py, default = the measured best
static int g_straus_waves = 3;
extern "C" void cvk_set_straus_waves(int w) { g_straus_waves = (w == 2 || w == 3 || w == 4) ? w : 3; }

// lane j: signatures [8j, 8j+8) -> bitmap byte j (bytes past n are written as zero)
template <bool LAT>
__global__ __launch_bounds__(CV_BLOCK) void cv_finish_kernel(uint32_t n, uint32_t nbytes,
                                                             const uint8_t *__restrict__ sig,
                                                             const uint32_t *__restrict__ ws_R,
                                                             const uint8_t *__restrict__ ws_ok,
                                                             uint8_t *__restrict__ bitmap_bytes) {
    const uint32_t j = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (j >= nbytes) return;
    const uint32_t b = j * CV_FIN_CHUNK;
    uint32_t bits = 0;
    if (b < n) {
        const int cnt = (int)(n - b < CV_FIN_CHUNK ? n - b : CV_FIN_CHUNK);
        bits = cv_verify_finish<LAT>(ws_R + (size_t)b * CV_R_WORDS, reinterpret_cast<const uint32_t *>(sig + (size_t)b * 64),
                                ws_ok + b, cnt);
    }
    bitmap_bytes[j] = (uint8_t)bits;
}

// ---------------------------------------------------------------- half-size verify (cv_verify.h)
// hsprep: decode R canonically (r_ok folded into the key-ok byte), k*R table, lattice-reduced
// (u, v, w) as packed per-window digit words, window-major: ws_dig[win * cap + i].
template <bool LAT>
__global__ __launch_bounds__(CV_BLOCK, 2) void cv_hsprep_kernel(uint32_t n, uint32_t cap, const uint8_t *__restrict__ sig,
                                                                const uint32_t *__restrict__ ws_hs,
                                                                uint32_t *__restrict__ ws_dig,
                                                                uint32_t *__restrict__ ws_tabR,
                                                                uint8_t *__restrict__ ws_ok, int reduce) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t rw[8], hs[CV_HS_WORDS];
    load_words8(rw, sig + (size_t)i * 64);
    const uint4 *hp = reinterpret_cast<const uint4 *>(ws_hs + (size_t)i * CV_HS_WORDS);
#pragma unroll
    for (int q = 0; q < CV_HS_WORDS / 4; q++) {
        const uint4 x = hp[q];
        hs[4 * q] = x.x; hs[4 * q + 1] = x.y; hs[4 * q + 2] = x.z; hs[4 * q + 3] = x.w;
    }
    const bool r_ok = cv_hs_prep<LAT>(rw, hs, ws_dig + i, cap, ws_tabR + (size_t)i * CV_TAB_WORDS, reduce != 0);
    if (!r_ok) ws_ok[i] = 0;
}

// scalars of the half-size group, one lane per signature: h = SHA-512(R || Abyte || M) mod L, the
// effective S, the lattice (u, v, w) and the packed window digits -> ws_dig (cv_hs_scalars).  Its own
// kernel, at the occupancy its registers allow (3 waves per SIMD), because inside the 256-VGPR point
// kernel (2 waves per SIMD) the hash's serial 64-bit chains were 32 % of the prep's cycles
// (tools/prep_probe.py).  Any block size (small latency batches launch 64-thread blocks so the few
// waves spread over CUs).
template <bool B16 = false>
__device__ __forceinline__ void cv_scalars_lane(uint32_t i, uint32_t cap, const uint8_t *pk, const uint8_t *sig,
                                                const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                                                uint32_t *ws_dig) {
    uint32_t aw[8], rw[8], sw[8];
    load_words8(aw, pk + (size_t)i * 32);
    load_words8(rw, sig + (size_t)i * 64);
    load_words8(sw, sig + (size_t)i * 64 + 32);
    uint32_t hs[CV_HS_WORDS];
    cv_keyed_hs(aw, rw, sw, arena + off[i], len[i], hs);
    cv_hs_scalars<B16>(hs, ws_dig + i, cap);
}
__global__ __launch_bounds__(CV_BLOCK, 3) void cv_scalars_kernel(uint32_t n, uint32_t cap, const uint8_t *__restrict__ pk,
                                                                 const uint8_t *__restrict__ sig,
                                                                 const uint8_t *__restrict__ arena,
                                                                 const uint64_t *__restrict__ off,
                                                                 const uint32_t *__restrict__ len,
                                                                 uint32_t *__restrict__ ws_dig) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i < n) cv_scalars_lane(i, cap, pk, sig, arena, off, len, ws_dig);
}
// Small (latency) batches: 64-thread blocks (one wave each, spread over CUs) and the whole register
// file for the lone wave — no spills.  A spilling version took 62 us at 256 signatures but 208 us at
// 4,096 (rocprofv3, profiles/r02_notary_kernels.txt): waves that need scratch queue for scratch slots.
__global__ __launch_bounds__(64, 1) void cv_scalars_lat_kernel(uint32_t n, uint32_t cap, const uint8_t *__restrict__ pk,
                                                               const uint8_t *__restrict__ sig,
                                                               const uint8_t *__restrict__ arena,
                                                               const uint64_t *__restrict__ off,
                                                               const uint32_t *__restrict__ len,
                                                               uint32_t *__restrict__ ws_dig) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i < n) cv_scalars_lane(i, cap, pk, sig, arena, off, len, ws_dig);
}

// points of the half-size group (throughput form): A and R decoded as one interleaved pair per lane,
// both odd-multiple tables (cv_hs_points); ws_ok = key_ok AND r_ok, status = key status.
template <bool SUB = false>
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
template <int WAVES, bool SUB = false>
__global__ __launch_bounds__(CV_BLOCK, WAVES) void cv_points_one_kernel(uint32_t n, const uint8_t *__restrict__ pk,
                                                                        const uint8_t *__restrict__ sig,
                                                                        uint32_t *__restrict__ ws_tab,
                                                                        uint32_t *__restrict__ ws_tabR,
                                                                        uint8_t *__restrict__ ws_ok,
                                                                        uint8_t *__restrict__ status) {
    const uint32_t g = blockIdx.x * CV_BLOCK + threadIdx.x;
    const uint32_t i = g >> 1;
    if (i >= n) return;                       // both lanes of a pair leave together
    const bool is_r = (g & 1u) != 0;
    uint32_t w[8];
    load_words8(w, is_r ? sig + (size_t)i * 64 : pk + (size_t)i * 32);
    const bool ok = cv_hs_point_one<false>(w, is_r, (is_r ? ws_tabR : ws_tab) + (size_t)i * CV_TAB_WORDS);
    const bool r_ok = __shfl_xor((int)ok, 1) != 0;
    if (!is_r) {
        ws_ok[i] = (ok && r_ok) ? 1 : 0;
        if (status) status[i] = ok ? 0 : 1;
    }
}
// 0 = one lane decodes both points (cv_points_kernel: 256 VGPRs, 23 spilled, 2 waves/SIMD), 2 / 3 =
// lane pairs at that many waves per SIMD.  Default 3: points 2.46 -> 2.37 ms per 1M, C2 -0.8 % per step
// (same-box A/B, 3 alternating rounds, profiles/r02_ab_points_modes.log)
static int g_points_mode = 3;
extern "C" void cvk_set_points_mode(int v) { g_points_mode = (v == 2 || v == 3) ? v : 0; }
template <bool SUB>
static void launch_points(uint32_t m, const uint8_t *pk, const uint8_t *sig, uint32_t *tabA, uint32_t *tabR, uint8_t *ok,
                          uint8_t *status, hipStream_t st) {
    if (g_points_mode == 3)
        hipLaunchKernelGGL((cv_points_one_kernel<3, SUB>), dim3((2 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, st,
                           m, pk, sig, tabA, tabR, ok, status);
    else if (g_points_mode == 2)
        hipLaunchKernelGGL((cv_points_one_kernel<2, SUB>), dim3((2 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, st,
                           m, pk, sig, tabA, tabR, ok, status);
    else
        hipLaunchKernelGGL(cv_points_kernel<SUB>, dim3((m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, st, m, pk, sig,
                           tabA, tabR, ok, status);
}

// points of the half-size group (latency form, small batches): a lane PAIR per signature, the even
// lane decoding the key A into k*(-A), the odd lane R into k*R, side by side (the same instructions
// on both lanes: cv_hs_point_one) with the latency (ILP) field forms — half the serial chain of the
// throughput form, whose single lane runs both decodes.  The even lane writes ok = key_ok AND r_ok.
__device__ __forceinline__ void cv_points_pair_lane(uint32_t g, uint32_t n, const uint8_t *pk, const uint8_t *sig,
                                                    uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok,
                                                    uint8_t *status) {
    const uint32_t i = g >> 1;
    if (i >= n) return;                       // both lanes of a pair leave together
    const bool is_r = (g & 1u) != 0;
    uint32_t w[8];
    load_words8(w, is_r ? sig + (size_t)i * 64 : pk + (size_t)i * 32);
    const bool ok = cv_hs_point_one<true>(w, is_r, (is_r ? ws_tabR : ws_tab) + (size_t)i * CV_TAB_WORDS);
    const bool r_ok = __shfl_xor((int)ok, 1) != 0;
    if (!is_r) {
        ws_ok[i] = (ok && r_ok) ? 1 : 0;
        if (status) status[i] = ok ? 0 : 1;
    }
}
__global__ __launch_bounds__(64) void cv_points_pair_kernel(uint32_t n, const uint8_t *__restrict__ pk,
                                                            const uint8_t *__restrict__ sig,
                                                            uint32_t *__restrict__ ws_tab,
                                                            uint32_t *__restrict__ ws_tabR,
                                                            uint8_t *__restrict__ ws_ok,
                                                            uint8_t *__restrict__ status) {
    cv_points_pair_lane(blockIdx.x * 64 + threadIdx.x, n, pk, sig, ws_tab, ws_tabR, ws_ok, status);
}

// Small (latency) batches: the scalars and the point pairs of a signature are independent (both
// read only the inputs), so one launch runs them side by side on otherwise idle SIMDs — blocks
// [0, nbp) decode point pairs, blocks [nbp, grid) derive the scalars — and the batch pays
// max(scalars, points) instead of their sum.  One wave per 64-thread block, the whole register
// file for it (no spills in either role).
template <bool B16>
__global__ __launch_bounds__(64, 1) void cv_prep_lat_kernel(uint32_t n, uint32_t cap, uint32_t nbp,
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
        cv_points_pair_lane(blockIdx.x * 64 + threadIdx.x, n, pk, sig, ws_tab, ws_tabR, ws_ok, status);
    } else {
        const uint32_t i = (blockIdx.x - nbp) * 64 + threadIdx.x;
        if (i < n) cv_scalars_lane<B16>(i, cap, pk, sig, arena, off, len, ws_dig);
    }
}

// hs_straus: E = [v]R + [u]A + [w]B per lane over the wave's largest window count, the identity
// test, and the verdict word by wave ballot (bit i of word i/64 = signature i).  Lanes past n
// replay signature n-1 so the whole wave takes part in the window-count reduction.
template <int WAVES, bool SUB = false>
__global__ __launch_bounds__(CV_BLOCK, WAVES) void cv_hs_straus_kernel(uint32_t n, uint32_t cap,
                                                                       const uint32_t *__restrict__ ws_dig,
                                                                       const uint32_t *__restrict__ ws_tab,
                                                                       const uint32_t *__restrict__ ws_tabR,
                                                                       const uint8_t *__restrict__ ws_ok,
                                                                       uint64_t *__restrict__ bitmap) {
    __shared__ __attribute__((aligned(16))) uint32_t btab[2 * CV_BTAB_ENTRIES * CV_BTAB_STRIDE];
    constexpr int ROW = CV_BTAB_ENTRIES * CV_BTAB_STRIDE;
    for (int k = threadIdx.x; k < ROW; k += blockDim.x) {
        btab[k] = CV_BCOMB[k];                 // k * B
        btab[ROW + k] = CV_BCOMB[2 * ROW + k]; // k * 2^128 * B
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
    const bool eq = cv_hs_straus(btab, btab + ROW, ws_dig + i, cap, ws_tab + (size_t)i * CV_TAB_WORDS,
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

// 1 = half-size verify for throughput batches (default), 0 = the full-width prep/straus/finish group
static int g_verify_mode = 1;
static int g_hs_waves = 3;
extern "C" void cvk_set_verify_mode(int m) { g_verify_mode = m ? 1 : 0; }
extern "C" int cvk_get_verify_mode(void) { return g_verify_mode; }
extern "C" void cvk_set_hs_waves(int w) { g_hs_waves = (w == 2) ? 2 : 3; }
// latency (ILP) field forms in the prep / hsprep kernels of throughput batches (2 waves per SIMD)
static int g_prep_lat = 0, g_hsprep_lat = 0;
// 0 = skip the lattice reduction ((u, v) = (h, 1), 64 windows: still exact) — A/B timing only
static int g_hs_reduce = 1;
// 1 = one fused prep kernel (interleaved A/R decodes), 0 = prep + hsprep
static int g_hs_fused = 1;
// 1 = small batches (<= g_quad_max) run the half-size quad kernel, 0 = the full-width quad group
static int g_hs_quad = 1;
extern "C" void cvk_set_hs_quad(int v) { g_hs_quad = v ? 1 : 0; }
extern "C" void cvk_set_hs_fused(int v) { g_hs_fused = v ? 1 : 0; }
extern "C" void cvk_set_hs_reduce(int v) { g_hs_reduce = v ? 1 : 0; }
extern "C" void cvk_set_prep_lat(int v) { g_prep_lat = v ? 1 : 0; }
extern "C" void cvk_set_hsprep_lat(int v) { g_hsprep_lat = v ? 1 : 0; }

// ---------------------------------------------------------------- quad (latency) Straus kernels
// Four lanes per signature (cv_quad.h) for batches too small to fill the chip.  Grid: 4n lanes.
__global__ __launch_bounds__(CV_BLOCK) void cv_straus_quad_kernel(uint32_t n, const uint32_t *__restrict__ ws_hs,
                                                                  const uint32_t *__restrict__ ws_tab,
                                                                  uint32_t *__restrict__ ws_R) {
    __shared__ __attribute__((aligned(16))) uint32_t btab[CV_BTAB_ENTRIES * CV_BTAB_STRIDE];
    stage_btab(btab);
    const uint32_t i = (blockIdx.x * CV_BLOCK + threadIdx.x) >> 2;
    const int r = threadIdx.x & 3;
    if (i >= n) return;                       // whole quads leave together
    fe P;
    cv_quad_straus(btab, ws_hs + (size_t)i * CV_HS_WORDS, ws_tab + (size_t)i * CV_TAB_WORDS, r, P);
    if (r < 3) fe_store(ws_R + (size_t)i * CV_R_WORDS + 10 * r, P);
}

__global__ __launch_bounds__(CV_BLOCK) void cv_comb_quad_kernel(uint32_t n, const uint32_t *__restrict__ ws_hs,
                                                                const uint32_t *__restrict__ key_index,
                                                                const uint32_t *__restrict__ slot_of_key,
                                                                const uint32_t *__restrict__ ktab_pool,
                                                                uint32_t *__restrict__ ws_R) {
    const uint32_t i = (blockIdx.x * CV_BLOCK + threadIdx.x) >> 2;
    const int r = threadIdx.x & 3;
    if (i >= n) return;
    const uint32_t slot = slot_of_key[key_index[i]];
    fe P;
    cv_quad_comb(CV_BCOMB, ws_hs + (size_t)i * CV_HS_WORDS, ktab_pool + (size_t)slot * CV_KTAB_WORDS, r, P);
    if (r < 3) fe_store(ws_R + (size_t)i * CV_R_WORDS + 10 * r, P);
}

// Half-size quad kernel (cv_hsquad.h): grid 4n lanes.  The chunk's bitmap words must be zero on
// entry (the launcher clears them): each wave ORs its 16 verdict bits into its word.  Quads past n
// replay signature n-1 (whole waves take part in the window-count reduction) and add no bits.
__global__ __launch_bounds__(CV_BLOCK) void cv_hs_straus_quad_kernel(uint32_t n, uint32_t cap,
                                                                     const uint32_t *__restrict__ ws_dig,
                                                                     const uint32_t *__restrict__ ws_tab,
                                                                     const uint32_t *__restrict__ ws_tabR,
                                                                     const uint8_t *__restrict__ ws_ok,
                                                                     uint64_t *__restrict__ bitmap) {
    constexpr int ROW = CV_BTAB_ENTRIES * CV_BTAB_STRIDE;
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
    const bool eq = cv_quad_hs_straus(CV_BCOMB, CV_BCOMB + 2 * ROW, ws_dig + i, cap, ws_tab + (size_t)i * CV_TAB_WORDS,
                                      ws_tabR + (size_t)i * CV_TAB_WORDS, nw, r);
    const bool acc = eq && ws_ok[i] && i0 < n;
    const uint32_t bits = cv_quad_ballot_bits(__ballot(acc));
    if ((threadIdx.x & 63u) == 0 && bits)
        atomicOr(reinterpret_cast<unsigned long long *>(bitmap + (sig0 >> 6)), (unsigned long long)bits << (sig0 & 63u));
}

// Tri-chain kernel (cv_hsquad.h): grid 16n lanes, 4 signatures per wave; digits from
// cv_hs_scalars<true>.  Bitmap words zero on entry, as for the quad kernel.
__global__ __launch_bounds__(CV_BLOCK) void cv_hs_straus_tri_kernel(uint32_t n, uint32_t cap,
                                                                    const uint32_t *__restrict__ ws_dig,
                                                                    const uint32_t *__restrict__ ws_tab,
                                                                    const uint32_t *__restrict__ ws_tabR,
                                                                    const uint8_t *__restrict__ ws_ok,
                                                                    uint64_t *__restrict__ bitmap) {
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
    const bool eq = cv_tri_hs_straus(ws_dig + i, cap, tab, c >= 2, field, nw, r);
    const bool acc = eq && ws_ok[i] && i0 < n && (threadIdx.x & 15u) == 0;
    uint64_t b = __ballot(acc) & 0x0001000100010001ull;      // lanes 0, 16, 32, 48
    b = (b | (b >> 15)) & 0x0000000300000003ull;
    b = (b | (b >> 30)) & 0xfull;
    if ((threadIdx.x & 63u) == 0 && b) atomicOr((unsigned long long *)(bitmap + sig0 / 64), (unsigned long long)b << (sig0 & 63));
}

// Batches of at most this many signatures run the tri-chain kernel (cvk_set_tri_max; 0 = never)
static uint32_t g_tri_max = 4096;
extern "C" void cvk_set_tri_max(int m) { g_tri_max = (uint32_t)(m < 0 ? 0 : m); }
extern "C" uint32_t cvk_get_tri_max(void) { return g_tri_max; }

// 1 = small batches run scalars and point pairs in one launch (cv_prep_lat_kernel), 0 = two launches
static int g_prep_lat_fused = 1;
extern "C" void cvk_set_prep_lat_fused(int v) { g_prep_lat_fused = v ? 1 : 0; }

// Batches of at most this many signatures run the quad kernels (set by cvk_set_quad_max; 0 = never)
static uint32_t g_quad_max = 32768;
extern "C" void cvk_set_quad_max(uint32_t m) { g_quad_max = m; }

// ---------------------------------------------------------------- two-stream sub-chunk overlap
// A chunk of the half-size group is cut into a head and a tail sub-chunk; the tail runs on a helper
// stream so its waves fill the partial last rounds (drain) of the head's kernels.  mode 0 = off,
// 1 = both sub-chunks start together, 2 = the tail's prep waits for the head's prep, 3 = auto: mode 1
// when the chunk's last round of hs_straus waves is at most 12 % full (a near-empty drain round: 1M
// signatures = 5.09 rounds of 3072 resident waves on 256 CUs; measured 11.0-11.2 -> 10.7 ms), else off.
static int g_split_mode = 3, g_split_pct = 10;
extern "C" void cvk_set_split_mode(int m) { g_split_mode = (m >= 0 && m <= 3) ? m : 0; }
extern "C" void cvk_set_split_pct(int p) { g_split_pct = (p >= 5 && p <= 50) ? p : 10; }
struct SplitAux {
    hipStream_t s2 = nullptr;
    hipEvent_t start = nullptr, prep1 = nullptr, done2 = nullptr;
    int cus = 0;
    bool ready = false;
    std::mutex mu;   // creation, and record/wait of the shared events, happen under it
};
static SplitAux g_split_aux[16];
static hipError_t split_aux(SplitAux **out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 16) return hipErrorInvalidDevice;
    SplitAux &a = g_split_aux[dev];
    // lazily created once per device; the lock makes two first callers (different threads) safe
    std::lock_guard<std::mutex> lk(a.mu);
    if (!a.ready) {
        if (!a.s2 && (e = hipStreamCreateWithFlags(&a.s2, hipStreamNonBlocking)) != hipSuccess) return e;
        if (!a.start && (e = hipEventCreateWithFlags(&a.start, hipEventDisableTiming)) != hipSuccess) return e;
        if (!a.prep1 && (e = hipEventCreateWithFlags(&a.prep1, hipEventDisableTiming)) != hipSuccess) return e;
        if (!a.done2 && (e = hipEventCreateWithFlags(&a.done2, hipEventDisableTiming)) != hipSuccess) return e;
        if ((e = hipDeviceGetAttribute(&a.cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
        a.ready = true;
    }
    *out = &a;
    return hipSuccess;
}

// ---------------------------------------------------------------- keyed verify (per-key comb, f2)
// key precompute: one lane per key (decode + 4 comb row tables of 8 cached multiples) into its slot
__global__ __launch_bounds__(CV_BLOCK) void cv_keyprep_kernel(uint32_t nk, const uint8_t *__restrict__ keys,
                                                              const uint32_t *__restrict__ slots,
                                                              uint32_t *__restrict__ scratch,
                                                              uint32_t *__restrict__ ktab_pool,
                                                              uint8_t *__restrict__ kok_pool) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i >= nk) return;
    uint32_t aw[8];
    load_words8(aw, keys + (size_t)i * 32);
    const uint32_t slot = slots[i];
    const bool ok = cv_key_prep(aw, scratch + (size_t)i * CV_KTAB_WORDS, ktab_pool + (size_t)slot * CV_KTAB_WORDS);
    kok_pool[slot] = ok ? 1 : 0;
}

// keyed phase 1: hash + scalar per signature; key validity from the key's slot
__global__ __launch_bounds__(CV_BLOCK) void cv_keyed_prep_kernel(
    uint32_t n, const uint8_t *__restrict__ keys, const uint32_t *__restrict__ key_index,
    const uint32_t *__restrict__ slot_of_key, const uint8_t *__restrict__ kok_pool, const uint8_t *__restrict__ sig,
    const uint8_t *__restrict__ arena, const uint64_t *__restrict__ off, const uint32_t *__restrict__ len,
    uint32_t *__restrict__ ws_hs, uint8_t *__restrict__ ws_ok, uint8_t *__restrict__ status) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t ki = key_index[i];
    uint32_t aw[8], rw[8], sw[8];
    load_words8(aw, keys + (size_t)ki * 32);
    load_words8(rw, sig + (size_t)i * 64);
    load_words8(sw, sig + (size_t)i * 64 + 32);
    uint32_t hs[CV_HS_WORDS];
    cv_keyed_hs(aw, rw, sw, arena + off[i], len[i], hs);
    store_words(ws_hs + (size_t)i * CV_HS_WORDS, hs, CV_HS_WORDS / 4);
    const uint8_t ok = kok_pool[slot_of_key[ki]];
    ws_ok[i] = ok;
    if (status) status[i] = ok ? 0 : 1;
}

// keyed phase 2: the 4-row comb.  The basepoint comb tables (66 KB) are read from global memory
// (L2-resident: every lane of the chip reads the same table) so LDS does not cap the occupancy.
#define CV_BCOMB_WORDS (4 * CV_BTAB_ENTRIES * CV_BTAB_STRIDE)
template <int WAVES>
__global__ __launch_bounds__(CV_BLOCK, WAVES) void cv_comb_kernel(uint32_t n, const uint32_t *__restrict__ ws_hs,
                                                                  const uint32_t *__restrict__ key_index,
                                                                  const uint32_t *__restrict__ slot_of_key,
                                                                  const uint32_t *__restrict__ ktab_pool,
                                                                  uint32_t *__restrict__ ws_R) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t slot = slot_of_key[key_index[i]];
    ge_p2 R;
    cv_comb_straus(CV_BCOMB, ws_hs + (size_t)i * CV_HS_WORDS, ktab_pool + (size_t)slot * CV_KTAB_WORDS, R);
    uint32_t rec[CV_R_WORDS];
    fe_store(rec, R.X);
    fe_store(rec + 10, R.Y);
    fe_store(rec + 20, R.Z);
    rec[30] = rec[31] = 0;
    store_words(ws_R + (size_t)i * CV_R_WORDS, rec, CV_R_WORDS / 4);
}
template __global__ void cv_comb_kernel<2>(uint32_t, const uint32_t *, const uint32_t *, const uint32_t *,
                                           const uint32_t *, uint32_t *);
template __global__ void cv_comb_kernel<3>(uint32_t, const uint32_t *, const uint32_t *, const uint32_t *,
                                           const uint32_t *, uint32_t *);
static int g_comb_waves = 3;
extern "C" void cvk_set_comb_waves(int w) { g_comb_waves = (w == 2) ? 2 : 3; }

// ---------------------------------------------------------------- sign (synthetic inputs)
__global__ __launch_bounds__(CV_BLOCK, 2) void cv_sign_kernel(
    uint32_t n, const uint8_t *__restrict__ seed, const uint8_t *__restrict__ arena,
    const uint64_t *__restrict__ off, const uint32_t *__restrict__ len, uint8_t *__restrict__ pk_out,
    uint8_t *__restrict__ sig_out) {
    __shared__ __attribute__((aligned(16))) uint32_t btab[CV_BTAB_ENTRIES * CV_BTAB_STRIDE];
    stage_btab(btab);
    const uint32_t gid = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (gid >= n) return;
    uint32_t sd[8], pkw[8], sgw[16];
    load_words8(sd, seed + (size_t)gid * 32);
    cv_sign_one(btab, sd, arena + off[gid], len[gid], pkw, sgw);
    uint4 *po = reinterpret_cast<uint4 *>(pk_out + (size_t)gid * 32);
    uint4 *so = reinterpret_cast<uint4 *>(sig_out + (size_t)gid * 64);
    po[0] = make_uint4(pkw[0], pkw[1], pkw[2], pkw[3]);
    po[1] = make_uint4(pkw[4], pkw[5], pkw[6], pkw[7]);
#pragma unroll
    for (int q = 0; q < 4; q++) so[q] = make_uint4(sgw[4 * q], sgw[4 * q + 1], sgw[4 * q + 2], sgw[4 * q + 3]);
}

// ---------------------------------------------------------------- Merkle tx ids
__global__ __launch_bounds__(CV_BLOCK) void cv_leaf_hash_kernel(uint32_t nleaves, const uint8_t *__restrict__ arena,
                                                                const uint64_t *__restrict__ off,
                                                                const uint32_t *__restrict__ len,
                                                                uint32_t *__restrict__ leaf_digest) {
    const uint32_t gid = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (gid >= nleaves) return;
    uint32_t d[8];
    sha256_bytes(d, arena + off[gid], len[gid]);
    uint4 *o = reinterpret_cast<uint4 *>(leaf_digest + (size_t)gid * 8);
    o[0] = make_uint4(d[0], d[1], d[2], d[3]);
    o[1] = make_uint4(d[4], d[5], d[6], d[7]);
}

// one lane per transaction, in place over its leaf digests; ids are written as digest bytes
__global__ __launch_bounds__(CV_BLOCK) void cv_merkle_tree_kernel(uint32_t ntx, const uint32_t *__restrict__ tx_begin,
                                                                  uint32_t *__restrict__ leaf_digest,
                                                                  uint8_t *__restrict__ ids,
                                                                  uint8_t *__restrict__ status) {
    const uint32_t gid = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (gid >= ntx) return;
    const uint32_t b = tx_begin[gid], e = tx_begin[gid + 1];
    uint32_t root[8];
    const bool ok = cv_merkle_root_inplace(leaf_digest + (size_t)b * 8, e - b, root);
    uint4 *o = reinterpret_cast<uint4 *>(ids + (size_t)gid * 32);
    o[0] = make_uint4(cv_bswap32(root[0]), cv_bswap32(root[1]), cv_bswap32(root[2]), cv_bswap32(root[3]));
    o[1] = make_uint4(cv_bswap32(root[4]), cv_bswap32(root[5]), cv_bswap32(root[6]), cv_bswap32(root[7]));
    if (status) status[gid] = ok ? 0 : 1;
}

// ---------------------------------------------------------------- partial Merkle trees (f3)
// one lane per tree (FilteredTransaction.verify / PartialMerkleTree.verify, cv_verify.h)
__global__ __launch_bounds__(CV_BLOCK) void cv_pmt_verify_kernel(uint32_t ntrees, const uint8_t *__restrict__ kind,
                                                                 const uint32_t *__restrict__ left,
                                                                 const uint32_t *__restrict__ right,
                                                                 const uint8_t *__restrict__ leaf_hash,
                                                                 const uint32_t *__restrict__ tree_begin,
                                                                 const uint8_t *__restrict__ root,
                                                                 const uint8_t *__restrict__ check,
                                                                 const uint32_t *__restrict__ check_begin,
                                                                 uint32_t *__restrict__ dig, uint8_t *__restrict__ flag,
                                                                 uint8_t *__restrict__ verdict, uint8_t *__restrict__ status) {
    const uint32_t t = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (t >= ntrees) return;
    bool v = false;
    const int st = cv_pmt_verify(tree_begin[t], tree_begin[t + 1], kind, left, right, leaf_hash, root + 32 * (size_t)t,
                                 check, check_begin[t], check_begin[t + 1], dig, flag, v);
    verdict[t] = v ? 1 : 0;
    status[t] = (uint8_t)st;
}

// ---------------------------------------------------------------- launchers (internal ABI)
extern "C" {

// Verify n signatures with the workspace ws (capacity ws_cap signatures, a multiple of 512); the
// batch is processed in chunks of ws_cap.  bitmap gets ceil(n/64) words.  ws_tab holds 2 * ws_cap
// tables (k*(-A), then k*R for the half-size group); ws_dig CV_HS_DIGWORDS * ws_cap words.  ev phases: prep | straus | finish, or in the
// half-size group prep | hsprep | hs_straus.
hipError_t cvk_verify(uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off,
                      const uint32_t *len, uint64_t *bitmap, uint8_t *status, uint32_t *ws_hs, uint32_t *ws_tab,
                      uint32_t *ws_R, uint8_t *ws_ok, uint32_t *ws_dig, uint32_t ws_cap, hipStream_t stream,
                      hipEvent_t *ev) {
    if (n == 0) return hipSuccess;
    if (ws_cap == 0 || ws_cap % 512) return hipErrorInvalidValue;
    for (uint32_t c0 = 0; c0 < n; c0 += ws_cap) {
        const uint32_t m = (n - c0 < ws_cap) ? n - c0 : ws_cap;
        const uint32_t blocks = (m + CV_BLOCK - 1) / CV_BLOCK;
        // ev (optional, single-chunk batches): phase boundaries for live per-kernel timing
        if (ev && c0 == 0) (void)hipEventRecord(ev[0], stream);
        const bool lat = n <= g_quad_max;   // small batch: latency forms of the single chains
        if (lat && g_verify_mode == 1 && g_hs_quad) {
            // half-size quad group: phases = scalars + point pairs | bitmap clear | hs_straus_quad
            uint32_t *ws_tabR = ws_tab + (size_t)ws_cap * CV_TAB_WORDS;
            // 64-thread blocks: the few waves of a small batch spread over CUs (one per SIMD)
            const bool tri = m <= g_tri_max;
            if (g_prep_lat_fused || tri) {
                const uint32_t nbp = (2 * m + 63) / 64, nbs = (m + 63) / 64;
                if (tri)
                    hipLaunchKernelGGL(cv_prep_lat_kernel<true>, dim3(nbp + nbs), dim3(64), 0, stream, m, ws_cap, nbp,
                                       pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0,
                                       ws_dig, ws_tab, ws_tabR, ws_ok, status ? status + c0 : nullptr);
                else
                    hipLaunchKernelGGL(cv_prep_lat_kernel<false>, dim3(nbp + nbs), dim3(64), 0, stream, m, ws_cap, nbp,
                                       pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0,
                                       ws_dig, ws_tab, ws_tabR, ws_ok, status ? status + c0 : nullptr);
            } else {
                hipLaunchKernelGGL(cv_scalars_lat_kernel, dim3((m + 63) / 64), dim3(64), 0, stream, m, ws_cap,
                                   pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0, ws_dig);
                hipLaunchKernelGGL(cv_points_pair_kernel, dim3((2 * m + 63) / 64), dim3(64), 0, stream, m,
                                   pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, ws_tab, ws_tabR, ws_ok,
                                   status ? status + c0 : nullptr);
            }
            if (ev && c0 == 0) (void)hipEventRecord(ev[1], stream);
            (void)hipMemsetAsync(bitmap + (size_t)c0 / 64, 0, (size_t)((m + 63) / 64) * 8, stream);
            if (ev && c0 == 0) (void)hipEventRecord(ev[2], stream);
            if (tri)
                hipLaunchKernelGGL(cv_hs_straus_tri_kernel, dim3((16 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0,
                                   stream, m, ws_cap, ws_dig, ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64);
            else
                hipLaunchKernelGGL(cv_hs_straus_quad_kernel, dim3((4 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK),
                                   0, stream, m, ws_cap, ws_dig, ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64);
            if (ev && c0 == 0) (void)hipEventRecord(ev[3], stream);
            continue;
        }
        SplitAux *ax = nullptr;
        bool split = false;
        if (!lat && g_verify_mode == 1 && g_hs_fused && g_split_mode && !ev && m >= 131072) {
            hipError_t e = split_aux(&ax);
            if (e != hipSuccess) return e;
            const uint32_t resident = (uint32_t)ax->cus * 4u * (uint32_t)g_hs_waves;   // waves in one round
            const uint32_t last = ((m + 63) / 64) % resident;
            split = g_split_mode != 3 || (resident && last && last * 100u <= resident * 12u);
        }
        if (split) {
            // fused half-size group in two sub-chunks: head [0, m1) on `stream`, tail [m1, m) on the
            // helper stream; `stream` waits for the tail before anything queued after this call.
            // Sub-chunk launches use the <.., true> instances so traces tell them from whole-chunk ones.
            uint32_t *ws_tabR = ws_tab + (size_t)ws_cap * CV_TAB_WORDS;
            const uint32_t m1 = (uint32_t)(((uint64_t)m * (100 - g_split_pct) / 100) & ~(uint64_t)255);
            const uint32_t m2 = m - m1;                 // the tail keeps the batch's ragged end
            const uint32_t sub0[2] = {0, m1}, subn[2] = {m1, m2};
            std::lock_guard<std::mutex> lk(ax->mu);
            (void)hipEventRecord(ax->start, stream);
            (void)hipStreamWaitEvent(ax->s2, ax->start, 0);
            for (int h = 0; h < 2; h++) {
                hipStream_t st = h ? ax->s2 : stream;
                const uint32_t a = c0 + sub0[h], mm = subn[h], bl = (mm + CV_BLOCK - 1) / CV_BLOCK;
                if (h == 1 && g_split_mode == 2) (void)hipStreamWaitEvent(st, ax->prep1, 0);
                hipLaunchKernelGGL(cv_scalars_kernel, dim3(bl), dim3(CV_BLOCK), 0, st, mm, ws_cap,
                                   pk + (size_t)a * 32, sig + (size_t)a * 64, arena, off + a, len + a,
                                   ws_dig + sub0[h]);
                launch_points<true>(mm, pk + (size_t)a * 32, sig + (size_t)a * 64, ws_tab + (size_t)sub0[h] * CV_TAB_WORDS,
                                    ws_tabR + (size_t)sub0[h] * CV_TAB_WORDS, ws_ok + sub0[h],
                                    status ? status + a : nullptr, st);
                if (h == 0) (void)hipEventRecord(ax->prep1, st);
                if (g_hs_waves == 2)
                    hipLaunchKernelGGL((cv_hs_straus_kernel<2, true>), dim3(bl), dim3(CV_BLOCK), 0, st, mm, ws_cap,
                                       ws_dig + sub0[h], ws_tab + (size_t)sub0[h] * CV_TAB_WORDS,
                                       ws_tabR + (size_t)sub0[h] * CV_TAB_WORDS, ws_ok + sub0[h], bitmap + a / 64);
                else
                    hipLaunchKernelGGL((cv_hs_straus_kernel<3, true>), dim3(bl), dim3(CV_BLOCK), 0, st, mm, ws_cap,
                                       ws_dig + sub0[h], ws_tab + (size_t)sub0[h] * CV_TAB_WORDS,
                                       ws_tabR + (size_t)sub0[h] * CV_TAB_WORDS, ws_ok + sub0[h], bitmap + a / 64);
            }
            (void)hipEventRecord(ax->done2, ax->s2);
            (void)hipStreamWaitEvent(stream, ax->done2, 0);
            continue;
        }
        if (!lat && g_verify_mode == 1 && g_hs_fused) {
            // half-size group: phases = scalars (hash, lattice, digits) | points (decodes, tables) | hs_straus
            uint32_t *ws_tabR = ws_tab + (size_t)ws_cap * CV_TAB_WORDS;
            hipLaunchKernelGGL(cv_scalars_kernel, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap,
                               pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0, ws_dig);
            if (ev && c0 == 0) (void)hipEventRecord(ev[1], stream);
            launch_points<false>(m, pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, ws_tab, ws_tabR, ws_ok,
                                 status ? status + c0 : nullptr, stream);
            if (ev && c0 == 0) (void)hipEventRecord(ev[2], stream);
            if (g_hs_waves == 2)
                hipLaunchKernelGGL(cv_hs_straus_kernel<2>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap, ws_dig,
                                   ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64);
            else
                hipLaunchKernelGGL(cv_hs_straus_kernel<3>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap, ws_dig,
                                   ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64);
            if (ev && c0 == 0) (void)hipEventRecord(ev[3], stream);
            continue;
        }
        if (lat || g_prep_lat)
            hipLaunchKernelGGL(cv_prep_kernel<true>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, pk + (size_t)c0 * 32,
                               sig + (size_t)c0 * 64, arena, off + c0, len + c0, ws_hs, ws_tab, ws_ok,
                               status ? status + c0 : nullptr);
        else
            hipLaunchKernelGGL(cv_prep_kernel<false>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, pk + (size_t)c0 * 32,
                               sig + (size_t)c0 * 64, arena, off + c0, len + c0, ws_hs, ws_tab, ws_ok,
                               status ? status + c0 : nullptr);
        if (ev && c0 == 0) (void)hipEventRecord(ev[1], stream);
        if (!lat && g_verify_mode == 1) {
            // half-size group: phases = prep | hsprep | hs_straus (verdict bits included)
            uint32_t *ws_tabR = ws_tab + (size_t)ws_cap * CV_TAB_WORDS;
            if (g_hsprep_lat)
                hipLaunchKernelGGL(cv_hsprep_kernel<true>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap,
                                   sig + (size_t)c0 * 64, ws_hs, ws_dig, ws_tabR, ws_ok, g_hs_reduce);
            else
                hipLaunchKernelGGL(cv_hsprep_kernel<false>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap,
                                   sig + (size_t)c0 * 64, ws_hs, ws_dig, ws_tabR, ws_ok, g_hs_reduce);
            if (ev && c0 == 0) (void)hipEventRecord(ev[2], stream);
            if (g_hs_waves == 2)
                hipLaunchKernelGGL(cv_hs_straus_kernel<2>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap, ws_dig,
                                   ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64);
            else
                hipLaunchKernelGGL(cv_hs_straus_kernel<3>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap, ws_dig,
                                   ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64);
            if (ev && c0 == 0) (void)hipEventRecord(ev[3], stream);
            continue;
        }
        if (n <= g_quad_max)
            hipLaunchKernelGGL(cv_straus_quad_kernel, dim3((4 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0,
                               stream, m, ws_hs, ws_tab, ws_R);
        else if (g_straus_waves == 2)
            hipLaunchKernelGGL(cv_straus_kernel<2>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_hs, ws_tab, ws_R);
        else if (g_straus_waves == 4)
            hipLaunchKernelGGL(cv_straus_kernel<4>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_hs, ws_tab, ws_R);
        else
            hipLaunchKernelGGL(cv_straus_kernel<3>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_hs, ws_tab, ws_R);
        if (ev && c0 == 0) (void)hipEventRecord(ev[2], stream);
        const uint32_t nbytes = ((m + 63) / 64) * 8;
        if (n <= g_quad_max)
            hipLaunchKernelGGL(cv_finish_kernel<true>, dim3((nbytes + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0,
                               stream, m, nbytes, sig + (size_t)c0 * 64, ws_R, ws_ok,
                               reinterpret_cast<uint8_t *>(bitmap) + (size_t)c0 / 8);
        else
            hipLaunchKernelGGL(cv_finish_kernel<false>, dim3((nbytes + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0,
                               stream, m, nbytes, sig + (size_t)c0 * 64, ws_R, ws_ok,
                               reinterpret_cast<uint8_t *>(bitmap) + (size_t)c0 / 8);
        if (ev && c0 == 0) (void)hipEventRecord(ev[3], stream);
    }
    return hipGetLastError();
}

// scratch: nk * CV_KTAB_WORDS words
hipError_t cvk_keyprep(uint32_t nk, const uint8_t *keys, const uint32_t *slots, uint32_t *scratch, uint32_t *ktab_pool,
                       uint8_t *kok_pool, hipStream_t stream) {
    if (nk == 0) return hipSuccess;
    hipLaunchKernelGGL(cv_keyprep_kernel, dim3((nk + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream, nk, keys,
                       slots, scratch, ktab_pool, kok_pool);
    return hipGetLastError();
}

// Keyed verify of n signatures (key i = keys[key_index[i]], its tables in slot slot_of_key[...]),
// chunked by the workspace capacity like cvk_verify.  ev: as in cvk_verify.
hipError_t cvk_verify_keyed(uint32_t n, const uint8_t *keys, const uint32_t *key_index, const uint32_t *slot_of_key,
                            const uint32_t *ktab_pool, const uint8_t *kok_pool, const uint8_t *sig,
                            const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint64_t *bitmap,
                            uint8_t *status, uint32_t *ws_hs, uint32_t *ws_R, uint8_t *ws_ok, uint32_t ws_cap,
                            hipStream_t stream, hipEvent_t *ev) {
    if (n == 0) return hipSuccess;
    if (ws_cap == 0 || ws_cap % 512) return hipErrorInvalidValue;
    for (uint32_t c0 = 0; c0 < n; c0 += ws_cap) {
        const uint32_t m = (n - c0 < ws_cap) ? n - c0 : ws_cap;
        const uint32_t blocks = (m + CV_BLOCK - 1) / CV_BLOCK;
        if (ev && c0 == 0) (void)hipEventRecord(ev[0], stream);
        hipLaunchKernelGGL(cv_keyed_prep_kernel, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, keys, key_index + c0,
                           slot_of_key, kok_pool, sig + (size_t)c0 * 64, arena, off + c0, len + c0, ws_hs, ws_ok,
                           status ? status + c0 : nullptr);
        if (ev && c0 == 0) (void)hipEventRecord(ev[1], stream);
        if (n <= g_quad_max)
            hipLaunchKernelGGL(cv_comb_quad_kernel, dim3((4 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream,
                               m, ws_hs, key_index + c0, slot_of_key, ktab_pool, ws_R);
        else if (g_comb_waves == 2)
            hipLaunchKernelGGL(cv_comb_kernel<2>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_hs, key_index + c0,
                               slot_of_key, ktab_pool, ws_R);
        else
            hipLaunchKernelGGL(cv_comb_kernel<3>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_hs, key_index + c0,
                               slot_of_key, ktab_pool, ws_R);
        if (ev && c0 == 0) (void)hipEventRecord(ev[2], stream);
        const uint32_t nbytes = ((m + 63) / 64) * 8;
        if (n <= g_quad_max)
            hipLaunchKernelGGL(cv_finish_kernel<true>, dim3((nbytes + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0,
                               stream, m, nbytes, sig + (size_t)c0 * 64, ws_R, ws_ok,
                               reinterpret_cast<uint8_t *>(bitmap) + (size_t)c0 / 8);
        else
            hipLaunchKernelGGL(cv_finish_kernel<false>, dim3((nbytes + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0,
                               stream, m, nbytes, sig + (size_t)c0 * 64, ws_R, ws_ok,
                               reinterpret_cast<uint8_t *>(bitmap) + (size_t)c0 / 8);
        if (ev && c0 == 0) (void)hipEventRecord(ev[3], stream);
    }
    return hipGetLastError();
}

hipError_t cvk_sign(uint32_t n, const uint8_t *seed, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                    uint8_t *pk, uint8_t *sig, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t blocks = (n + CV_BLOCK - 1) / CV_BLOCK;
    hipLaunchKernelGGL(cv_sign_kernel, dim3(blocks), dim3(CV_BLOCK), 0, stream, n, seed, arena, off, len, pk, sig);
    return hipGetLastError();
}

hipError_t cvk_pmt_verify(uint32_t ntrees, const uint8_t *kind, const uint32_t *left, const uint32_t *right,
                          const uint8_t *leaf_hash, const uint32_t *tree_begin, const uint8_t *root, const uint8_t *check,
                          const uint32_t *check_begin, uint32_t *dig, uint8_t *flag, uint8_t *verdict, uint8_t *status,
                          hipStream_t stream) {
    if (ntrees == 0) return hipSuccess;
    hipLaunchKernelGGL(cv_pmt_verify_kernel, dim3((ntrees + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream, ntrees,
                       kind, left, right, leaf_hash, tree_begin, root, check, check_begin, dig, flag, verdict, status);
    return hipGetLastError();
}

hipError_t cvk_merkle(uint32_t ntx, uint32_t nleaves, const uint8_t *arena, const uint64_t *leaf_off,
                      const uint32_t *leaf_len, const uint32_t *tx_begin, uint32_t *leaf_digest, uint8_t *ids,
                      uint8_t *status, hipStream_t stream) {
    if (nleaves) {
        hipLaunchKernelGGL(cv_leaf_hash_kernel, dim3((nleaves + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream,
                           nleaves, arena, leaf_off, leaf_len, leaf_digest);
    }
    if (ntx) {
        hipLaunchKernelGGL(cv_merkle_tree_kernel, dim3((ntx + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream,
                           ntx, tx_begin, leaf_digest, ids, status);
    }
    return hipGetLastError();
}

}  // extern "C"

// ---------------------------------------------------------------- calibration microbenchmarks
// Peak rate of the multiply-accumulate instruction the field arithmetic is built on (roofline
// denominator): 8 independent accumulators x 16 unrolled v_mad_u64_u32 per iteration, no other VALU.
// (cv_field.h accumulates every limb product with v_mad_u64_u32.)
__global__ __launch_bounds__(CV_BLOCK) void cv_mad_bench_kernel(uint32_t iters, uint64_t *out) {
    uint64_t acc[8];
    uint32_t a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        acc[k] = threadIdx.x + k;
        a[k] = threadIdx.x * 2654435761u + k;
        b[k] = blockIdx.x * 40503u + 7 * k + 1;
    }
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int k = 0; k < 8; k++)
                asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b[(k + r) & 7]) : "vcc");
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) s ^= acc[k];
    if (s == 0x1234567) out[0] = s;   // keep the chains alive
}

// Practical field-multiply rate: 4 independent fe_mul chains per lane.
__global__ __launch_bounds__(CV_BLOCK, 2) void cv_femul_bench_kernel(uint32_t iters, int32_t *out) {
    fe x[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int i = 0; i < 10; i++) x[k].v[i] = (threadIdx.x * 977u + k * 131u + i * 7919u) & 0xffffff;
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 4; k++) fe_mul(x[k], x[k], x[(k + 1) & 3]);
    }
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int i = 0; i < 10; i++) s ^= x[k].v[i];
    if (s == 0x1234567) out[0] = s;
}

// ---------------------------------------------------------------- diagnostics: phase cycle probe
// The fused prep (cv_hs_prep_fused) with s_memtime stamps at its phase boundaries: per wave, lane 0
// stores the shader-clock cycles of hash | lattice | digit packing | A+R decode | tables into
// stamps[wave * 8 + k] (vector stores).  Same code and launch shape as the product kernel; each
// stamp is ordered after the phase's result by a data dependency.  Diagnostic build only.
__device__ __forceinline__ uint64_t cv_stamp() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
    return t;
}
#define CV_DEP(x) asm volatile("" ::"v"(x))

__global__ __launch_bounds__(CV_BLOCK, 2) void cv_prep_probe_kernel(
    uint32_t n, uint32_t cap, const uint8_t *__restrict__ pk, const uint8_t *__restrict__ sig,
    const uint8_t *__restrict__ arena, const uint64_t *__restrict__ off, const uint32_t *__restrict__ len,
    uint32_t *__restrict__ ws_dig, uint32_t *__restrict__ ws_tab, uint32_t *__restrict__ ws_tabR,
    uint64_t *__restrict__ stamps) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t aw[8], rw[8], sw[8];
    load_words8(aw, pk + (size_t)i * 32);
    load_words8(rw, sig + (size_t)i * 64);
    load_words8(sw, sig + (size_t)i * 64 + 32);
    CV_DEP(aw[0]); CV_DEP(rw[0]); CV_DEP(sw[0]);
    uint64_t t[8];
    t[0] = cv_stamp();
    uint32_t hs[CV_HS_WORDS];
    {   // cv_keyed_hs, split: SHA-512 | the two mod-L scalars
        uint32_t pre[16], dg[16], hh[8], abyte[8], ss[8];
        ge_abyte_from_key(abyte, aw);
#pragma unroll
        for (int q = 0; q < 8; q++) { pre[q] = rw[q]; pre[8 + q] = abyte[q]; }
        sha512_pre_msg(dg, pre, 64, arena + off[i], len[i]);
        CV_DEP(dg[0]); CV_DEP(dg[15]);
        t[6] = cv_stamp();
        sc_reduce512(hh, dg);
        sc_effective_s(ss, sw);
#pragma unroll
        for (int q = 0; q < 8; q++) { hs[q] = hh[q]; hs[8 + q] = ss[q]; }
    }
    CV_DEP(hs[0]); CV_DEP(hs[15]);
    t[1] = cv_stamp();
    uint32_t h[8], s8[8], u[8], v[8], w[8];
#pragma unroll
    for (int q = 0; q < 8; q++) { h[q] = hs[q]; s8[q] = hs[8 + q]; }
    bool v_neg;
    int nwin;
    sc_halfsize(u, v, v_neg, nwin, w, h, s8);
    CV_DEP(u[7]); CV_DEP(v[7]); CV_DEP(w[7]);
    t[2] = cv_stamp();
    uint32_t *dig = ws_dig + i;
#pragma unroll 4
    for (int win = 0; win < 64; win++) {
        const int da = -digit16(u, win), dr = v_neg ? -digit16(v, win) : digit16(v, win);
        const bool bw = (win & 1) == 0 && win < 32;
        const int dlo = bw ? digit256(w, win >> 1) : 0, dhi = bw ? digit256(w, 16 + (win >> 1)) : 0;
        dig[(size_t)win * cap] = ((uint32_t)da & 0x1fu) | (((uint32_t)dr & 0x1fu) << 5) |
                                 (((uint32_t)dlo & 0x1ffu) << 10) | (((uint32_t)dhi & 0x1ffu) << 19);
    }
    dig[64 * (size_t)cap] = (uint32_t)nwin;
    t[3] = cv_stamp();
    ge_p3 P[2];
    bool ok[2];
    ge_decode2_0_1_0<false>(P, ok, aw, rw);
    CV_DEP(P[0].T.v[0]); CV_DEP(P[1].T.v[0]);
    t[4] = cv_stamp();
    ge_p3 nA;
    ge_p3_neg(nA, P[0]);
    ge_cached_multiples8(ws_tab + (size_t)i * CV_TAB_WORDS, nA);
    ge_cached_multiples8(ws_tabR + (size_t)i * CV_TAB_WORDS, P[1]);
    t[5] = cv_stamp();
    if ((threadIdx.x & 63u) == 0) {
        uint64_t *o = stamps + (size_t)(i >> 6) * 8;
#pragma unroll
        for (int k = 0; k < 5; k++) o[k] = t[k + 1] - t[k];
        o[5] = t[6] - t[0];                     // SHA-512 alone (part of phase 0)
    }
}

// Cycle-basis calibration: the chip-wide v_mad_u64_u32 bench again, with block 0's lane 0 stamping
// s_memtime (shader clock) and s_memrealtime (100 MHz) around its loop, so the rate converts to
// cycles per wave-instruction per SIMD at the clock the chip actually ran.
__global__ __launch_bounds__(CV_BLOCK) void cv_mad_clock_kernel(uint32_t iters, uint64_t *out) {
    uint64_t acc[8];
    uint32_t a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        acc[k] = threadIdx.x + k;
        a[k] = threadIdx.x * 2654435761u + k;
        b[k] = blockIdx.x * 40503u + 7 * k + 1;
    }
    uint64_t c0, r0, c1, r1;
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(c0), "=s"(r0));
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int k = 0; k < 8; k++)
                asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k]) : "v"(a[k]), "v"(b[(k + r) & 7]) : "vcc");
        }
    }
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(c1), "=s"(r1));
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) s ^= acc[k];
    if (s == 0x1234567) out[2] = s;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[0] = c1 - c0;
        out[1] = r1 - r0;
    }
}

extern "C" hipError_t cvk_prep_probe(uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                                     const uint64_t *off, const uint32_t *len, uint32_t *ws_dig, uint32_t *ws_tab,
                                     uint32_t ws_cap, uint64_t *stamps, hipStream_t stream) {
    if (n == 0 || n > ws_cap) return hipErrorInvalidValue;
    hipLaunchKernelGGL(cv_prep_probe_kernel, dim3((n + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream, n, ws_cap,
                       pk, sig, arena, off, len, ws_dig, ws_tab, ws_tab + (size_t)ws_cap * CV_TAB_WORDS, stamps);
    return hipGetLastError();
}
extern "C" hipError_t cvk_mad_clock(uint32_t iters, uint32_t blocks, uint64_t *out, hipStream_t stream) {
    hipLaunchKernelGGL(cv_mad_clock_kernel, dim3(blocks), dim3(CV_BLOCK), 0, stream, iters, out);
    return hipGetLastError();
}

extern "C" hipError_t cvk_calibrate(uint32_t iters, int which, uint32_t blocks, void *scratch, hipStream_t stream) {
    if (which == 0)
        hipLaunchKernelGGL(cv_mad_bench_kernel, dim3(blocks), dim3(CV_BLOCK), 0, stream, iters,
                           static_cast<uint64_t *>(scratch));
    else
        hipLaunchKernelGGL(cv_femul_bench_kernel, dim3(blocks), dim3(CV_BLOCK), 0, stream, iters,
                           static_cast<int32_t *>(scratch));
    return hipGetLastError();
}
