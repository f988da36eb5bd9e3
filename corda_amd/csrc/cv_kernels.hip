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
//
// This file holds the launchers (internal C ABI used by cv_api.cpp) and the runtime knobs; the
// kernels live in cv_k_*.hip (see cv_kcommon.h).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "cv_kcommon.h"
#include "cv_launch.h"

// occupancy variant of the Straus kernel (waves per SIMD the register budget is built for);
// tuned on the box with tools/ab_straus.py, default = the measured best
static int g_straus_waves = 3;
extern "C" void cvk_set_straus_waves(int w) { g_straus_waves = (w == 2 || w == 3 || w == 4) ? w : 3; }

// 0 = one lane decodes both points (cv_points_kernel: 256 VGPRs, 23 spilled, 2 waves/SIMD), 2 / 3 =
// lane pairs at that many waves per SIMD.  Default 3: points 2.46 -> 2.37 ms per 1M, C2 -0.8 % per step
// (same-box A/B, 3 alternating rounds, profiles/r02_ab_points_modes.log)
static int g_points_mode = 3;
extern "C" void cvk_set_points_mode(int v) { g_points_mode = (v == 2 || v == 3) ? v : 0; }
// 1 = scalars and point pairs of a throughput chunk in one launch (cv_prep_tp_kernel), 0 = two launches
static int g_prep_tp = 0;   // neutral in the same-box A/B (3.25 ms fused vs 0.89 + 2.39 ms), kept as a knob
extern "C" void cvk_set_prep_tp(int v) { g_prep_tp = v ? 1 : 0; }
// waves per SIMD of the throughput scalars kernel (2 = no VGPR spills, 3 = more latency hiding)
static int g_scalars_waves = 3;
extern "C" void cvk_set_scalars_waves(int v) { g_scalars_waves = (v == 2) ? 2 : 3; }
// the prep of a throughput (sub-)chunk [a, a + m): scalars -> ws_dig, decodes + tables -> tabA / tabR;
// mid (optional) is recorded between the two launches of the unfused form
template <bool SUB>
static void launch_points(uint32_t m, const uint8_t *pk, const uint8_t *sig, uint32_t *tabA, uint32_t *tabR, uint8_t *ok,
                          uint8_t *status, hipStream_t st);
// 1 = the scalars as two launches (cv_hash_kernel -> ws_hs -> cv_lattice_kernel), each at its own
// occupancy (g_hash_waves / g_lattice_waves per SIMD); 0 = one cv_scalars_kernel
static int g_scalars_split = 0, g_hash_waves = 3, g_lattice_waves = 3;
extern "C" void cvk_set_scalars_split(int v, int hash_waves, int lattice_waves) {
    g_scalars_split = v ? 1 : 0;
    g_hash_waves = hash_waves == 4 ? 4 : 3;
    g_lattice_waves = (lattice_waves == 2 || lattice_waves == 4) ? lattice_waves : 3;
}
template <bool SUB>
static void launch_prep_tp(uint32_t m, uint32_t cap, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                           const uint64_t *off, const uint32_t *len, uint32_t *dig, uint32_t *tabA, uint32_t *tabR,
                           uint8_t *ok, uint8_t *status, hipStream_t st, hipEvent_t mid, uint32_t *hs) {
    if (g_prep_tp && g_points_mode == 3) {
        const uint32_t nbp = (2 * m + CV_BLOCK - 1) / CV_BLOCK, nbs = (m + CV_BLOCK - 1) / CV_BLOCK;
        hipLaunchKernelGGL(cv_prep_tp_kernel<SUB>, dim3(nbp + nbs), dim3(CV_BLOCK), 0, st, m, cap, nbp, pk, sig, arena,
                           off, len, dig, tabA, tabR, ok, status);
        if (mid) (void)hipEventRecord(mid, st);
        return;
    }
    if (g_scalars_split && hs) {
        const dim3 g((m + CV_BLOCK - 1) / CV_BLOCK);
        if (g_hash_waves == 4)
            hipLaunchKernelGGL(cv_hash_kernel<4>, g, dim3(CV_BLOCK), 0, st, m, cap, pk, sig, arena, off, len, hs);
        else
            hipLaunchKernelGGL(cv_hash_kernel<3>, g, dim3(CV_BLOCK), 0, st, m, cap, pk, sig, arena, off, len, hs);
        if (g_lattice_waves == 4)
            hipLaunchKernelGGL(cv_lattice_kernel<4>, g, dim3(CV_BLOCK), 0, st, m, cap, hs, dig);
        else if (g_lattice_waves == 2)
            hipLaunchKernelGGL(cv_lattice_kernel<2>, g, dim3(CV_BLOCK), 0, st, m, cap, hs, dig);
        else
            hipLaunchKernelGGL(cv_lattice_kernel<3>, g, dim3(CV_BLOCK), 0, st, m, cap, hs, dig);
    } else if (g_scalars_waves == 2)
        hipLaunchKernelGGL(cv_scalars_kernel<2>, dim3((m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, st, m, cap, pk,
                           sig, arena, off, len, dig);
    else
        hipLaunchKernelGGL(cv_scalars_kernel<3>, dim3((m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, st, m, cap, pk,
                           sig, arena, off, len, dig);
    if (mid) (void)hipEventRecord(mid, st);
    launch_points<SUB>(m, pk, sig, tabA, tabR, ok, status, st);
}
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

// Batches of at most this many signatures run the tri-chain kernel (cvk_set_tri_max; 0 = never)
static uint32_t g_tri_max = 4096;
extern "C" void cvk_set_tri_max(int m) { g_tri_max = (uint32_t)(m < 0 ? 0 : m); }
extern "C" uint32_t cvk_get_tri_max(void) { return g_tri_max; }

// 1 = small batches run scalars and point pairs in one launch (cv_prep_lat_kernel), 0 = two launches
static int g_prep_lat_fused = 1;
extern "C" void cvk_set_prep_lat_fused(int v) { g_prep_lat_fused = v ? 1 : 0; }

// field forms of the latency kernels: bit 0 = tri, bit 1 = quad Straus, bit 2 = the fused latency
// prep's point decodes use the sequential-carry multiplications (fewer instructions) instead of the
// ILP forms
static int g_lat_seq = 7;
extern "C" void cvk_set_lat_seq(int v) { g_lat_seq = v & 7; }

// latency prep points with four lanes per signature (split odd-multiple tables, cv_points_quad_lane):
// 0 = never (lane pairs), 1 = tri-form batches, 2 = tri and quad forms
static int g_lat_points_quad = 1;
extern "C" void cvk_set_lat_points_quad(int v) { g_lat_points_quad = (v >= 0 && v <= 2) ? v : 1; }

// Batches of at most this many signatures run the quad kernels (set by cvk_set_quad_max; 0 = never)
static uint32_t g_quad_max = 32768;
extern "C" void cvk_set_quad_max(uint32_t m) { g_quad_max = m; }

// Does a batch of n take the tri-chain form with these settings (the zero-copy host path's condition:
// one chunk, half-size mode, latency forms on)?
extern "C" int cvk_tri_zc_ok(uint32_t n, uint32_t ws_cap) {
    return n > 0 && n <= g_tri_max && n <= g_quad_max && n <= ws_cap && g_verify_mode == 1 && g_hs_quad;
}

// ---------------------------------------------------------------- two-stream sub-chunk overlap
// A chunk of the half-size group is cut into a head and a tail sub-chunk; the tail runs on a helper
// stream so its waves fill the partial last rounds (drain) of the head's kernels.  mode 0 = off,
// 1 = both sub-chunks start together, 2 = the tail's prep waits for the head's prep, 3 = auto: mode 1
// when the chunk's last round of hs_straus waves is at most 12 % full (a near-empty drain round: 1M
// signatures = 5.09 rounds of 3072 resident waves on 256 CUs; measured 11.0-11.2 -> 10.7 ms), else off.
static int g_split_mode = 3, g_split_pct = 10;
extern "C" void cvk_set_split_mode(int m) { g_split_mode = (m >= 0 && m <= 3) ? m : 0; }
extern "C" void cvk_set_split_pct(int p) { g_split_pct = (p >= 5 && p <= 50) ? p : 10; }
static int g_comb_waves = 3;
extern "C" void cvk_set_comb_waves(int w) { g_comb_waves = (w == 2) ? 2 : 3; }

// ---------------------------------------------------------------- launchers (internal ABI)
// The CV_BW16 basepoint rows of the throughput group (cv_bw16_init_kernel), built once per device on
// first use: 4 x 32,769 entries x 128 B = 16.8 MB of device memory for the process's lifetime.
static uint32_t *g_bw16[16];
static std::mutex g_bw16_mu;
static hipError_t bw16_table(const uint32_t **out, hipStream_t st) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 16) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(g_bw16_mu);
    if (!g_bw16[dev]) {
        uint32_t *p = nullptr;
        if ((e = hipMalloc(&p, (size_t)CV_BW16_ROWS * CV_BW16_ROW * 4)) != hipSuccess) return e;
        hipLaunchKernelGGL(cv_bw16_init_kernel, dim3((CV_BW16_ROWS * CV_BW16_ENTRIES + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK),
                           0, st, p);
        if ((e = hipGetLastError()) == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            (void)hipFree(p);
            return e;
        }
        g_bw16[dev] = p;
    }
    *out = g_bw16[dev];
    return hipSuccess;
}

extern "C" {

// Build the current device's per-process tables now (cv_open calls this per device), so the first
// verify pays no table build and no hipStreamSynchronize runs inside a later stream capture.
hipError_t cvk_prepare(hipStream_t stream) {
    const uint32_t *bw16 = nullptr;
    return bw16_table(&bw16, stream);
}

// Zero-copy form of the tri-chain group (notary batches from host buffers, cv_api.cpp
// verify_shard_small): pk/sig/arena/off/len are device-visible pinned HOST memory that the fused prep
// reads over PCIe, status and nib are pinned host memory the kernels store into — no DMA in or out,
// so the call is one packing memcpy, two launches and one synchronisation.  nib gets one byte per
// wave (4 verdict bits, nib[i / 4] bit i % 4); the caller assembles the bitmap words.  Requires the
// tri form (n <= cvk_get_tri_max(), half-size mode) and n <= ws_cap: hipErrorInvalidValue otherwise.
//
// copy_src / copy_dst / copy_bytes (optional, 16-B aligned, copy_bytes a multiple of 16): a gather kernel
// first moves the packed records from pinned host memory into device memory with every lane of the
// grid reading its own 16-B pieces (many PCIe reads in flight at once), and pk..len point into copy_dst —
// instead of the prep's lanes reading them over PCIe one dependent load at a time.
hipError_t cvk_verify_tri_zc(uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                             const uint64_t *off, const uint32_t *len, uint8_t *nib, uint8_t *status,
                             uint32_t *ws_tab, uint8_t *ws_ok, uint32_t *ws_dig, uint32_t ws_cap, hipStream_t stream,
                             const void *copy_src, void *copy_dst, size_t copy_bytes) {
    if (n == 0) return hipSuccess;
    if (!cvk_tri_zc_ok(n, ws_cap) || !nib) return hipErrorInvalidValue;
    if (copy_bytes) {
        if (!copy_src || !copy_dst || copy_bytes % 16 || ((uintptr_t)copy_src | (uintptr_t)copy_dst) % 16)
            return hipErrorInvalidValue;
        const size_t q = copy_bytes / 16;
        const uint32_t blocks = (uint32_t)std::min<size_t>((q + 255) / 256, 2048);
        hipLaunchKernelGGL(cv_gather16_kernel, dim3(blocks), dim3(256), 0, stream,
                           static_cast<const uint4 *>(copy_src), static_cast<uint4 *>(copy_dst), q);
    }
    uint32_t *ws_tabR = ws_tab + (size_t)ws_cap * CV_TAB_WORDS;
    const uint32_t pts4 = g_lat_points_quad >= 1 ? 1u : 0u;
    const uint32_t nbp = ((pts4 ? 4 : 2) * n + 63) / 64, nbs = (n + 63) / 64;
    if (g_lat_seq & 4)
        hipLaunchKernelGGL((cv_prep_lat_kernel<true, false>), dim3(nbp + nbs), dim3(64), 0, stream, n, ws_cap, nbp,
                           pts4, pk, sig, arena, off, len, ws_dig, ws_tab, ws_tabR, ws_ok, status, nullptr);
    else
        hipLaunchKernelGGL((cv_prep_lat_kernel<true, true>), dim3(nbp + nbs), dim3(64), 0, stream, n, ws_cap, nbp,
                           pts4, pk, sig, arena, off, len, ws_dig, ws_tab, ws_tabR, ws_ok, status, nullptr);
    if (g_lat_seq & 1)
        hipLaunchKernelGGL(cv_hs_straus_tri_kernel<true>, dim3((16 * n + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0,
                           stream, n, ws_cap, ws_dig, ws_tab, ws_tabR, ws_ok, nullptr, nib);
    else
        hipLaunchKernelGGL(cv_hs_straus_tri_kernel<false>, dim3((16 * n + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0,
                           stream, n, ws_cap, ws_dig, ws_tab, ws_tabR, ws_ok, nullptr, nib);
    return hipGetLastError();
}

// Verify n signatures with the workspace ws (capacity ws_cap signatures, a multiple of 512); the
// batch is processed in chunks of ws_cap.  bitmap gets ceil(n/64) words.  ws_tab holds 2 * ws_cap
// tables (k*(-A), then k*R for the half-size group); ws_dig CV_HS_DIGWORDS * ws_cap words.  ev phases: prep | straus | finish, or in the
// half-size group prep | hsprep | hs_straus.
hipError_t cvk_verify(uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off,
                      const uint32_t *len, uint64_t *bitmap, uint8_t *status, uint32_t *ws_hs, uint32_t *ws_tab,
                      uint32_t *ws_R, uint8_t *ws_ok, uint32_t *ws_dig, uint32_t ws_cap, hipStream_t stream,
                      hipEvent_t *ev, const CvkSplit *ax) {
    if (n == 0) return hipSuccess;
    if (ws_cap == 0 || ws_cap % 512) return hipErrorInvalidValue;
    // the radix-2^16 basepoint rows, for the throughput (n > quad max) and quad (n > tri max) forms
    const uint32_t *bw16 = nullptr;
    if (g_verify_mode == 1 && (n > g_quad_max || n > g_tri_max)) {
        const hipError_t e = bw16_table(&bw16, stream);
        if (e != hipSuccess) return e;
    }
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
            if (!tri && !bw16) return hipErrorInvalidValue;   // (cannot happen: fetched above)
            if (g_prep_lat_fused || tri) {
                const uint32_t pts4 = (g_lat_points_quad == 2 || (g_lat_points_quad == 1 && tri)) ? 1u : 0u;
                const uint32_t nbp = ((pts4 ? 4 : 2) * m + 63) / 64, nbs = (m + 63) / 64;
                if (tri && (g_lat_seq & 4))
                    hipLaunchKernelGGL((cv_prep_lat_kernel<true, false>), dim3(nbp + nbs), dim3(64), 0, stream, m, ws_cap, nbp, pts4,
                                       pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0,
                                       ws_dig, ws_tab, ws_tabR, ws_ok, status ? status + c0 : nullptr,
                                       bitmap + (size_t)c0 / 64);
                else if (!tri && (g_lat_seq & 4))
                    hipLaunchKernelGGL((cv_prep_lat_kernel<false, false>), dim3(nbp + nbs), dim3(64), 0, stream, m, ws_cap, nbp, pts4,
                                       pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0,
                                       ws_dig, ws_tab, ws_tabR, ws_ok, status ? status + c0 : nullptr,
                                       bitmap + (size_t)c0 / 64);
                else if (tri)
                    hipLaunchKernelGGL((cv_prep_lat_kernel<true, true>), dim3(nbp + nbs), dim3(64), 0, stream, m, ws_cap, nbp, pts4,
                                       pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0,
                                       ws_dig, ws_tab, ws_tabR, ws_ok, status ? status + c0 : nullptr,
                                       bitmap + (size_t)c0 / 64);
                else
                    hipLaunchKernelGGL((cv_prep_lat_kernel<false, true>), dim3(nbp + nbs), dim3(64), 0, stream, m, ws_cap, nbp, pts4,
                                       pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0,
                                       ws_dig, ws_tab, ws_tabR, ws_ok, status ? status + c0 : nullptr,
                                       bitmap + (size_t)c0 / 64);
            } else {
                hipLaunchKernelGGL(cv_scalars_lat_kernel, dim3((m + 63) / 64), dim3(64), 0, stream, m, ws_cap,
                                   pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0, ws_dig);
                hipLaunchKernelGGL(cv_points_pair_kernel, dim3((2 * m + 63) / 64), dim3(64), 0, stream, m,
                                   pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, ws_tab, ws_tabR, ws_ok,
                                   status ? status + c0 : nullptr);
            }
            if (ev && c0 == 0) (void)hipEventRecord(ev[1], stream);
            // the fused prep zeroes the chunk's verdict words itself (no memset launch: -9 us)
            if (!(g_prep_lat_fused || tri))
                (void)hipMemsetAsync(bitmap + (size_t)c0 / 64, 0, (size_t)((m + 63) / 64) * 8, stream);
            if (ev && c0 == 0) (void)hipEventRecord(ev[2], stream);
            if (tri && (g_lat_seq & 1))
                hipLaunchKernelGGL(cv_hs_straus_tri_kernel<true>, dim3((16 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0,
                                   stream, m, ws_cap, ws_dig, ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64, nullptr);
            else if (tri)
                hipLaunchKernelGGL(cv_hs_straus_tri_kernel<false>, dim3((16 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0,
                                   stream, m, ws_cap, ws_dig, ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64, nullptr);
            else if (g_lat_seq & 2)
                hipLaunchKernelGGL(cv_hs_straus_quad_kernel<true>, dim3((4 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK),
                                   0, stream, m, ws_cap, ws_dig, ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64, bw16);
            else
                hipLaunchKernelGGL(cv_hs_straus_quad_kernel<false>, dim3((4 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK),
                                   0, stream, m, ws_cap, ws_dig, ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64, bw16);
            if (ev && c0 == 0) (void)hipEventRecord(ev[3], stream);
            continue;
        }
        if (g_verify_mode == 1 && !bw16) return hipErrorInvalidValue;   // (cannot happen: fetched above)
        bool split = false;
        if (ax && ax->s2 && !lat && g_verify_mode == 1 && g_hs_fused && g_split_mode && !ev && m >= 131072) {
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
            (void)hipEventRecord(ax->start, stream);
            (void)hipStreamWaitEvent(ax->s2, ax->start, 0);
            for (int h = 0; h < 2; h++) {
                hipStream_t st = h ? ax->s2 : stream;
                const uint32_t a = c0 + sub0[h], mm = subn[h], bl = (mm + CV_BLOCK - 1) / CV_BLOCK;
                if (h == 1 && g_split_mode == 2) (void)hipStreamWaitEvent(st, ax->prep1, 0);
                launch_prep_tp<true>(mm, ws_cap, pk + (size_t)a * 32, sig + (size_t)a * 64, arena, off + a, len + a,
                                     ws_dig + sub0[h], ws_tab + (size_t)sub0[h] * CV_TAB_WORDS,
                                     ws_tabR + (size_t)sub0[h] * CV_TAB_WORDS, ws_ok + sub0[h],
                                     status ? status + a : nullptr, st, nullptr, ws_hs + (size_t)sub0[h] * 4);
                if (h == 0) (void)hipEventRecord(ax->prep1, st);
                if (g_hs_waves == 2)
                    hipLaunchKernelGGL((cv_hs_straus_kernel<2, true>), dim3(bl), dim3(CV_BLOCK), 0, st, mm, ws_cap,
                                       ws_dig + sub0[h], ws_tab + (size_t)sub0[h] * CV_TAB_WORDS,
                                       ws_tabR + (size_t)sub0[h] * CV_TAB_WORDS, ws_ok + sub0[h], bitmap + a / 64, bw16);
                else
                    hipLaunchKernelGGL((cv_hs_straus_kernel<3, true>), dim3(bl), dim3(CV_BLOCK), 0, st, mm, ws_cap,
                                       ws_dig + sub0[h], ws_tab + (size_t)sub0[h] * CV_TAB_WORDS,
                                       ws_tabR + (size_t)sub0[h] * CV_TAB_WORDS, ws_ok + sub0[h], bitmap + a / 64, bw16);
            }
            (void)hipEventRecord(ax->done2, ax->s2);
            (void)hipStreamWaitEvent(stream, ax->done2, 0);
            continue;
        }
        if (!lat && g_verify_mode == 1 && g_hs_fused) {
            // half-size group: phases = scalars (hash, lattice, digits) | points (decodes, tables) | hs_straus
            uint32_t *ws_tabR = ws_tab + (size_t)ws_cap * CV_TAB_WORDS;
            // (fused prep: ev[1] and ev[2] both follow the one launch, so its time shows as "scalars")
            launch_prep_tp<false>(m, ws_cap, pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0,
                                  ws_dig, ws_tab, ws_tabR, ws_ok, status ? status + c0 : nullptr, stream,
                                  ev && c0 == 0 ? ev[1] : nullptr, ws_hs);
            if (ev && c0 == 0) (void)hipEventRecord(ev[2], stream);
            if (g_hs_waves == 2)
                hipLaunchKernelGGL(cv_hs_straus_kernel<2>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap, ws_dig,
                                   ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64, bw16);
            else
                hipLaunchKernelGGL(cv_hs_straus_kernel<3>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap, ws_dig,
                                   ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64, bw16);
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
                                   ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64, bw16);
            else
                hipLaunchKernelGGL(cv_hs_straus_kernel<3>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap, ws_dig,
                                   ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64, bw16);
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
    hipLaunchKernelGGL(cv_keyprep_kernel, dim3((CV_COMB_ROWS * nk + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream, nk, keys,
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
    const uint32_t *bw16 = nullptr;            // the comb kernel's radix-2^16 basepoint rows
    if (n > g_quad_max) {
        const hipError_t e = bw16_table(&bw16, stream);
        if (e != hipSuccess) return e;
    }
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
                               slot_of_key, ktab_pool, ws_R, bw16);
        else
            hipLaunchKernelGGL(cv_comb_kernel<3>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_hs, key_index + c0,
                               slot_of_key, ktab_pool, ws_R, bw16);
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

}  // extern "C"
// leaf hashing: 0 = length-sorted passes (cv_leaf_hash_kernel), 1 = balanced pairs (cv_leaf_hash_pair_kernel)
static int g_leaf_mode = 1;
extern "C" {
void cvk_set_leaf_mode(int m) { g_leaf_mode = m == 1 ? 1 : 0; }

hipError_t cvk_merkle(uint32_t ntx, uint32_t nleaves, const uint8_t *arena, const uint64_t *leaf_off,
                      const uint32_t *leaf_len, const uint32_t *tx_begin, uint32_t *leaf_digest, uint8_t *ids,
                      uint8_t *status, hipStream_t stream) {
    if (nleaves && g_leaf_mode == 1) {
        hipLaunchKernelGGL(cv_leaf_hash_pair_kernel, dim3((nleaves + 2 * CV_LEAF_BLOCK - 1) / (2 * CV_LEAF_BLOCK)),
                           dim3(CV_LEAF_BLOCK), 0, stream, nleaves, arena, leaf_off, leaf_len, leaf_digest);
    } else if (nleaves) {
        hipLaunchKernelGGL(cv_leaf_hash_kernel, dim3((nleaves + CV_LEAF_SPAN - 1) / CV_LEAF_SPAN), dim3(CV_LEAF_BLOCK), 0, stream,
                           nleaves, arena, leaf_off, leaf_len, leaf_digest);
    }
    if (ntx) {
        hipLaunchKernelGGL(cv_merkle_tree_kernel, dim3((ntx + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream,
                           ntx, tx_begin, leaf_digest, ids, status);
    }
    return hipGetLastError();
}

}  // extern "C"

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
