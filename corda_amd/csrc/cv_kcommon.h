// cv_kcommon.h — device helpers shared by the kernel translation units and the declarations of every
// kernel, so the launchers (cv_kernels.hip) and the kernels (cv_k_*.hip) build as separate objects in
// parallel:
//   cv_k_hs.hip    half-size throughput group: scalars, points (cv_k_hss.hip: hs_straus) — the C2/C3/C5 hot path
//   cv_k_lat.hip   latency forms for notary-sized batches: fused prep, quad and tri-chain Straus
//   cv_k_keyed.hip keyed per-key comb path (key tables, hash, comb, finish)
//   cv_k_misc.hip  signing, Merkle ids, partial Merkle trees, calibration kernels
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cv_verify.h"
#include "cv_quad.h"
#include "cv_hsquad.h"

#define CV_BLOCK 256
// waves per SIMD the throughput Straus kernel is built for (its __launch_bounds__; 168 VGPRs fit 3).  A build
// knob for A/Bs only (tools/ab_build_waves.sh NAME 2): both cv_k_hss.hip and the launchers must agree.
#ifndef CV_HSS_WAVES
#define CV_HSS_WAVES 3
#endif

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

// scalars of the half-size group, one lane per signature: h = SHA-512(R || Abyte || M) mod L, the
// effective S, the lattice (u, v, w) and the packed window digits -> ws_dig (cv_hs_scalars).  Its own
// kernel, at the occupancy its registers allow (3 waves per SIMD), because inside the 256-VGPR point
// kernel (2 waves per SIMD) the hash's serial 64-bit chains were 32 % of the prep's cycles
// (tools/prep_probe.py).  Any block size (small latency batches launch 64-thread blocks so the few
// waves spread over CUs).
template <bool B16 = false, bool W16 = false>
__device__ __forceinline__ void cv_scalars_lane(uint32_t i, uint32_t cap, const uint8_t *pk, const uint8_t *sig,
                                                const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                                                uint32_t *ws_dig) {
    uint32_t aw[8], rw[8], sw[8];
    load_words8(aw, pk + (size_t)i * 32);
    load_words8(rw, sig + (size_t)i * 64);
    load_words8(sw, sig + (size_t)i * 64 + 32);
    uint32_t hs[CV_HS_WORDS];
    cv_keyed_hs(aw, rw, sw, arena + off[i], len[i], hs);
    cv_hs_scalars<B16, W16>(hs, ws_dig + i, cap);
}

// points of the half-size group (latency form, small batches): a lane PAIR per signature, the even
// lane decoding the key A into k*(-A), the odd lane R into k*R, side by side (the same instructions
// on both lanes: cv_hs_point_one) with the latency (ILP) field forms — half the serial chain of the
// throughput form, whose single lane runs both decodes.  The even lane writes ok = key_ok AND r_ok.
// LAT = false: the sequential-carry field forms for the lone wave's decode chain (as the latency Straus
// kernels' SEQ forms), true: the ILP forms
template <bool LAT = true>
__device__ __forceinline__ void cv_points_pair_lane(uint32_t g, uint32_t n, const uint8_t *pk, const uint8_t *sig,
                                                    uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok,
                                                    uint8_t *status) {
    const uint32_t i = g >> 1;
    if (i >= n) return;                       // both lanes of a pair leave together
    const bool is_r = (g & 1u) != 0;
    uint32_t w[8];
    load_words8(w, is_r ? sig + (size_t)i * 64 : pk + (size_t)i * 32);
    const bool ok = cv_hs_point_one<LAT>(w, is_r, (is_r ? ws_tabR : ws_tab) + (size_t)i * CV_TAB_WORDS);
    const bool r_ok = __shfl_xor((int)ok, 1) != 0;
    if (!is_r) {
        ws_ok[i] = (ok && r_ok) ? 1 : 0;
        if (status) status[i] = ok ? 0 : 1;
    }
}

// points of the latency prep with FOUR lanes per signature (cv_prep_lat_kernel<true, ...>, the tri form): lanes 4i + {0, 1}
// decode A / R and build entries 0, 1, 3, 5, 7 of their table, lanes 4i + {2, 3} decode the same points
// (the redundant decode costs no time: the lanes are idle otherwise) and build entries 2, 4, 6, 8 —
// each lane's chain is the decode + 1 doubling + 3 additions instead of + 1 + 6
// (ge_cached_multiples8_half).  Lane 4i writes ok = key_ok AND r_ok.
template <bool LAT = true>
__device__ __forceinline__ void cv_points_quad_lane(uint32_t g, uint32_t n, const uint8_t *pk, const uint8_t *sig,
                                                    uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok,
                                                    uint8_t *status) {
    const uint32_t i = g >> 2;
    if (i >= n) return;                       // the four lanes of a signature leave together
    const bool is_r = (g & 1u) != 0;
    const int half = (int)((g >> 1) & 1u);
    uint32_t w[8];
    load_words8(w, is_r ? sig + (size_t)i * 64 : pk + (size_t)i * 32);
    const bool ok = cv_hs_point_one<LAT>(w, is_r, (is_r ? ws_tabR : ws_tab) + (size_t)i * CV_TAB_WORDS, half);
    const bool r_ok = __shfl_xor((int)ok, 1) != 0;
    if (!is_r && half == 0) {
        ws_ok[i] = (ok && r_ok) ? 1 : 0;
        if (status) status[i] = ok ? 0 : 1;
    }
}

// points of the half-size group, lane-pair throughput form: lane g of the grid handles signature
// g/2, the even lane decoding A into k*(-A), the odd lane R into k*R (sequential-carry field forms)
__device__ __forceinline__ void cv_points_one_lane(uint32_t g, uint32_t n, const uint8_t *pk, const uint8_t *sig,
                                                   uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok,
                                                   uint8_t *status) {
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

// ---------------------------------------------------------------- kernel declarations
template <bool LAT> __global__ void cv_finish_kernel(uint32_t n, uint32_t nbytes, const uint8_t *sig, const uint32_t *ws_R, const uint8_t *ws_ok, uint8_t *bitmap_bytes);
__global__ void cv_comb_quad_kernel(uint32_t n, const uint32_t *ws_hs, const uint32_t *key_index, const uint32_t *slot_of_key, const uint32_t *ktab_pool, uint32_t *ws_R);
__global__ void cv_keyprep_kernel(uint32_t nk, const uint8_t *keys, const uint32_t *slots, uint32_t *scratch, uint32_t *ktab_pool, uint8_t *kok_pool);
__global__ void cv_keyed_prep_kernel( uint32_t n, const uint8_t *keys, const uint32_t *key_index, const uint32_t *slot_of_key, const uint8_t *kok_pool, const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *ws_hs, uint8_t *ws_ok, uint8_t *status);
template <int WAVES> __global__ void cv_comb_kernel(uint32_t n, uint32_t *ws_hs, const uint32_t *key_index, const uint32_t *slot_of_key, const uint32_t *ktab_pool, uint32_t *ws_R, const uint32_t *bw16);
template <int WAVES> __global__ void cv_scalars_kernel(uint32_t n, uint32_t cap, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *ws_dig);
template <int WAVES, bool SUB = false> __global__ void cv_points_one_kernel(uint32_t n, const uint8_t *pk, const uint8_t *sig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status);
template <int WAVES, bool SUB = false> __global__ void cv_hs_straus_kernel(uint32_t n, uint32_t cap, const uint32_t *ws_dig, const uint32_t *ws_tab, const uint32_t *ws_tabR, const uint8_t *ws_ok, uint64_t *bitmap, const uint32_t *bw16);
__global__ void cv_bw16_init_kernel(uint32_t *tab);
template <bool B16, bool LAT = true> __global__ void cv_prep_lat_kernel(uint32_t n, uint32_t cap, uint32_t nbp, uint32_t pts4, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *ws_dig, uint32_t *ws_tab, uint32_t *ws_tabR, uint8_t *ws_ok, uint8_t *status, uint64_t *bitmap);
template <bool SEQ> __global__ void cv_hs_straus_quad_kernel(uint32_t n, uint32_t cap, const uint32_t *ws_dig, const uint32_t *ws_tab, const uint32_t *ws_tabR, const uint8_t *ws_ok, uint64_t *bitmap, const uint32_t *bw16);
__global__ void cv_gather16_kernel(const uint4 *src, uint4 *dst, size_t q);
template <bool SEQ> __global__ void cv_hs_straus_tri_kernel(uint32_t n, uint32_t cap, const uint32_t *ws_dig, const uint32_t *ws_tab, const uint32_t *ws_tabR, const uint8_t *ws_ok, uint64_t *bitmap, uint8_t *nib);
__global__ void cv_sign_kernel( uint32_t n, const uint8_t *seed, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint8_t *pk_out, uint8_t *sig_out);
// leaves per leaf-hash workgroup (each workgroup sorts 2 x CV_LEAF_BLOCK leaves by SHA-256 block count)
#define CV_LEAF_BLOCK 256
__global__ void cv_leaf_hash_pair_kernel(uint32_t nleaves, const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t *leaf_digest);
__global__ void cv_merkle_tree_kernel(uint32_t ntx, uint32_t leaf_base, const uint32_t *tx_begin, uint32_t *leaf_digest, uint8_t *ids, uint8_t *status);
__global__ void cv_tx_sig_refs_kernel(uint32_t m, uint32_t c0, uint32_t nt, uint32_t s0, const uint32_t *tsb, uint64_t *off, uint32_t *len);
__global__ void cv_tx_verdict_kernel(uint32_t nt, uint32_t s0, const uint32_t *tsb, const uint8_t *mstatus, const uint64_t *bitmap, uint8_t *tx_ok);
__global__ void cv_pmt_verify_kernel(uint32_t ntrees, const uint8_t *kind, const uint32_t *left, const uint32_t *right, const uint8_t *leaf_hash, const uint32_t *tree_begin, const uint8_t *root, const uint8_t *check, const uint32_t *check_begin, uint32_t *dig, uint8_t *flag, uint8_t *verdict, uint8_t *status);
__global__ void cv_mad_bench_kernel(uint32_t iters, uint64_t *out);
__global__ void cv_femul_bench_kernel(uint32_t iters, int32_t *out);
__global__ void cv_mad_clock_kernel(uint32_t iters, uint64_t *out);
