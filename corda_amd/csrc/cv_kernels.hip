// cv_kernels.hip — the launchers of the gfx950 kernels (internal C ABI used by cv_api.cpp, cv_launch.h).
//
//   verify (half-size scalars): eddsa-0.1.0-exact Ed25519 verify behind
//       PublicKey.verifyWithECDSA (reference core/src/main/kotlin/net/corda/core/crypto/CryptoUtilities.kt:90-96),
//       in three forms by batch size (CvkPlan): throughput (scalars -> points -> hs_straus, one signature per
//       lane), quad (4 lanes per signature) and tri-chain (16 lanes per signature) for notary-sized batches
//   keyed comb, signing (synthetic inputs), Merkle tx ids
//       (core/.../transactions/MerkleTransaction.kt:26-38,66-99), partial Merkle trees, calibration
//
// The kernels live in cv_k_*.hip (declarations: cv_kcommon.h).  No launcher state is global except the
// per-device basepoint rows (built once per process); every schedule choice comes from the caller's plan.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "cv_kcommon.h"
#include "cv_launch.h"

// ---------------------------------------------------------------- per-device basepoint rows
// The CV_BW16 rows of the throughput, quad and keyed forms (cv_bw16_init_kernel), built once per device:
// 4 x 32,769 entries x 128 B = 16.8 MB of device memory for the process's lifetime.
static uint32_t *g_bw16[64];
static std::mutex g_bw16_mu;
static hipError_t bw16_table(const uint32_t **out, hipStream_t st) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
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

// The prep of a throughput (sub-)chunk of m signatures: scalars -> dig, decodes + odd-multiple tables ->
// tabA / tabR (lane pairs at 3 waves per SIMD).  mid (optional) is recorded between the two launches.
template <bool SUB>
static void launch_prep_tp(uint32_t m, uint32_t cap, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                           const uint64_t *off, const uint32_t *len, uint32_t *dig, uint32_t *tabA, uint32_t *tabR,
                           uint8_t *ok, uint8_t *status, hipStream_t st, hipEvent_t mid) {
    hipLaunchKernelGGL(cv_scalars_kernel<3>, dim3((m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, st, m, cap, pk, sig,
                       arena, off, len, dig);
    if (mid) (void)hipEventRecord(mid, st);
    hipLaunchKernelGGL((cv_points_one_kernel<3, SUB>), dim3((2 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, st, m,
                       pk, sig, tabA, tabR, ok, status);
}

extern "C" {

// Build the current device's per-process tables now (cv_open calls this per device), so the first
// verify pays no table build and no hipStreamSynchronize runs inside a later stream capture.
hipError_t cvk_prepare(hipStream_t stream) {
    const uint32_t *bw16 = nullptr;
    return bw16_table(&bw16, stream);
}

int cvk_tri_zc_ok(const CvkPlan *plan, uint32_t n, uint32_t ws_cap) {
    return plan && n > 0 && n <= plan->tri_max && n <= plan->quad_max && n <= ws_cap;
}

// Zero-copy form of the tri-chain group (notary batches from host buffers, cv_api.cpp
// verify_shard_small_zc): pk/sig/arena/off/len are device-visible pinned HOST memory that the fused prep
// reads over PCIe, status and nib are pinned host memory the kernels store into — no DMA in or out,
// so the call is one packing memcpy, two launches and one synchronisation.  nib gets one byte per
// wave (4 verdict bits, nib[i / 4] bit i % 4); the caller assembles the bitmap words.  Requires the
// tri form (cvk_tri_zc_ok): hipErrorInvalidValue otherwise.
//
// copy_src / copy_dst / copy_bytes (optional, 16-B aligned, copy_bytes a multiple of 16): a gather kernel
// first moves the packed records from pinned host memory into device memory with every lane of the
// grid reading its own 16-B pieces (many PCIe reads in flight at once), and pk..len point into copy_dst —
// instead of the prep's lanes reading them over PCIe one dependent load at a time.
hipError_t cvk_verify_tri_zc(const CvkPlan *plan, uint32_t n, const uint8_t *pk, const uint8_t *sig,
                             const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint8_t *nib,
                             uint8_t *status, uint32_t *ws_tab, uint8_t *ws_ok, uint32_t *ws_dig, uint32_t ws_cap,
                             hipStream_t stream, const void *copy_src, void *copy_dst, size_t copy_bytes) {
    if (n == 0) return hipSuccess;
    if (!cvk_tri_zc_ok(plan, n, ws_cap) || !nib) return hipErrorInvalidValue;
    if (copy_bytes) {
        if (!copy_src || !copy_dst || copy_bytes % 16 || ((uintptr_t)copy_src | (uintptr_t)copy_dst) % 16)
            return hipErrorInvalidValue;
        const size_t q = copy_bytes / 16;
        const uint32_t blocks = (uint32_t)std::min<size_t>((q + 255) / 256, 2048);
        hipLaunchKernelGGL(cv_gather16_kernel, dim3(blocks), dim3(256), 0, stream,
                           static_cast<const uint4 *>(copy_src), static_cast<uint4 *>(copy_dst), q);
    }
    uint32_t *ws_tabR = ws_tab + (size_t)ws_cap * CV_TAB_WORDS;
    // four lanes per signature in the point half (split odd-multiple tables): prep 80.3 -> 73.8 us at 256
    const uint32_t nbp = (4 * n + 63) / 64, nbs = (n + 63) / 64;
    hipLaunchKernelGGL((cv_prep_lat_kernel<true, false>), dim3(nbp + nbs), dim3(64), 0, stream, n, ws_cap, nbp, 1u, pk,
                       sig, arena, off, len, ws_dig, ws_tab, ws_tabR, ws_ok, status, nullptr);
    hipLaunchKernelGGL(cv_hs_straus_tri_kernel<true>, dim3((16 * n + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream,
                       n, ws_cap, ws_dig, ws_tab, ws_tabR, ws_ok, nullptr, nib);
    return hipGetLastError();
}

// Verify n signatures with the workspace (capacity ws_cap signatures, a multiple of 512); the batch is
// processed in chunks of ws_cap.  bitmap gets ceil(n/64) words.  ws_tab holds 2 * ws_cap tables (k*(-A),
// then k*R); ws_dig CV_HS_DIGWORDS * ws_cap words.  ev phases (first chunk): throughput form scalars |
// points | hs_straus; latency forms scalars + point pairs | (nothing: the prep clears the bitmap) | Straus.
hipError_t cvk_verify(const CvkPlan *plan, uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                      const uint64_t *off, const uint32_t *len, uint64_t *bitmap, uint8_t *status, uint32_t *ws_tab,
                      uint8_t *ws_ok, uint32_t *ws_dig, uint32_t ws_cap, hipStream_t stream, hipEvent_t *ev,
                      const CvkSplit *ax, const CvkPrepOverlap *po) {
    if (n == 0) return hipSuccess;
    if (!plan || ws_cap == 0 || ws_cap % 512) return hipErrorInvalidValue;
    // prep overlap (one chunk only): points on po->aux after po->ready, scalars here, Straus after both
    const bool ov = po && po->aux && po->ready && po->done && n <= ws_cap && !ev;
    if (ov) (void)hipStreamWaitEvent(po->aux, po->ready, 0);
    // the radix-2^16 basepoint rows, for the throughput and quad forms
    const uint32_t *bw16 = nullptr;
    if (n > plan->tri_max || n > plan->quad_max) {
        const hipError_t e = bw16_table(&bw16, stream);
        if (e != hipSuccess) return e;
    }
    uint32_t *ws_tabR = ws_tab + (size_t)ws_cap * CV_TAB_WORDS;
    for (uint32_t c0 = 0; c0 < n; c0 += ws_cap) {
        const uint32_t m = (n - c0 < ws_cap) ? n - c0 : ws_cap;
        const uint32_t blocks = (m + CV_BLOCK - 1) / CV_BLOCK;
        if (ev && c0 == 0) (void)hipEventRecord(ev[0], stream);
        if (n <= plan->quad_max) {
            // latency forms: scalars and point pairs side by side in one launch (64-thread blocks: the few
            // waves spread over CUs), which also zeroes the chunk's verdict words; then the quad or
            // tri-chain Straus ORs each wave's bits in
            const bool tri = m <= plan->tri_max;
            const uint32_t nbp = ((tri ? 4 : 2) * m + 63) / 64, nbs = (m + 63) / 64;
            if (ov) {
                // the same kernel as two launches: point blocks only (grid nbp) on aux, scalar blocks only
                // (nbp = 0) here; the scalar blocks also clear the verdict words
                if (tri) {
                    hipLaunchKernelGGL((cv_prep_lat_kernel<true, false>), dim3(nbp), dim3(64), 0, po->aux, m, ws_cap, nbp,
                                       1u, pk, sig, arena, off, len, ws_dig, ws_tab, ws_tabR, ws_ok, status, bitmap);
                    (void)hipEventRecord(po->done, po->aux);
                    hipLaunchKernelGGL((cv_prep_lat_kernel<true, false>), dim3(nbs), dim3(64), 0, stream, m, ws_cap, 0u, 1u,
                                       pk, sig, arena, off, len, ws_dig, ws_tab, ws_tabR, ws_ok, status, bitmap);
                } else {
                    hipLaunchKernelGGL((cv_prep_lat_kernel<false, false>), dim3(nbp), dim3(64), 0, po->aux, m, ws_cap, nbp,
                                       0u, pk, sig, arena, off, len, ws_dig, ws_tab, ws_tabR, ws_ok, status, bitmap);
                    (void)hipEventRecord(po->done, po->aux);
                    hipLaunchKernelGGL((cv_prep_lat_kernel<false, false>), dim3(nbs), dim3(64), 0, stream, m, ws_cap, 0u, 0u,
                                       pk, sig, arena, off, len, ws_dig, ws_tab, ws_tabR, ws_ok, status, bitmap);
                }
                (void)hipStreamWaitEvent(stream, po->done, 0);
            } else if (tri)
                hipLaunchKernelGGL((cv_prep_lat_kernel<true, false>), dim3(nbp + nbs), dim3(64), 0, stream, m, ws_cap, nbp, 1u,
                                   pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0, ws_dig,
                                   ws_tab, ws_tabR, ws_ok, status ? status + c0 : nullptr, bitmap + (size_t)c0 / 64);
            else
                hipLaunchKernelGGL((cv_prep_lat_kernel<false, false>), dim3(nbp + nbs), dim3(64), 0, stream, m, ws_cap, nbp, 0u,
                                   pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0, ws_dig,
                                   ws_tab, ws_tabR, ws_ok, status ? status + c0 : nullptr, bitmap + (size_t)c0 / 64);
            if (ev && c0 == 0) (void)hipEventRecord(ev[1], stream);
            if (ev && c0 == 0) (void)hipEventRecord(ev[2], stream);
            if (tri)
                hipLaunchKernelGGL(cv_hs_straus_tri_kernel<true>, dim3((16 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0,
                                   stream, m, ws_cap, ws_dig, ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64, nullptr);
            else if (!bw16)
                return hipErrorInvalidValue;   // (cannot happen: fetched above)
            else
                hipLaunchKernelGGL(cv_hs_straus_quad_kernel<true>, dim3((4 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK),
                                   0, stream, m, ws_cap, ws_dig, ws_tab, ws_tabR, ws_ok, bitmap + (size_t)c0 / 64, bw16);
            if (ev && c0 == 0) (void)hipEventRecord(ev[3], stream);
            continue;
        }
        if (!bw16) return hipErrorInvalidValue;   // (cannot happen: fetched above)
        // Drain overlap: a chunk whose last round of hs_straus waves is near-empty is cut into a head
        // (90 %) on `stream` and a tail on the slot's helper stream starting with it, so the tail's waves
        // fill the head's drain (1M signatures = 5.09 rounds of 3,072 resident waves: 11.0-11.2 -> 10.7 ms).
        bool split = false;
        if (!ov && ax && ax->s2 && plan->split && !ev && m >= 131072) {
            const uint32_t resident = (uint32_t)ax->cus * 4u * 3u;   // hs_straus waves in one round
            const uint32_t last = ((m + 63) / 64) % resident;
            split = plan->split == 2 || (resident && last && last * 100u <= resident * 12u);
        }
        if (split) {
            // head [0, m1) on `stream`, tail [m1, m) on the helper; `stream` waits for the tail before
            // anything queued after this call.  Sub-chunk launches use the <.., true> instances so traces
            // tell them from whole-chunk ones.
            const int pct = plan->split_pct >= 5 && plan->split_pct <= 50 ? plan->split_pct : 10;
            const uint32_t m1 = (uint32_t)(((uint64_t)m * (100 - pct) / 100) & ~(uint64_t)255);
            const uint32_t m2 = m - m1;                 // the tail keeps the batch's ragged end
            const uint32_t sub0[2] = {0, m1}, subn[2] = {m1, m2};
            (void)hipEventRecord(ax->start, stream);
            (void)hipStreamWaitEvent(ax->s2, ax->start, 0);
            for (int h = 0; h < 2; h++) {
                hipStream_t st = h ? ax->s2 : stream;
                const uint32_t a = c0 + sub0[h], mm = subn[h], bl = (mm + CV_BLOCK - 1) / CV_BLOCK;
                launch_prep_tp<true>(mm, ws_cap, pk + (size_t)a * 32, sig + (size_t)a * 64, arena, off + a, len + a,
                                     ws_dig + sub0[h], ws_tab + (size_t)sub0[h] * CV_TAB_WORDS,
                                     ws_tabR + (size_t)sub0[h] * CV_TAB_WORDS, ws_ok + sub0[h],
                                     status ? status + a : nullptr, st, nullptr);
                hipLaunchKernelGGL((cv_hs_straus_kernel<CV_HSS_WAVES, true>), dim3(bl), dim3(CV_BLOCK), 0, st, mm, ws_cap,
                                   ws_dig + sub0[h], ws_tab + (size_t)sub0[h] * CV_TAB_WORDS,
                                   ws_tabR + (size_t)sub0[h] * CV_TAB_WORDS, ws_ok + sub0[h], bitmap + a / 64, bw16);
            }
            (void)hipEventRecord(ax->done2, ax->s2);
            (void)hipStreamWaitEvent(stream, ax->done2, 0);
            continue;
        }
        // throughput group: scalars (hash, lattice, digits) | points (decodes, tables) | hs_straus
        if (ov) {
            hipLaunchKernelGGL((cv_points_one_kernel<3, false>), dim3((2 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0,
                               po->aux, m, pk, sig, ws_tab, ws_tabR, ws_ok, status);
            (void)hipEventRecord(po->done, po->aux);
            hipLaunchKernelGGL(cv_scalars_kernel<3>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap, pk, sig, arena, off,
                               len, ws_dig);
            (void)hipStreamWaitEvent(stream, po->done, 0);
            hipLaunchKernelGGL(cv_hs_straus_kernel<CV_HSS_WAVES>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap, ws_dig, ws_tab,
                               ws_tabR, ws_ok, bitmap, bw16);
            continue;
        }
        launch_prep_tp<false>(m, ws_cap, pk + (size_t)c0 * 32, sig + (size_t)c0 * 64, arena, off + c0, len + c0, ws_dig,
                              ws_tab, ws_tabR, ws_ok, status ? status + c0 : nullptr, stream,
                              ev && c0 == 0 ? ev[1] : nullptr);
        if (ev && c0 == 0) (void)hipEventRecord(ev[2], stream);
        hipLaunchKernelGGL(cv_hs_straus_kernel<CV_HSS_WAVES>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_cap, ws_dig, ws_tab,
                           ws_tabR, ws_ok, bitmap + (size_t)c0 / 64, bw16);
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
// chunked by the workspace capacity like cvk_verify; batches up to the plan's quad size use the quad comb.
// ev: key tables (recorded by the caller) | hash | comb | finish.
hipError_t cvk_verify_keyed(const CvkPlan *plan, uint32_t n, const uint8_t *keys, const uint32_t *key_index,
                            const uint32_t *slot_of_key, const uint32_t *ktab_pool, const uint8_t *kok_pool,
                            const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                            uint64_t *bitmap, uint8_t *status, uint32_t *ws_hs, uint32_t *ws_R, uint8_t *ws_ok,
                            uint32_t ws_cap, hipStream_t stream, hipEvent_t *ev) {
    if (n == 0) return hipSuccess;
    if (!plan || ws_cap == 0 || ws_cap % 512) return hipErrorInvalidValue;
    const bool quad = n <= plan->quad_max;
    const uint32_t *bw16 = nullptr;            // the comb kernel's radix-2^16 basepoint rows
    if (!quad) {
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
        if (quad)
            hipLaunchKernelGGL(cv_comb_quad_kernel, dim3((4 * m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream,
                               m, ws_hs, key_index + c0, slot_of_key, ktab_pool, ws_R);
        else
            hipLaunchKernelGGL(cv_comb_kernel<3>, dim3(blocks), dim3(CV_BLOCK), 0, stream, m, ws_hs, key_index + c0,
                               slot_of_key, ktab_pool, ws_R, bw16);
        if (ev && c0 == 0) (void)hipEventRecord(ev[2], stream);
        const uint32_t nbytes = ((m + 63) / 64) * 8;
        // the sequential-carry finish for both comb forms: its ILP twin (the former quad-comb finish) kept its
        // eight prefix products in 336 B of scratch
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

// Leaf hashing: balanced pairs (round 3: 2.58 -> 2.47 ms per 1M C3 txs against the length-sorted passes,
// profiles/r03a_ab_leaf_mode.log), then one lane per transaction for the tree.
hipError_t cvk_merkle(uint32_t ntx, uint32_t nleaves, uint32_t leaf_base, const uint8_t *arena, const uint64_t *leaf_off,
                      const uint32_t *leaf_len, const uint32_t *tx_begin, uint32_t *leaf_digest, uint8_t *ids,
                      uint8_t *status, hipStream_t stream) {
    if (nleaves)
        hipLaunchKernelGGL(cv_leaf_hash_pair_kernel, dim3((nleaves + 2 * CV_LEAF_BLOCK - 1) / (2 * CV_LEAF_BLOCK)),
                           dim3(CV_LEAF_BLOCK), 0, stream, nleaves, arena, leaf_off, leaf_len, leaf_digest);
    if (ntx)
        hipLaunchKernelGGL(cv_merkle_tree_kernel, dim3((ntx + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream, ntx,
                           leaf_base, tx_begin, leaf_digest, ids, status);
    return hipGetLastError();
}

hipError_t cvk_tx_sig_refs(uint32_t m, uint32_t c0, uint32_t nt, uint32_t s0, const uint32_t *tsb, uint64_t *off,
                           uint32_t *len, hipStream_t stream) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(cv_tx_sig_refs_kernel, dim3((m + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream, m, c0, nt,
                       s0, tsb, off, len);
    return hipGetLastError();
}

hipError_t cvk_tx_verdicts(uint32_t nt, uint32_t s0, const uint32_t *tsb, const uint8_t *mstatus, const uint64_t *bitmap,
                           uint8_t *tx_ok, hipStream_t stream) {
    if (nt == 0) return hipSuccess;
    hipLaunchKernelGGL(cv_tx_verdict_kernel, dim3((nt + CV_BLOCK - 1) / CV_BLOCK), dim3(CV_BLOCK), 0, stream, nt, s0, tsb,
                       mstatus, bitmap, tx_ok);
    return hipGetLastError();
}

hipError_t cvk_mad_clock(uint32_t iters, uint32_t blocks, uint64_t *out, hipStream_t stream) {
    hipLaunchKernelGGL(cv_mad_clock_kernel, dim3(blocks), dim3(CV_BLOCK), 0, stream, iters, out);
    return hipGetLastError();
}

hipError_t cvk_calibrate(uint32_t iters, int which, uint32_t blocks, void *scratch, hipStream_t stream) {
    if (which == 0)
        hipLaunchKernelGGL(cv_mad_bench_kernel, dim3(blocks), dim3(CV_BLOCK), 0, stream, iters,
                           static_cast<uint64_t *>(scratch));
    else
        hipLaunchKernelGGL(cv_femul_bench_kernel, dim3(blocks), dim3(CV_BLOCK), 0, stream, iters,
                           static_cast<int32_t *>(scratch));
    return hipGetLastError();
}

}  // extern "C"
