// cv_launch.h — internal ABI between the host library (cv_api.cpp) and the kernel launchers
// (cv_kernels.hip).  Not part of the public C-ABI (include/cordaverify.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Helper stream and events of one verify workspace slot, used by cvk_verify's drain overlap (a
// near-empty last round of a chunk is filled by a tail sub-chunk on s2).  Owned by cv_api.cpp (one per
// workspace slot, so two slots' calls never share a helper stream); cvk_verify only records and waits.
struct CvkSplit {
    hipStream_t s2 = nullptr;
    hipEvent_t start = nullptr, done2 = nullptr;
    int cus = 0;   // compute units of the device (resident waves per round = cus * 4 SIMDs * 3 waves)
};

// Prep overlap of a one-chunk verify (cv_api.cpp verify_shard_small): the caller records `ready` on the
// launch stream once the keys and signatures are enqueued for DMA, before the offsets, lengths and message
// bytes.  The point decodes and tables (which read only keys and signatures) wait for `ready` on `aux` and run
// beside the rest of the DMA and the scalars; the launch stream waits for `done` before the Straus kernel.
struct CvkPrepOverlap {
    hipStream_t aux = nullptr;
    hipEvent_t ready = nullptr, done = nullptr;
};

// The launch plan of one verify call, from the context's options (cv_set_option): which kernel form a
// batch of n signatures takes.  Read per call, so no launcher state is shared between contexts.
struct CvkPlan {
    uint32_t tri_max = 4096;    // n <= tri_max: tri-chain latency form (16 lanes per signature; 0 = never)
    uint32_t quad_max = 32768;  // n <= quad_max: quad latency form (4 lanes per signature; 0 = never)
    int split = 1;              // drain overlap of throughput chunks: 0 off, 1 auto (last round <= 12 % full), 2 always
    int split_pct = 10;         // the tail sub-chunk's share of a split chunk, percent
};

extern "C" {
// Verify n signatures with the workspace (capacity ws_cap signatures, a multiple of 512), in chunks of
// ws_cap.  split == nullptr disables the drain-overlap sub-chunks (the host pipeline overlaps its own
// sub-chunks across slots instead).  ev (optional, 4 events): phase boundaries of the first chunk.
// po (optional): prep overlap, taken when the batch is one chunk and ev is null (else ignored).
hipError_t cvk_verify(const CvkPlan *plan, uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                      const uint64_t *off, const uint32_t *len, uint64_t *bitmap, uint8_t *status, uint32_t *ws_tab,
                      uint8_t *ws_ok, uint32_t *ws_dig, uint32_t ws_cap, hipStream_t stream, hipEvent_t *ev,
                      const CvkSplit *split, const CvkPrepOverlap *po);
hipError_t cvk_sign(uint32_t n, const uint8_t *seed, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                    uint8_t *pk, uint8_t *sig, hipStream_t stream);
hipError_t cvk_pmt_verify(uint32_t ntrees, const uint8_t *kind, const uint32_t *left, const uint32_t *right,
                          const uint8_t *leaf_hash, const uint32_t *tree_begin, const uint8_t *root, const uint8_t *check,
                          const uint32_t *check_begin, uint32_t *dig, uint8_t *flag, uint8_t *verdict, uint8_t *status,
                          hipStream_t stream);
// Merkle ids of ntx transactions whose leaves are nleaves records starting at leaf index leaf_base:
// leaf_off / leaf_len index the records (leaf i of the call = record i), tx_begin[0..ntx] holds absolute
// leaf indices (tx_begin[0] >= leaf_base), leaf_digest is nleaves * 32 bytes of workspace.
hipError_t cvk_merkle(uint32_t ntx, uint32_t nleaves, uint32_t leaf_base, const uint8_t *arena, const uint64_t *leaf_off,
                      const uint32_t *leaf_len, const uint32_t *tx_begin, uint32_t *leaf_digest, uint8_t *ids,
                      uint8_t *status, hipStream_t stream);
// cv_verify_transactions: message references (off = 32 x the signature's transaction within the shard, len = 32)
// of shard-local signatures [c0, c0 + m); per-transaction verdicts from the shard's Merkle statuses and
// verdict bitmap.  tsb: the shard's nt + 1 absolute signature boundaries, tsb[0] = s0.
hipError_t cvk_tx_sig_refs(uint32_t m, uint32_t c0, uint32_t nt, uint32_t s0, const uint32_t *tsb, uint64_t *off,
                           uint32_t *len, hipStream_t stream);
hipError_t cvk_tx_verdicts(uint32_t nt, uint32_t s0, const uint32_t *tsb, const uint8_t *mstatus, const uint64_t *bitmap,
                           uint8_t *tx_ok, hipStream_t stream);
hipError_t cvk_calibrate(uint32_t iters, int which, uint32_t blocks, void *scratch, hipStream_t stream);
hipError_t cvk_mad_clock(uint32_t iters, uint32_t blocks, uint64_t *out, hipStream_t stream);
// Does a batch of n take the tri-chain form under this plan, in one chunk of a workspace of ws_cap?
int cvk_tri_zc_ok(const CvkPlan *plan, uint32_t n, uint32_t ws_cap);
hipError_t cvk_verify_tri_zc(const CvkPlan *plan, uint32_t n, const uint8_t *pk, const uint8_t *sig,
                             const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint8_t *nib,
                             uint8_t *status, uint32_t *ws_tab, uint8_t *ws_ok, uint32_t *ws_dig, uint32_t ws_cap,
                             hipStream_t stream, const void *copy_src, void *copy_dst, size_t copy_bytes);
hipError_t cvk_prepare(hipStream_t stream);
hipError_t cvk_keyprep(uint32_t nk, const uint8_t *keys, const uint32_t *slots, uint32_t *scratch, uint32_t *ktab_pool,
                       uint8_t *kok_pool, hipStream_t stream);
hipError_t cvk_verify_keyed(const CvkPlan *plan, uint32_t n, const uint8_t *keys, const uint32_t *key_index,
                            const uint32_t *slot_of_key, const uint32_t *ktab_pool, const uint8_t *kok_pool,
                            const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                            uint64_t *bitmap, uint8_t *status, uint32_t *ws_hs, uint32_t *ws_R, uint8_t *ws_ok,
                            uint32_t ws_cap, hipStream_t stream, hipEvent_t *ev);
}
