/*
 * cordaverify.h — C-ABI of the MI355X batched signature-verification engine for Corda's
 * transaction-validation hot path.  Plain pointers and sizes only (no C++ / torch types), so the
 * JVM binds it directly through JNA or JNI (binding stubs: INTEGRATION.md).
 *
 * What each entry point replaces in the reference (MarioAriasC/corda @ 0.7-SNAPSHOT):
 *
 *   cv_ed25519_verify_batch   N x  PublicKey.verifyWithECDSA(content, signature)
 *                                 core/src/main/kotlin/net/corda/core/crypto/CryptoUtilities.kt:90-96
 *                             i.e. net.i2p.crypto:eddsa:0.1.0 EdDSAEngine.initVerify/update/verify
 *                             (jar pinned at core/build.gradle:80), looped sequentially by
 *                             SignedTransaction.checkSignaturesAreValid()
 *                                 core/src/main/kotlin/net/corda/core/transactions/SignedTransaction.kt:82-87
 *                             and by the notary / resolve flows (NotaryFlow.kt:97-113,
 *                             ValidatingNotaryFlow.kt:24-45, ResolveTransactionsFlow.kt:105-111).
 *                             Verdicts are bit-exact with eddsa-0.1.0, adversarial inputs included.
 *   cv_merkle_tx_ids          N x  WireTransaction.id  (= MerkleTree.getMerkleTree(leafHashes).hash)
 *                                 core/src/main/kotlin/net/corda/core/transactions/WireTransaction.kt:45-52
 *                                 core/src/main/kotlin/net/corda/core/transactions/MerkleTransaction.kt:26-38,66-99
 *                             leaf hash = SecureHash.sha256(leaf bytes)  (core/.../crypto/SecureHash.kt:33)
 *   cv_ed25519_sign_batch     N x  PrivateKey.signWithECDSA(bytes) after entropyToKeyPair/seed
 *                                 CryptoUtilities.kt:63-73,123-130 (deterministic RFC 8032; used to
 *                                 generate synthetic workloads, not on the validation path)
 *   cv_tx_verdicts            per-transaction AND of signature verdicts (the "all sigs valid" half of
 *                                 SignedTransaction.verifySignatures, SignedTransaction.kt:58-72)
 *   cv_verify_transactions    N x  SignedTransaction.verifySignatures' id + signature checks in one call
 *                                 (SignedTransaction.kt:59-71, 83-87; WireTransaction.kt:45-52)
 *   cv_partial_merkle_verify  N x  PartialMerkleTree.verify(merkleRootHash, hashesToCheck)
 *                                 core/src/main/kotlin/net/corda/core/crypto/PartialMerkleTree.kt:117-144
 *                             behind FilteredTransaction.verify (MerkleTransaction.kt:170-178; the
 *                             oracle tear-off check of NodeInterestRates.kt:189-191)
 *
 * Conventions
 *   - Return codes: CV_OK (0) or a negative CV_E* code; nothing throws, aborts or longjmps across
 *     the ABI.  cv_strerror() gives a static message.
 *   - Host-buffer calls are synchronous unless named _async; the caller owns every buffer.  A cv_ctx is
 *     thread-safe: calls from several threads run concurrently on different devices (each device has
 *     its own lock and worker thread) and queue on the same one.  A notary's batching threads share one
 *     context (the JVM shim holds one ctx per process, no mutex around it).
 *   - Record layout (structure-of-arrays): pk[n][32], sig[n][64] (R || S), message i is
 *     msg_arena[msg_off[i] .. msg_off[i] + msg_len[i]).
 *   - verdict_bitmap: ceil(n/64) uint64 words, bit (i % 64) of word (i / 64) = signature i valid.
 *   - status (optional, may be NULL): one byte per signature, CV_SIG_OK or CV_SIG_BAD_KEY (the key
 *     bytes are not a valid point: the reference throws IllegalArgumentException when building the
 *     EdDSAPublicKey).  Length errors (sig != 64 B -> SignatureException, key != 32 B) cannot be
 *     expressed in these fixed-width records; the host shim rejects them before the call.
 *   - Multi-GPU: cv_open(mask) with several bits set routes host-buffer batches over the devices: a batch
 *     up to CV_OPT_SHARD_MIN records goes whole to the least loaded device; a throughput batch (from
 *     CV_OPT_SPREAD_MIN records) is cut into contiguous ranges (multiples of 64) over all of them; a batch
 *     between the two is cut over the devices idle at submission (at most ceil(n / CV_OPT_SHARD_MIN) of
 *     them, at least the least loaded one).  No collective: each shard's results land in the caller's
 *     arrays.
 */
#ifndef CORDAVERIFY_H
#define CORDAVERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CV_OK 0
#define CV_E_NO_DEVICE (-1)   /* no HIP device matches the mask */
#define CV_E_HIP (-2)         /* a HIP runtime call failed */
#define CV_E_ARGS (-3)        /* null pointer / bad size */
#define CV_E_OOM (-4)         /* device allocation failed */
#define CV_E_TOO_LARGE (-5)   /* more than 2^32-1 records in one shard */

#define CV_SIG_OK 0
#define CV_SIG_BAD_KEY 1
#define CV_TX_OK 0
#define CV_TX_EMPTY 1         /* no leaves: MerkleTreeException("Cannot calculate Merkle root on empty hash list.") */

typedef struct cv_ctx cv_ctx;

/* Open a context on the devices in device_mask (bit d = HIP device ordinal d; 0 = all devices).
 * The first open on a device also builds that device's basepoint rows (16.8 MB, kept for the
 * process lifetime, shared by every context), so it takes a few milliseconds longer. */
int cv_open(uint32_t device_mask, cv_ctx **out);
/* As cv_open; slots_per_device (1..16) > 1 makes each GPU of the mask appear that many times in THIS context
 * as independent device slots (own lock, worker thread, streams, workspaces, key pool), so the multi-device
 * routing below runs on a one-GPU machine (tests).  slots_per_device = 1 is cv_open. */
int cv_open_ex(uint32_t device_mask, int slots_per_device, cv_ctx **out);
void cv_close(cv_ctx *ctx);
const char *cv_strerror(int code);
const char *cv_version(void);
/* Number of devices in the context. */
int cv_device_count(const cv_ctx *ctx);

/* ---------------------------------------------------------------- host-buffer API (JVM drop-in) */

int cv_ed25519_verify_batch(cv_ctx *ctx, size_t n, const uint8_t *pk, const uint8_t *sig,
                            const uint8_t *msg_arena, const uint64_t *msg_off, const uint32_t *msg_len,
                            uint64_t *verdict_bitmap, uint8_t *status);

/* Asynchronous form of cv_ed25519_verify_batch (same records, same verdicts and status, the same
 * automatic keyed path for batches whose keys repeat): enqueues the batch on the context's devices and
 * returns a ticket; cv_wait(ticket) returns once verdict_bitmap and status hold the results.  Until then
 * the caller keeps every array of the call alive and unmodified (pinned inputs are read by DMA after this
 * call returns).  Four pipelined calls (verify or Merkle) per device may be in flight: a fifth first
 * completes the oldest (whose cv_wait then returns at once).  A node's batching loop submits batch k+1
 * before waiting for batch k, so its copies and kernels fill the first one's pipeline ramp and tail.
 * cv_wait may run on another thread than the submission and does not block submissions.  It returns the
 * call's own status — also when a later call already completed it (a HIP failure while finishing a call is
 * reported to that call's waiter, never to the later caller).  Tickets are waited at most once (again:
 * CV_E_ARGS); a completed ticket keeps its status for cv_wait until 4,096 later tickets have completed;
 * cv_close drops results not yet waited for. */
int cv_ed25519_verify_batch_async(cv_ctx *ctx, size_t n, const uint8_t *pk, const uint8_t *sig,
                                  const uint8_t *msg_arena, const uint64_t *msg_off, const uint32_t *msg_len,
                                  uint64_t *verdict_bitmap, uint8_t *status, uint64_t *ticket);
int cv_wait(cv_ctx *ctx, uint64_t ticket);

/* cv_ed25519_verify_batch (ticket NULL) or its _async form (ticket non-NULL) with the arena's size: a call whose
 * records reach past msg_arena[arena_bytes) returns CV_E_ARGS before the engine reads past it.  The check rides on
 * the staging scan every call makes anyway (the byte range its records reach, per shard and sub-chunk), so a
 * binding gets bounds safety without scanning the offsets itself (cv_msg_extent, an extra pass over 12 B per
 * record).  With a ticket, records past the bound in a later shard may be found after earlier shards were
 * enqueued: the call then waits for those before it returns CV_E_ARGS. */
int cv_ed25519_verify_batch_ex(cv_ctx *ctx, size_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg_arena,
                               uint64_t arena_bytes, const uint64_t *msg_off, const uint32_t *msg_len,
                               uint64_t *verdict_bitmap, uint8_t *status, uint64_t *ticket);

/* Pinned host memory for the host-buffer API's inputs (hipHostMalloc).  When all five input arrays of
 * cv_ed25519_verify_batch lie in pinned memory (from here, or any page-locked / registered host memory),
 * the engine DMAs each sub-chunk's records straight out of them and skips its packing copy into its own
 * staging: a JVM shim that builds its batches in buffers from cv_host_alloc (JNA Pointer ->
 * ByteBuffer) feeds the GPU at PCIe rate.  The memory stays valid until cv_host_free; ctx only selects
 * the allocator (any open context). */
int cv_host_alloc(cv_ctx *ctx, size_t bytes, void **out);
void cv_host_free(cv_ctx *ctx, void *p);

/* Keyed batch: the distinct keys once, keys[nkeys][32], and per signature
 * key_index[n] into them.  Replaces the same N x PublicKey.verifyWithECDSA as
 * cv_ed25519_verify_batch — identical verdicts and status — for batches whose keys repeat (a notary
 * batch, a ResolveTransactionsFlow chain, a party's transactions): the engine keeps per-key tables
 * (decoded A and comb multiples k * 2^(64j) * (-A), k = 0..128, 66 KB per key, affine) resident on each
 * device, keyed by the 32 key bytes, so a key is decoded once and each verify needs 56 doublings
 * instead of 252.
 * cv_ed25519_verify_batch(_async) takes this path by itself (host-side dedupe, any batch size above
 * CV_OPT_TRI_MAX) for batches with at least eight signatures per distinct key. */
int cv_ed25519_verify_batch_keyed(cv_ctx *ctx, size_t n, size_t nkeys, const uint8_t *keys, const uint32_t *key_index,
                                  const uint8_t *sig, const uint8_t *msg_arena, const uint64_t *msg_off,
                                  const uint32_t *msg_len, uint64_t *verdict_bitmap, uint8_t *status);

/* Per-device key-table pool capacity in keys (default 16384 = 1.1 GB of HBM per device: 66 KB of
 * comb tables per key); takes effect at the next keyed call.  A pool that fills up is emptied before
 * new keys go in; a call with more distinct keys than the capacity grows the pool to fit them. */
int cv_key_cache_reserve(cv_ctx *ctx, size_t max_keys);

/* out4 = {resident keys, capacity, lookups that hit, lookups that missed} for `device`. */
int cv_key_cache_stats(cv_ctx *ctx, int device, uint64_t *out4);

int cv_merkle_tx_ids(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                     const uint32_t *leaf_len, const uint32_t *tx_leaf_begin /* ntx+1 */, uint8_t *ids /* ntx*32 */);

/* as cv_merkle_tx_ids, with per-transaction status (CV_TX_OK / CV_TX_EMPTY).  Transactions are cut into
 * contiguous ranges over the context's devices (routed as the verify batches), each range's leaves copied
 * from its own byte window of leaf_arena (offsets need not be sorted; scattered leaves are gathered) and
 * pipelined through the devices' copy streams in sub-chunks of about CV_OPT_MERKLE_CHUNK leaves; leaf
 * arrays in pinned memory (cv_host_alloc) are DMAed in place. */
int cv_merkle_tx_ids_ex(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                        const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, uint8_t *ids, uint8_t *tx_status);

/* Asynchronous form of cv_merkle_tx_ids_ex (ticket and cv_wait as cv_ed25519_verify_batch_async): a C3 node
 * step submits the Merkle ids of batch k+1 while the verify of batch k runs, so their copies overlap. */
int cv_merkle_tx_ids_async(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                           const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, uint8_t *ids, uint8_t *tx_status,
                           uint64_t *ticket);

/* cv_merkle_tx_ids_ex (ticket NULL) or cv_merkle_tx_ids_async (ticket non-NULL) with the leaf arena's size: a call
 * whose leaves reach past leaf_arena[leaf_arena_bytes) (or whose off + len wraps) returns CV_E_ARGS before the
 * engine reads past it — the check rides on the staging scan of each sub-chunk's leaves, so a binding needs no
 * scan of its own (6M leaves: ~10 ms of host time per call).  With a ticket, leaves past the bound in a later
 * sub-chunk may be found after earlier ones were enqueued: the call then waits for those before returning. */
int cv_merkle_tx_ids_bounded(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, uint64_t leaf_arena_bytes,
                             const uint64_t *leaf_off, const uint32_t *leaf_len, const uint32_t *tx_leaf_begin,
                             uint8_t *ids, uint8_t *tx_status, uint64_t *ticket);

/* Partial Merkle trees (FilteredTransaction / PartialMerkleTree.verify), one verdict per tree.
 * The shim flattens each PartialTree object in post-order and concatenates the trees: node k has
 * kind[k] (CV_PMT_LEAF 0 = PartialTree.Leaf, CV_PMT_INCLUDED 1 = IncludedLeaf, CV_PMT_NODE 2 = Node),
 * for a Node left[k] / right[k] = absolute indices of its children (smaller than k, inside the same
 * tree), for a leaf leaf_hash[k][32] = its SecureHash bytes; tree t is nodes
 * [tree_begin[t], tree_begin[t+1]) with its root last.  root[t][32] = merkleRootHash, the
 * hashesToCheck of tree t are check[check_begin[t] .. check_begin[t+1]).
 * verdict[t] = 1 iff hashConcat recomputation gives root[t] AND the IncludedLeaf hashes equal the
 * check hashes as a multiset (the reference's groupBy compare).  status[t] (optional) = CV_PMT_OK,
 * or CV_PMT_MALFORMED when the nodes are not a tree encoding (verdict 0; the shim throws
 * IllegalArgumentException).  FilteredTransaction.verify's empty-check MerkleTreeException stays in
 * the shim. */
#define CV_PMT_OK 0
#define CV_PMT_MALFORMED 2
int cv_partial_merkle_verify(cv_ctx *ctx, size_t ntrees, size_t nnodes, const uint8_t *kind, const uint32_t *left,
                             const uint32_t *right, const uint8_t *leaf_hash /* nnodes*32 */,
                             const uint32_t *tree_begin /* ntrees+1 */, const uint8_t *root /* ntrees*32 */,
                             size_t ncheck, const uint8_t *check /* ncheck*32 */,
                             const uint32_t *check_begin /* ntrees+1 */, uint8_t *verdict /* ntrees */,
                             uint8_t *status /* ntrees, optional */);

int cv_ed25519_sign_batch(cv_ctx *ctx, size_t n, const uint8_t *seed /* n*32 */, const uint8_t *msg_arena,
                          const uint64_t *msg_off, const uint32_t *msg_len, uint8_t *pk_out /* n*32 */,
                          uint8_t *sig_out /* n*64 */);

/* tx_ok[t] = AND of verdict bits [tx_sig_begin[t], tx_sig_begin[t+1]); a transaction with no
 * signatures is not ok (SignedTransaction requires sigs.isNotEmpty(), SignedTransaction.kt:27-29). */
int cv_tx_verdicts(size_t ntx, const uint64_t *verdict_bitmap, const uint32_t *tx_sig_begin, uint8_t *tx_ok);

/* SignedTransaction.verifySignatures over a batch in one call (SignedTransaction.kt:59-71, 83-87 with
 * WireTransaction.id, WireTransaction.kt:45-52): the ids of ntx transactions (leaves as cv_merkle_tx_ids_ex) and
 * the verify of their signatures over those ids, the ids staying on the device as the messages.  The signatures
 * of transaction t are records [tx_sig_begin[t], tx_sig_begin[t+1]) of pk[][32] / sig[][64].
 *   tx_ok[t]      = 1 iff the transaction has at least one leaf, at least one signature, and every signature
 *                   verifies over its RECOMPUTED id (cv_merkle_tx_ids_ex + cv_ed25519_verify_batch over the ids +
 *                   cv_tx_verdicts, result for result).  The caller still compares ids with the claimed
 *                   SignedTransaction.id (line 70).  The accept/reject verdict is the reference's; the exception
 *                   is settled only for tx_ok == 1 with equal ids: for any other transaction the shim re-verifies
 *                   its signatures over the CLAIMED id (cv_ed25519_verify_batch), because the reference throws
 *                   the first bad signature's SignatureException before it compares ids.
 *   ids[ntx][32], tx_status[ntx] (CV_TX_OK / CV_TX_EMPTY), sig_status[nsig] (CV_SIG_*): optional (NULL).
 * Transactions are cut into contiguous ranges over the devices as cv_merkle_tx_ids_ex's; pinned inputs are
 * DMAed in place.  _async: ticket and cv_wait as cv_ed25519_verify_batch_async. */
int cv_verify_transactions(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                           const uint32_t *leaf_len, const uint32_t *tx_leaf_begin /* ntx+1 */, const uint8_t *pk,
                           const uint8_t *sig, const uint32_t *tx_sig_begin /* ntx+1 */, uint8_t *ids,
                           uint8_t *tx_status, uint8_t *sig_status, uint8_t *tx_ok /* ntx */);
int cv_verify_transactions_async(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                                 const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, const uint8_t *pk,
                                 const uint8_t *sig, const uint32_t *tx_sig_begin, uint8_t *ids, uint8_t *tx_status,
                                 uint8_t *sig_status, uint8_t *tx_ok, uint64_t *ticket);
/* cv_verify_transactions (ticket NULL) or its _async form (ticket non-NULL) with the leaf arena's size, bounded as
 * cv_merkle_tx_ids_bounded: leaves past leaf_arena[leaf_arena_bytes) or wrapping give CV_E_ARGS before any read. */
int cv_verify_transactions_ex(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, uint64_t leaf_arena_bytes,
                              const uint64_t *leaf_off, const uint32_t *leaf_len, const uint32_t *tx_leaf_begin,
                              const uint8_t *pk, const uint8_t *sig, const uint32_t *tx_sig_begin, uint8_t *ids,
                              uint8_t *tx_status, uint8_t *sig_status, uint8_t *tx_ok, uint64_t *ticket);

/* ---------------------------------------------------------------- device-resident API
 * All pointers are device pointers on HIP device `device` (which must be in the context); work is
 * enqueued on `stream` (a hipStream_t, NULL = the context's stream for that device) and the call
 * returns without synchronising.  These are the entry points bench.py times (inputs resident in HBM).
 * A large batch may internally run part of its work on a per-device helper stream of the engine (the
 * drain overlap); `stream` waits on that work before anything the caller
 * enqueues after the call, so completion is still stream-ordered on `stream`.
 * Calls may use different streams, from any thread: the engine orders every use of a device's shared
 * verify workspace and key pool (a call on a new stream first waits for the previous call's work on
 * that workspace), so concurrent calls serialise on the device instead of racing.
 */
int cv_ed25519_verify_device(cv_ctx *ctx, int device, size_t n, const void *d_pk, const void *d_sig,
                             const void *d_arena, const void *d_off, const void *d_len, void *d_bitmap,
                             void *d_status, void *stream);

/* Measurement entry point (bench.py): as cv_ed25519_verify_device (no status), but synchronous,
 * whole-chunk launches only (no drain overlap), and fills phase_ms[0..2] with the summed durations
 * of the verify kernels measured with HIP events on the launch stream.  Half-size schedule (default),
 * batches above 32,768: scalars (challenge hash, effective S, lattice, window digits) | points
 * (decode A and R, both odd-multiple tables) | hs_straus (multi-scalar multiplication + verdict
 * bits).  Batches up to 32,768 (latency forms): scalars and point pairs in one launch | bitmap clear |
 * tri-chain (<= 4,096) or quad Straus.  Full-width schedule: prep | Straus | finish (batched
 * inversion, encode, compare, bitmap). */
int cv_ed25519_verify_device_timed(cv_ctx *ctx, int device, size_t n, const void *d_pk, const void *d_sig,
                                   const void *d_arena, const void *d_off, const void *d_len, void *d_bitmap,
                                   void *stream, float *phase_ms);

/* Keyed device-resident batch: d_keys[nkeys][32], d_key_index[n] (uint32), the rest as
 * cv_ed25519_verify_device.  The nkeys key records are copied to the host (32 B each) to resolve
 * them against the key pool; new keys' tables are computed on `stream` before the verify.  Keyed
 * calls on one device must share one stream (the pool is reused across calls in stream order).
 * phase_ms NULL: returns without synchronising; else the call is synchronous and fills
 * phase_ms[0..3] = key tables, hash, comb, finish kernel durations (HIP events). */
int cv_ed25519_verify_device_keyed(cv_ctx *ctx, int device, size_t n, size_t nkeys, const void *d_keys,
                                   const void *d_key_index, const void *d_sig, const void *d_arena, const void *d_off,
                                   const void *d_len, void *d_bitmap, void *d_status, void *stream, float *phase_ms);

int cv_ed25519_sign_device(cv_ctx *ctx, int device, size_t n, const void *d_seed, const void *d_arena,
                           const void *d_off, const void *d_len, void *d_pk, void *d_sig, void *stream);

/* d_workspace: nleaves * 32 bytes (leaf digests, overwritten) */
int cv_merkle_tx_ids_device(cv_ctx *ctx, int device, size_t ntx, size_t nleaves, const void *d_arena,
                            const void *d_leaf_off, const void *d_leaf_len, const void *d_tx_leaf_begin,
                            void *d_workspace, void *d_ids, void *d_tx_status, void *stream);

/* Block until all work the context enqueued on `device` has finished. */
int cv_synchronize(cv_ctx *ctx, int device);

/* ---------------------------------------------------------------- roofline calibration
 * Measures, on `device`, the chip-wide issue rate of the 32x32->64 multiply-accumulate
 * (v_mad_u64_u32) the field arithmetic is built on, and the practical GF(2^255-19) multiply rate of
 * the engine's fe_mul.  Either output pointer may be NULL.  Used by bench.py for roofline.peak.
 */
int cv_calibrate(cv_ctx *ctx, int device, double *mad_per_s, double *femul_per_s);

/* The same multiply-accumulate peak on a cycle basis: out[5] = {MAC/s, shader clock in GHz read
 * in-kernel (s_memtime over s_memrealtime), cycles per v_mad_u64_u32 wave-instruction per SIMD,
 * SIMD count, MAC/s ceiling at the 2.4 GHz peak clock for that cycle count}. */
int cv_calibrate_cycles(cv_ctx *ctx, int device, double *out);

/* ---------------------------------------------------------------- options
 * Per-context tuning, read at the start of every call (cv_set_option from any thread; a call in progress
 * keeps the values it started with).  Defaults are the measured best on MI355X; the kernel-form
 * thresholds also let tests force each form on any batch size.  CV_E_ARGS for an unknown option or a value
 * out of range. */
#define CV_OPT_TRI_MAX 1            /* batches up to this many signatures: tri-chain latency kernels (4096; 0 = never) */
#define CV_OPT_QUAD_MAX 2           /* up to this: quad latency kernels (32768; 0 = never); above: throughput kernels */
#define CV_OPT_DRAIN_SPLIT 3        /* throughput chunks' drain overlap: 0 off, 1 auto (default), 2 always */
#define CV_OPT_DRAIN_SPLIT_PCT 4    /* the overlapped tail's share of a split chunk, percent (10) */
#define CV_OPT_PIPE_MIN 5           /* host batches (per device) above this are pipelined (131072) */
#define CV_OPT_PIPE_FIRST 6         /* first sub-chunk of a synchronous pipelined call (32768; sizes then double) */
#define CV_OPT_PIPE_CHUNK 7         /* largest sub-chunk of a synchronous pipelined call (262144); a call of n records
                                       uses about n / 16 per sub-chunk, at least 2 x CV_OPT_PIPE_FIRST */
#define CV_OPT_ASYNC_CHUNK 8        /* sub-chunk unit of the asynchronous calls: 1 or 2 of them per launch group, the
                                       multiple nearest n / 16 (196608 = one round of resident verify waves) */
#define CV_OPT_HOST_THREADS 9       /* host threads per device packing pageable inputs / deduping keys (8) */
#define CV_OPT_SMALL_ZERO_COPY 10   /* tri-form host batches: 0 DMA, 1 zero-copy reads, 2 gather kernel, 3 auto (default) */
#define CV_OPT_SMALL_DIRECT_MIN 11  /* unpipelined batches from pinned inputs DMA them in place from this size (16384) */
#define CV_OPT_AUTO_KEYED 12        /* host dedupe + keyed path for repeated keys: 1 on (default), 0 off */
#define CV_OPT_SHARD_MIN 13         /* routing: batches up to this go whole to one device; fewer per shard never (4096) */
#define CV_OPT_SPREAD_MIN 14        /* routing: batches from this size are cut over all devices (262144) */
#define CV_OPT_MERKLE_CHUNK 15      /* leaves per Merkle pipeline sub-chunk (262144) */
#define CV_OPT_PREP_OVERLAP_MIN 16  /* unpipelined host batches from this size send keys and signatures first and
                                       decode their points on a helper stream while the rest of their inputs is still
                                       in DMA (32768) */
#define CV_OPT_TIMELINE 17          /* diagnostics: 1 = time each synchronous pipelined call on the GPU (HIP events per
                                       sub-chunk, read back as CV_STATS_TIMELINE); 0 off (default) */
#define CV_OPT_PIPE_SPLIT 18        /* synchronous pipelined calls: about n / this records per sub-chunk after the ramp,
                                       clamped to [2 x CV_OPT_PIPE_FIRST, CV_OPT_PIPE_CHUNK] (16) */
#define CV_OPT_PIPE_OVERLAP_FIRST 19 /* synchronous pipelined calls: the first sub-chunk's keys and signatures go first and
                                       its point decodes start as soon as they land: 1 on, 0 off (default: measured
                                       neutral — the ramp shortens, the call does not) */
#define CV_OPT_MID_PIECES 20        /* unpipelined mid-size batches from pageable inputs: packed and DMAed in up to this
                                       many pieces (about 1 MB of keys + signatures each), the DMA of one piece beside
                                       the packing of the next (1 = one DMA per part, the default: measured neutral to
                                       slower at 65,536) */
#define CV_OPT_PIPE_SLOTS 21        /* compute streams (workspace slots) a pipelined verify call deals its sub-chunks over
                                       (2; 3 or 4 allowed) */
#define CV_OPT_TXS_MERKLE_STREAM 22 /* cv_verify_transactions: the stream its Merkle groups run on — 0 the compute streams
                                       beside the signature groups, 1 the copy stream behind their leaves, 2 a stream
                                       of their own (default) */
#define CV_OPT_COUNT 23
int cv_set_option(cv_ctx *ctx, int option, int64_t value);
int cv_get_option(cv_ctx *ctx, int option, int64_t *value);

/* Diagnostics (no reference counterpart): the context's counters since the last reset; returns the number
 * of values of that kind (fills at most nout of them), or CV_E_ARGS.
 *   CV_STATS_PIPE  {plan, pack, wait, enqueue, sync seconds of the pipelined host path; calls; sub-chunks;
 *                   sub-chunks DMAed in place from pinned inputs}
 *   CV_STATS_SMALL {setup, pack (+ input DMA issue), launch, sync, assemble seconds of the unpipelined host path
 *                   (notary-sized batches: zero-copy and one-DMA forms); calls}
 *   CV_STATS_ROUTE {calls, routed whole to one device, cut over several, shards, keyed shards, keyed
 *                   sub-chunks, Merkle calls, Merkle sub-chunks}
 *   CV_STATS_TIMELINE {sums over the synchronous pipelined calls (cv_ed25519_verify_batch, cv_verify_transactions)
 *                   timed with CV_OPT_TIMELINE = 1, in ms from each call's first input DMA: first kernel start (the
 *                   ramp), last input DMA end, last kernel end (the span), kernel-busy time (union over the launch
 *                   groups), idle gaps between the first kernel start and the span's end, the tail after the last DMA,
 *                   the result copy (host-timed); first sub-chunk records; Merkle-group busy, verify-group busy, last
 *                   Merkle DMA end (ms; cv_verify_transactions); launch groups; host time from the call's entry to
 *                   its first input DMA enqueued (verify calls) and from the GPU work joined to the results in the
 *                   caller's arrays (ms); calls timed} */
#define CV_STATS_PIPE 0
#define CV_STATS_SMALL 1
#define CV_STATS_ROUTE 2
#define CV_STATS_TIMELINE 3
int cv_diag_stats(cv_ctx *ctx, int which, double *out, size_t nout, int reset);

/* max(msg_off[i] + msg_len[i]) over n records (0 for n = 0): the arena bytes a batch reaches, for the
 * shim's bounds check before a call (multi-threaded above 2^20 records).  Host only. */
uint64_t cv_msg_extent(size_t n, const uint64_t *msg_off, const uint32_t *msg_len);

/* Diagnostics: the host-side key dedupe cv_ed25519_verify_batch runs before choosing the keyed path
 * (seeded hash of all 32 key bytes).  Returns 1 and fills key_index[n] / *nkeys (distinct keys in
 * first-seen order) when the batch repeats keys enough for the keyed path (n >= 64, at least eight
 * signatures per distinct key), else 0.  Above 4,096 signatures a sample of 4 sqrt(n) (512 .. 4,096) at
 * pseudo-random positions first estimates the repetition (birthday count) and a batch estimated below four
 * signatures per key is taken as distinct-keyed without hashing the rest.  Host only: needs no device and no
 * context. */
int cv_diag_dedupe_keys(size_t n, const uint8_t *pk, uint32_t *key_index, size_t *nkeys);

#ifdef __cplusplus
}
#endif
#endif /* CORDAVERIFY_H */
