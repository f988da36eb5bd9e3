// cv_k_misc.hip — signing (synthetic inputs), Merkle tx ids, partial Merkle trees, calibration and probe kernels.
// Shared helpers and every kernel declaration: cv_kcommon.h; launchers: cv_kernels.hip.
#include "cv_kcommon.h"

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
// One lane per leaf PAIR.  Each workgroup takes 2 x CV_LEAF_BLOCK consecutive leaves, orders them by SHA-256
// block count (counting sort in LDS: one LDS atomic per leaf, one wave scan), then lane t hashes the t-th shortest AND the t-th longest leaf of the span back to back in one block
// loop (the state restarts between them), so every lane's block count is about the span's mean and
// a wave no longer runs as long as its longest leaf.  Span = 2 x block.
__global__ __launch_bounds__(CV_LEAF_BLOCK) void cv_leaf_hash_pair_kernel(uint32_t nleaves, const uint8_t *__restrict__ arena,
                                                                          const uint64_t *__restrict__ off,
                                                                          const uint32_t *__restrict__ len,
                                                                          uint32_t *__restrict__ leaf_digest) {
    constexpr uint32_t SPAN = 2 * CV_LEAF_BLOCK;
    __shared__ uint32_t hist[64], base[64], perm[SPAN];
    const uint32_t t = threadIdx.x, first = blockIdx.x * SPAN;
    const uint32_t nlive = nleaves - first < SPAN ? nleaves - first : SPAN;
    if (t < 64) hist[t] = 0;
    __syncthreads();
    uint32_t bucket[2], pos[2];
#pragma unroll
    for (uint32_t k = 0; k < 2; k++) {
        const uint32_t j = k * CV_LEAF_BLOCK + t;
        bucket[k] = 0;
        pos[k] = 0;
        if (j < nlive) {
            const uint32_t nb = sha256_nblocks(len[first + j]);
            bucket[k] = nb < 63u ? nb : 63u;
            pos[k] = atomicAdd(&hist[bucket[k]], 1u);
        }
    }
    __syncthreads();
    if (t < 64) {                                                 // exclusive scan, one wave
        const uint32_t own = hist[t];
        uint32_t inc = own;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d, 64);
            if ((int)t >= d) inc += y;
        }
        base[t] = inc - own;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < 2; k++) {
        const uint32_t j = k * CV_LEAF_BLOCK + t;
        if (j < nlive) perm[base[bucket[k]] + pos[k]] = first + j;
    }
    __syncthreads();
    // ranks t and nlive-1-t; the middle rank of an odd span is taken once (as A)
    const bool has_a = 2 * t + 1 <= nlive, has_b = nlive - 1 - t > t && t < nlive;
    const uint32_t la = has_a ? perm[t] : 0u, lb = has_b ? perm[nlive - 1 - t] : 0u;
    const uint32_t na = has_a ? len[la] : 0u, nbl = has_b ? len[lb] : 0u;
    const uint8_t *pa = arena + (has_a ? off[la] : 0), *pb = arena + (has_b ? off[lb] : 0);
    const uint32_t ba = has_a ? sha256_nblocks(na) : 0u, bb = has_b ? sha256_nblocks(nbl) : 0u;
    uint32_t st[8];
    sha256_init(st);
#pragma nounroll
    for (uint32_t it = 0; it < ba + bb; it++) {
        const bool in_a = it < ba;
        uint32_t w[16];
        sha256_block_words(w, in_a ? pa : pb, in_a ? na : nbl, in_a ? it : it - ba, 64 * (in_a ? ba : bb));
        sha256_compress(st, w);
        if (it + 1 == ba) {
            uint4 *o = reinterpret_cast<uint4 *>(leaf_digest + (size_t)la * 8);
            o[0] = make_uint4(st[0], st[1], st[2], st[3]);
            o[1] = make_uint4(st[4], st[5], st[6], st[7]);
            sha256_init(st);
        }
    }
    if (has_b) {
        uint4 *o = reinterpret_cast<uint4 *>(leaf_digest + (size_t)lb * 8);
        o[0] = make_uint4(st[0], st[1], st[2], st[3]);
        o[1] = make_uint4(st[4], st[5], st[6], st[7]);
    }
}

// one lane per transaction, in place over its leaf digests; ids are written as digest bytes.  tx_begin holds
// absolute leaf indices; leaf_base is the index of leaf_digest[0] (a sub-chunk of a larger batch)
__global__ __launch_bounds__(CV_BLOCK) void cv_merkle_tree_kernel(uint32_t ntx, uint32_t leaf_base,
                                                                  const uint32_t *__restrict__ tx_begin,
                                                                  uint32_t *__restrict__ leaf_digest,
                                                                  uint8_t *__restrict__ ids,
                                                                  uint8_t *__restrict__ status) {
    const uint32_t gid = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (gid >= ntx) return;
    const uint32_t b = tx_begin[gid] - leaf_base, e = tx_begin[gid + 1] - leaf_base;
    uint32_t root[8];
    const bool ok = cv_merkle_root_inplace(leaf_digest + (size_t)b * 8, e - b, root);
    uint4 *o = reinterpret_cast<uint4 *>(ids + (size_t)gid * 32);
    o[0] = make_uint4(cv_bswap32(root[0]), cv_bswap32(root[1]), cv_bswap32(root[2]), cv_bswap32(root[3]));
    o[1] = make_uint4(cv_bswap32(root[4]), cv_bswap32(root[5]), cv_bswap32(root[6]), cv_bswap32(root[7]));
    if (status) status[gid] = ok ? 0 : 1;
}

// ---------------------------------------------------------------- transactions (cv_verify_transactions)
// Message references of signatures [c0, c0 + m) of a shard whose transactions' ids sit back to back on the
// device: signature s0 + c0 + i belongs to the transaction t with tsb[t] <= s0 + c0 + i < tsb[t + 1] (the
// largest such t, so empty transactions are passed over), and its message is that id, 32 bytes at t * 32.
// tsb: the shard's nt + 1 absolute signature boundaries (tsb[0] = s0).
__global__ __launch_bounds__(CV_BLOCK) void cv_tx_sig_refs_kernel(uint32_t m, uint32_t c0, uint32_t nt, uint32_t s0,
                                                                  const uint32_t *__restrict__ tsb,
                                                                  uint64_t *__restrict__ off, uint32_t *__restrict__ len) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i >= m) return;
    off[c0 + i] = (uint64_t)cv_tx_of_sig(s0 + c0 + i, nt, tsb) * 32;
    len[c0 + i] = 32;
}

// verifySignatures' verdict per transaction: its id was computed (at least one leaf) and it has at least one
// signature, all valid.  bitmap: the shard's verdicts, bit j = signature s0 + j.
__global__ __launch_bounds__(CV_BLOCK) void cv_tx_verdict_kernel(uint32_t nt, uint32_t s0, const uint32_t *__restrict__ tsb,
                                                                 const uint8_t *__restrict__ mstatus,
                                                                 const uint64_t *__restrict__ bitmap,
                                                                 uint8_t *__restrict__ tx_ok) {
    const uint32_t t = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (t >= nt) return;
    tx_ok[t] = mstatus[t] == 0 && cv_tx_all_valid(tsb[t] - s0, tsb[t + 1] - s0, bitmap) ? 1 : 0;
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
