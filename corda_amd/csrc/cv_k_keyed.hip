// cv_k_keyed.hip — the keyed per-key comb path: key tables, hash + scalar, comb, and the
// finish kernel (batched inversion, encode, byte compare, bitmap bytes).
// Shared helpers and every kernel declaration: cv_kcommon.h; launchers: cv_kernels.hip.
#include "cv_kcommon.h"

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

// ---------------------------------------------------------------- keyed verify (per-key comb, f2)
// key precompute: one lane per key (decode + 4 comb row tables of 8 cached multiples) into its slot
__global__ __launch_bounds__(CV_BLOCK) void cv_keyprep_kernel(uint32_t nk, const uint8_t *__restrict__ keys,
                                                              const uint32_t *__restrict__ slots,
                                                              uint32_t *__restrict__ scratch,
                                                              uint32_t *__restrict__ ktab_pool,
                                                              uint8_t *__restrict__ kok_pool) {
    // CV_COMB_ROWS consecutive lanes per key, one comb row each (129 entries)
    const uint32_t g = blockIdx.x * CV_BLOCK + threadIdx.x;
    const uint32_t i = g / CV_COMB_ROWS;
    if (i >= nk) return;
    const int j = (int)(g % CV_COMB_ROWS);
    uint32_t aw[8];
    load_words8(aw, keys + (size_t)i * 32);
    const uint32_t slot = slots[i];
    const bool ok = cv_key_prep_row(aw, j, scratch + (size_t)i * CV_KTAB_WORDS, ktab_pool + (size_t)slot * CV_KTAB_WORDS);
    if (j == 0) kok_pool[slot] = ok ? 1 : 0;
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
// The lane's h || s record: s is replaced by its radix-2^16 digit pairs first (the record is this lane's own; the
// finish kernel does not read it), then the comb reads both from it each window (cv_comb_straus_rec).
template <int WAVES>
__global__ __launch_bounds__(CV_BLOCK, WAVES) void cv_comb_kernel(uint32_t n, uint32_t *__restrict__ ws_hs,
                                                                  const uint32_t *__restrict__ key_index,
                                                                  const uint32_t *__restrict__ slot_of_key,
                                                                  const uint32_t *__restrict__ ktab_pool,
                                                                  uint32_t *__restrict__ ws_R,
                                                                  const uint32_t *__restrict__ bw16) {
    const uint32_t i = blockIdx.x * CV_BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t slot = slot_of_key[key_index[i]];
    uint32_t *rec = ws_hs + (size_t)i * CV_HS_WORDS;
    {
        uint32_t s[8], sd[8];
        load_words8(s, reinterpret_cast<const uint8_t *>(rec + 8));
        digits65536_pairs(sd, s);
        store_words(rec + 8, sd, 2);
    }
    ge_p2 R;
    // s * B from the radix-2^16 rows (16 madds instead of 32)
    cv_comb_straus_rec(bw16, rec, ktab_pool + (size_t)slot * CV_KTAB_WORDS, R);
    uint32_t out[CV_R_WORDS];
    fe_store(out, R.X);
    fe_store(out + 10, R.Y);
    fe_store(out + 20, R.Z);
    out[30] = out[31] = 0;
    store_words(ws_R + (size_t)i * CV_R_WORDS, out, CV_R_WORDS / 4);
}
template __global__ void cv_comb_kernel<3>(uint32_t, uint32_t *, const uint32_t *, const uint32_t *,
                                           const uint32_t *, uint32_t *, const uint32_t *);
template __global__ void cv_finish_kernel<false>(uint32_t n, uint32_t nbytes, const uint8_t *sig, const uint32_t *ws_R, const uint8_t *ws_ok, uint8_t *bitmap_bytes);
