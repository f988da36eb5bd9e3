// cv_sha.h — SHA-512 (Ed25519 challenge hash) and SHA-256 (Merkle leaves / nodes) for one lane.
//
// Each lane hashes its own record; the message bytes are read from the device arena with byte
// loads (records are variable length and unaligned — the reads are a rounding error next to the
// ~2.4e5 multiply-accumulates of a verify, see DESIGN.md roofline).
#pragma once
#include "cv_field.h"

#define CV_K512_INIT { \
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, \
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, \
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, \
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL, \
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL, \
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, \
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, \
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, \
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL, \
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL, \
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, \
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, \
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, \
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL, \
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL, \
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, \
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, \
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL, \
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL, \
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL}
__device__ __constant__ static const uint64_t CV_K512_D[80] = CV_K512_INIT;
static const uint64_t CV_K512_H[80] = CV_K512_INIT;

#define CV_K256_INIT { \
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, \
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, \
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, \
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, \
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, \
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, \
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3, \
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2}
__device__ __constant__ static const uint32_t CV_K256_D[64] = CV_K256_INIT;
static const uint32_t CV_K256_H[64] = CV_K256_INIT;

// Round constants: the __constant__ copy on the GPU, the host copy when the same code runs in the
// CPU test harness (tests/host_harness.cpp).
CV_HD uint64_t cv_k512(int i) {
#ifdef __HIP_DEVICE_COMPILE__
    return CV_K512_D[i];
#else
    return CV_K512_H[i];
#endif
}
CV_HD uint32_t cv_k256(int i) {
#ifdef __HIP_DEVICE_COMPILE__
    return CV_K256_D[i];
#else
    return CV_K256_H[i];
#endif
}

// 64-bit rotate right by a constant: two v_alignbit_b32 on the GPU (the generic shift/or form
// compiles to two 64-bit shifts and two ors).
template <int N> CV_HD uint64_t cv_rotr64(uint64_t x) {
    static_assert(N > 0 && N < 64, "rotate count");
#ifdef __HIP_DEVICE_COMPILE__
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if constexpr (N < 32) {
        return ((uint64_t)__builtin_amdgcn_alignbit(lo, hi, N) << 32) | __builtin_amdgcn_alignbit(hi, lo, N);
    } else if constexpr (N == 32) {
        return ((uint64_t)lo << 32) | hi;
    } else {
        return ((uint64_t)__builtin_amdgcn_alignbit(hi, lo, N - 32) << 32) | __builtin_amdgcn_alignbit(lo, hi, N - 32);
    }
#else
    return (x >> N) | (x << (64 - N));
#endif
}
CV_HD uint64_t cv_ror64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
// low 32 bits of (hi:lo) >> sh, sh < 32 (v_alignbit_b32; a 64-bit shift of two array words would make
// the compiler keep the array in scratch for an unaligned 8-byte load)
CV_HD uint32_t cv_funnel32(uint32_t hi, uint32_t lo, uint32_t sh) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh);
#endif
}
CV_HD uint32_t cv_ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
// Three-input bitwise functions in one v_bitop3_b32 per 32 bits (truth table indexed by
// S0<<2 | S1<<1 | S2): xor3 0x96, choose (x ? y : z) 0xCA, majority 0xE8.  The compiler emits two or
// three two-input ops for each otherwise (and does not fuse the 64-bit forms at all).
template <int TT> CV_HD uint32_t cv_bitop3(uint32_t a, uint32_t b, uint32_t c) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
#else
    return TT == 0x96 ? a ^ b ^ c : TT == 0xCA ? (a & b) | (~a & c) : (a & b) | (a & c) | (b & c);
#endif
}
CV_HD uint32_t cv_xor3(uint32_t a, uint32_t b, uint32_t c) { return cv_bitop3<0x96>(a, b, c); }
template <int TT> CV_HD uint64_t cv_bitop3_64(uint64_t a, uint64_t b, uint64_t c) {
    return (uint64_t)cv_bitop3<TT>((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32 |
           cv_bitop3<TT>((uint32_t)a, (uint32_t)b, (uint32_t)c);
}
CV_HD uint32_t cv_bswap32(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

CV_HD void sha512_init(uint64_t st[8]) {
    st[0] = 0x6a09e667f3bcc908ULL; st[1] = 0xbb67ae8584caa73bULL;
    st[2] = 0x3c6ef372fe94f82bULL; st[3] = 0xa54ff53a5f1d36f1ULL;
    st[4] = 0x510e527fade682d1ULL; st[5] = 0x9b05688c2b3e6c1fULL;
    st[6] = 0x1f83d9abfb41bd6bULL; st[7] = 0x5be0cd19137e2179ULL;
}

// One compression; w[16] = big-endian message words (clobbered: used as the schedule ring).
// Written so every index is a compile-time constant: rounds 0-15 straight from w, then four passes
// of 16 rounds that extend the schedule in place (w[j] for round 16 p + j), the eight working
// variables rotated by renaming in the round macro rather than by moves.  (A single loop over i with
// w[i & 15] compiled to indirect register indexing and a branch per round.)
#define CV_S512_BSIG0(x) (cv_rotr64<28>(x) ^ cv_rotr64<34>(x) ^ cv_rotr64<39>(x))
#define CV_S512_BSIG1(x) (cv_rotr64<14>(x) ^ cv_rotr64<18>(x) ^ cv_rotr64<41>(x))
#define CV_S512_SSIG0(x) (cv_rotr64<1>(x) ^ cv_rotr64<8>(x) ^ ((x) >> 7))
#define CV_S512_SSIG1(x) (cv_rotr64<19>(x) ^ cv_rotr64<61>(x) ^ ((x) >> 6))
#define CV_S512_ROUND(a, b, c, d, e, f, g, h, kw)                                                     \
    {                                                                                             \
        const uint64_t t1_ = (h) + CV_S512_BSIG1(e) + cv_bitop3_64<0xCA>((e), (f), (g)) + (kw);      \
        const uint64_t t2_ = CV_S512_BSIG0(a) + cv_bitop3_64<0xE8>((a), (b), (c));                  \
        (d) += t1_;                                                                               \
        (h) = t1_ + t2_;                                                                          \
    }
#define CV_S512_8ROUNDS(base, W)                                                                  \
    CV_S512_ROUND(a, b, c, d, e, f, g, h, cv_k512((base) + 0) + W(0))                             \
    CV_S512_ROUND(h, a, b, c, d, e, f, g, cv_k512((base) + 1) + W(1))                             \
    CV_S512_ROUND(g, h, a, b, c, d, e, f, cv_k512((base) + 2) + W(2))                             \
    CV_S512_ROUND(f, g, h, a, b, c, d, e, cv_k512((base) + 3) + W(3))                             \
    CV_S512_ROUND(e, f, g, h, a, b, c, d, cv_k512((base) + 4) + W(4))                             \
    CV_S512_ROUND(d, e, f, g, h, a, b, c, cv_k512((base) + 5) + W(5))                             \
    CV_S512_ROUND(c, d, e, f, g, h, a, b, cv_k512((base) + 6) + W(6))                             \
    CV_S512_ROUND(b, c, d, e, f, g, h, a, cv_k512((base) + 7) + W(7))

__host__ __device__ __forceinline__ void sha512_compress(uint64_t st[8], uint64_t w[16]) {
    uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#define CV_W_LO(j) w[(j)]
#define CV_W_HI(j) w[8 + (j)]
    CV_S512_8ROUNDS(0, CV_W_LO)
    CV_S512_8ROUNDS(8, CV_W_HI)
#pragma unroll 1
    for (int p = 1; p < 5; p++) {
#pragma unroll
        for (int j = 0; j < 16; j++)
            w[j] += CV_S512_SSIG0(w[(j + 1) & 15]) + w[(j + 9) & 15] + CV_S512_SSIG1(w[(j + 14) & 15]);
        CV_S512_8ROUNDS(16 * p, CV_W_LO)
        CV_S512_8ROUNDS(16 * p + 8, CV_W_HI)
    }
#undef CV_W_LO
#undef CV_W_HI
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Little-endian dword of message bytes [t, t+4) (t a multiple of 4 relative to the message start),
// with bytes past mlen replaced by the SHA padding (0x80 at mlen, zeros after).  Reads are aligned
// dwords, and only dwords that contain at least one message byte are touched, so an unaligned
// message ending at the very end of an allocation never reads past it.
CV_HD uint32_t msg_dword_le(const uint8_t *msg, uint32_t mlen, uint32_t t) {
    if (t > mlen) return 0;
    const uintptr_t a = (uintptr_t)(msg + t);
    const uint32_t sh = (uint32_t)(a & 3u);
    const uint32_t *p = reinterpret_cast<const uint32_t *>(a - sh);
    const uint32_t lo = t < mlen ? p[0] : 0u;
    const uint32_t hi = (sh != 0u && t + 4 - sh < mlen) ? p[1] : 0u;
    uint32_t v = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh));
    if (t + 4 > mlen) {
        const uint32_t valid = mlen - t;                      // 0..3 bytes of message left
        v = (v & ((1u << (8 * valid)) - 1u)) | (0x80u << (8 * valid));
    }
    return v;
}

// The message dwords one SHA-512 block needs: dw[k] = aligned dword at floor4(msg + tstart) + 4k,
// k < 33 (any 128 message bytes lie in 33 aligned dwords).  Only dwords holding at least one message
// byte are read — dwords past the last one repeat it (their value is discarded by the padding rule
// of the caller) — and a lane with no message byte in the window reads nothing, so a message that
// ends at the very end of an allocation is never read past (the same guarantee as msg_dword_le).
// One branch per block instead of two conditional loads per dword.
template <int K>
CV_HD void cv_msg_window(uint32_t dw[K], const uint8_t *msg, uint32_t mlen, uint32_t tstart) {
    const uint32_t sh = (uint32_t)((uintptr_t)msg & 3u);              // tstart is a multiple of 4
    const uint32_t rem = mlen > tstart ? mlen - tstart + sh : 0u;     // message bytes from the window base
    const uint32_t kmax = rem >= 4u * K ? (uint32_t)K : (rem + 3) >> 2; // dwords holding message bytes
#pragma unroll
    for (int k = 0; k < K; k++) dw[k] = 0;
    if (kmax > 0) {
        const uint32_t *p = reinterpret_cast<const uint32_t *>(msg + tstart - sh);
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint32_t kk = (uint32_t)k < kmax ? (uint32_t)k : kmax - 1;
            dw[k] = p[kk];
        }
    }
}
CV_HD void sha512_msg_window(uint32_t dw[33], const uint8_t *msg, uint32_t mlen, uint32_t tstart) {
    cv_msg_window<33>(dw, msg, mlen, tstart);
}

// The 16 schedule words of SHA-512 block `blk` of pre[0:NPRE] || msg[0:mlen] || padding || length.
// Message dword at offset t (a multiple of 4) = bytes msg[t..t+4) little-endian, funnel-shifted out
// of the block's aligned window (Q0 = first window dword of the block: NPRE/4 in block 0, else 0,
// a compile-time constant so the window stays in registers); bytes past mlen are the SHA padding
// (0x80, zeros) — msg_dword_le's rules, applied branch-free.
template <int NPRE, bool FIRST>
CV_HD void sha512_block_words(uint64_t w[16], const uint32_t pre[16], const uint8_t *msg, uint32_t mlen, uint32_t blk,
                              uint32_t total, uint64_t bits) {
    const uint32_t tstart = FIRST ? 0u : blk * 128 - NPRE;
    uint32_t dw[33];
    sha512_msg_window(dw, msg, mlen, tstart);
    const uint32_t sh8 = 8u * (uint32_t)((uintptr_t)msg & 3u);
#pragma unroll
    for (int j = 0; j < 16; j++) {
        uint32_t d[2];
#pragma unroll
        for (int hl = 0; hl < 2; hl++) {
            const int jj = 2 * j + hl;                              // dword of the block
            const uint32_t u = blk * 128 + 4 * jj;                  // stream offset of this dword
            uint32_t le;
            if (FIRST && jj < NPRE / 4) {
                le = pre[jj];
            } else {
                const int q = FIRST ? jj - NPRE / 4 : jj;           // window dword (constant)
                const uint32_t t = u - NPRE;                        // message offset
                le = cv_funnel32(dw[q + 1], dw[q], sh8);
                const uint32_t valid = mlen - t;                    // message bytes left at t
                const uint32_t keep = valid >= 4 ? 0xffffffffu : ((1u << (8 * (valid & 3u))) - 1u);
                const uint32_t pad = valid >= 4 ? 0u : (0x80u << (8 * (valid & 3u)));
                le = (le & keep) | pad;
                if (t > mlen) le = 0;
            }
            d[hl] = cv_bswap32(le);
            if (u >= total - 8) d[hl] = (uint32_t)(bits >> (hl ? 0 : 32));
        }
        w[j] = ((uint64_t)d[0] << 32) | d[1];
    }
}

// SHA-512(pre[0:NPRE] || msg[0:mlen]) with NPRE in {32, 64} (pre as LE words); out = 16 LE words
// of the 64-byte digest (byte order as produced by the hash, i.e. digest byte k = out[k/4] >> 8(k%4)).
template <int NPRE>
__host__ __device__ __forceinline__ void sha512_pre_msg_t(uint32_t out[16], const uint32_t pre[16], const uint8_t *msg,
                                                          uint32_t mlen) {
    uint64_t st[8];
    sha512_init(st);
    const uint32_t data = NPRE + mlen;
    const uint32_t nblocks = (data + 1 + 16 + 127) / 128;
    const uint32_t total = nblocks * 128;
    const uint64_t bits = (uint64_t)data * 8;
    {
        uint64_t w[16];
        sha512_block_words<NPRE, true>(w, pre, msg, mlen, 0, total, bits);
        sha512_compress(st, w);
    }
#pragma nounroll
    for (uint32_t blk = 1; blk < nblocks; blk++) {
        uint64_t w[16];
        sha512_block_words<NPRE, false>(w, pre, msg, mlen, blk, total, bits);
        sha512_compress(st, w);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        out[2 * i] = cv_bswap32((uint32_t)(st[i] >> 32));
        out[2 * i + 1] = cv_bswap32((uint32_t)st[i]);
    }
}
__host__ __device__ __forceinline__ void sha512_pre_msg(uint32_t out[16], const uint32_t pre[16], int npre,
                                                        const uint8_t *msg, uint32_t mlen) {
    if (npre == 32) sha512_pre_msg_t<32>(out, pre, msg, mlen);
    else sha512_pre_msg_t<64>(out, pre, msg, mlen);
}

// ---------------------------------------------------------------- SHA-256
CV_HD void sha256_init(uint32_t st[8]) {
    st[0] = 0x6a09e667; st[1] = 0xbb67ae85; st[2] = 0x3c6ef372; st[3] = 0xa54ff53a;
    st[4] = 0x510e527f; st[5] = 0x9b05688c; st[6] = 0x1f83d9ab; st[7] = 0x5be0cd19;
}

__host__ __device__ __forceinline__ void sha256_compress(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i & 15];
        } else {
            const uint32_t x15 = w[(i - 15) & 15], x2 = w[(i - 2) & 15];
            const uint32_t s0 = cv_xor3(cv_ror32(x15, 7), cv_ror32(x15, 18), x15 >> 3);
            const uint32_t s1 = cv_xor3(cv_ror32(x2, 17), cv_ror32(x2, 19), x2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
        }
        const uint32_t t1 = h + cv_xor3(cv_ror32(e, 6), cv_ror32(e, 11), cv_ror32(e, 25)) + ((e & f) ^ (~e & g)) +
                            cv_k256(i) + wi;
        const uint32_t t2 = cv_xor3(cv_ror32(a, 2), cv_ror32(a, 13), cv_ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// SHA-256 of an arbitrary byte string in device memory; out = 8 big-endian state words.
// Per 64-byte block the message comes from one window of 17 aligned dwords (cv_msg_window: one
// branch per block, nothing read past the last message byte), funnel-shifted into the 16 schedule
// words, with msg_dword_le's padding rules applied branch-free.
// The 16 schedule words of SHA-256 block `blk` of the n-byte message at p (padding and the bit
// length applied branch-free; total = the padded length in bytes).
__host__ __device__ __forceinline__ void sha256_block_words(uint32_t w[16], const uint8_t *p, uint32_t n, uint32_t blk,
                                                            uint32_t total) {
    const uint64_t bits = (uint64_t)n * 8;
    const uint32_t sh8 = 8u * (uint32_t)((uintptr_t)p & 3u);
    uint32_t dw[17];
    cv_msg_window<17>(dw, p, n, blk * 64);
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint32_t u = blk * 64 + 4 * j;
        uint32_t le = cv_funnel32(dw[j + 1], dw[j], sh8);
        const uint32_t valid = n - u;                            // message bytes left at u
        const uint32_t keep = valid >= 4 ? 0xffffffffu : ((1u << (8 * (valid & 3u))) - 1u);
        const uint32_t pad = valid >= 4 ? 0u : (0x80u << (8 * (valid & 3u)));
        le = (le & keep) | pad;
        if (u > n) le = 0;
        uint32_t v = cv_bswap32(le);
        if (u == total - 8) v = (uint32_t)(bits >> 32);
        if (u == total - 4) v = (uint32_t)bits;
        w[j] = v;
    }
}
CV_HD uint32_t sha256_nblocks(uint32_t n) { return (n + 1 + 8 + 63) / 64; }

// SHA-256 of an arbitrary byte string in device memory; out = 8 big-endian state words.
// Per 64-byte block the message comes from one window of 17 aligned dwords (cv_msg_window: one
// branch per block, nothing read past the last message byte), funnel-shifted into the 16 schedule
// words, with msg_dword_le's padding rules applied branch-free.
__host__ __device__ __forceinline__ void sha256_bytes(uint32_t out[8], const uint8_t *p, uint32_t n) {
    uint32_t st[8];
    sha256_init(st);
    const uint32_t nblocks = sha256_nblocks(n);
#pragma nounroll
    for (uint32_t blk = 0; blk < nblocks; blk++) {
        uint32_t w[16];
        sha256_block_words(w, p, n, blk, nblocks * 64);
        sha256_compress(st, w);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = st[i];
}

// SHA-256(left32 || right32) for two digests held as 8 big-endian state words each (Merkle node).
__host__ __device__ __forceinline__ void sha256_node(uint32_t out[8], const uint32_t l[8], const uint32_t r[8]) {
    uint32_t st[8], w[16];
    sha256_init(st);
#pragma unroll
    for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; }
    sha256_compress(st, w);
    // padding block for a 64-byte message
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = 0;
    w[0] = 0x80000000u;
    w[15] = 512;
    sha256_compress(st, w);
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = st[i];
}
