// cv_verify.h — the per-lane verify / sign / Merkle procedures, written once as __host__ __device__
// code: the GPU kernels (cv_kernels.hip) run them one record per lane, and the CPU test harness
// (tests/host_harness.cpp) runs the very same code on the host to debug the kernel logic without a
// GPU.  The harness is test infrastructure; the product path is the GPU kernel.
#pragma once
#include "cv_field.h"
#include "cv_group.h"
#include "cv_scalar.h"
#include "cv_sha.h"
#include "cv_tables.h"

// k*B for a signed digit k in [-128, 128] from the precomp table (LDS on the GPU)
CV_HD void btab_select(ge_precomp &r, const int32_t *btab, int k) {
    const int m = k < 0 ? -k : k;
    const int4 *row = reinterpret_cast<const int4 *>(btab + m * CV_BTAB_STRIDE);
    int32_t t[32];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const int4 v = row[q];
        t[4 * q] = v.x; t[4 * q + 1] = v.y; t[4 * q + 2] = v.z; t[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 10; i++) {
        r.yplusx.v[i] = t[i];
        r.yminusx.v[i] = t[10 + i];
        r.xy2d.v[i] = t[20 + i];
    }
    ge_precomp_cneg(r, k < 0);
}

// [k]B for a scalar k < 2^255: signed radix-256 digits from the table, 32 madds + 248 doublings.
__host__ __device__ inline void ge_scalarmult_base(ge_p3 &R, const uint32_t k[8], const int32_t *btab) {
    ge_p3_identity(R);
    ge_p1p1 t;
    ge_p2 q;
    for (int j = 31; j >= 0; j--) {
        if (j != 31) {
            ge_p3_to_p2(q, R);
#pragma unroll 1
            for (int d = 0; d < 7; d++) {
                ge_p2_dbl(t, q);
                ge_p1p1_to_p2(q, t);
            }
            ge_p2_dbl(t, q);
            ge_p1p1_to_p3(R, t);
        }
        ge_precomp e;
        btab_select(e, btab, digit256(k, j));
        ge_madd(t, R, e);
        ge_p1p1_to_p3(R, t);
    }
}

CV_HD void ge_p3_encode(uint32_t w[8], const ge_p3 &p) {
    ge_p2 q;
    ge_p3_to_p2(q, p);
    ge_p2_encode(w, q);
}

// ---------------------------------------------------------------- verify one signature
// eddsa-0.1.0 EdDSAEngine.verify for one record (see cv_kernels.hip header for the schedule).
// aw = public key words, rw / sw = R / S words (all 8 LE uint32), msg = message bytes.
// Returns the verdict; *key_ok = false where the reference cannot even build the key.
__host__ __device__ inline bool cv_verify_one(const int32_t *btab, const uint32_t aw[8], const uint32_t rw[8],
                                              const uint32_t sw[8], const uint8_t *msg, uint32_t mlen,
                                              bool *key_ok_out) {
    // ---- key decode + canonical re-encoding (EdDSAPublicKey.Abyte)
    ge_p3 A;
    const bool key_ok = ge_decode_0_1_0(A, aw);
    uint32_t abyte[8];
    {
        uint32_t xw[8];
        fe_to_words(abyte, A.Y);
        fe_to_words(xw, A.X);
        abyte[7] |= (xw[0] & 1u) << 31;
    }
    // ---- h = SHA-512(R || Abyte || M) mod L
    uint32_t h[8];
    {
        uint32_t pre[16], dig[16];
#pragma unroll
        for (int q = 0; q < 8; q++) { pre[q] = rw[q]; pre[8 + q] = abyte[q]; }
        sha512_pre_msg(dig, pre, 64, msg, mlen);
        sc_reduce512(h, dig);
    }
    // ---- effective S (slide carry loss) reduced mod L
    uint32_t s[8];
    sc_effective_s(s, sw);

    // ---- per-lane table: atab[k] = k * (-A), k = 0..8 (cached form)
    ge_cached atab[9];
    {
        ge_p3 nA, P;
        fe_neg(nA.X, A.X);
        nA.Y = A.Y;
        nA.Z = A.Z;
        fe_neg(nA.T, A.T);
        ge_cached_identity(atab[0]);
        ge_p3_to_cached(atab[1], nA);
        ge_p1p1 t;
        ge_p3_dbl(t, nA);
        ge_p1p1_to_p3(P, t);
        ge_p3_to_cached(atab[2], P);
#pragma unroll 1
        for (int k = 3; k <= 8; k++) {
            ge_add(t, P, atab[1]);
            ge_p1p1_to_p3(P, t);
            ge_p3_to_cached(atab[k], P);
        }
    }

    // ---- joint Straus: R' = sum_w 16^w (a_w * (-A) + [w even] b_{w/2} * B)
    ge_p3 R;
    ge_p3_identity(R);
#pragma unroll 1
    for (int w = 63; w >= 0; w--) {
        ge_p1p1 t;
        if (w != 63) {
            ge_p2 q;
            ge_p3_to_p2(q, R);
            ge_p2_dbl(t, q);
            ge_p1p1_to_p2(q, t);
            ge_p2_dbl(t, q);
            ge_p1p1_to_p2(q, t);
            ge_p2_dbl(t, q);
            ge_p1p1_to_p2(q, t);
            ge_p2_dbl(t, q);
            ge_p1p1_to_p3(R, t);
        }
        {
            const int a = digit16(h, w);
            ge_cached e = atab[a < 0 ? -a : a];
            ge_cached_cneg(e, a < 0);
            ge_add(t, R, e);
            ge_p1p1_to_p3(R, t);
        }
        if ((w & 1) == 0) {
            ge_precomp e;
            btab_select(e, btab, digit256(s, w >> 1));
            ge_madd(t, R, e);
            ge_p1p1_to_p3(R, t);
        }
    }

    // ---- encode R' and byte-compare with the signature's R
    uint32_t enc[8];
    ge_p3_encode(enc, R);
    uint32_t diff = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) diff |= enc[q] ^ rw[q];
    *key_ok_out = key_ok;
    return key_ok && diff == 0;
}

// ---------------------------------------------------------------- keygen + sign one message
// EdDSAPrivateKeySpec(seed) + EdDSAEngine.sign (RFC 8032): pk = [a]B, R = [r]B, S = r + k a.
__host__ __device__ inline void cv_sign_one(const int32_t *btab, const uint32_t seed[8], const uint8_t *msg,
                                            uint32_t mlen, uint32_t pk_out[8], uint32_t sig_out[16]) {
    uint32_t sd[16], hd[16];
#pragma unroll
    for (int q = 0; q < 8; q++) { sd[q] = seed[q]; sd[8 + q] = 0; }
    sha512_pre_msg(hd, sd, 32, msg, 0);               // h = SHA-512(seed)
    uint32_t a[8], prefix[16];
#pragma unroll
    for (int q = 0; q < 8; q++) { a[q] = hd[q]; prefix[q] = hd[8 + q]; prefix[8 + q] = 0; }
    a[0] &= 0xfffffff8u;                               // clamp: h[0] &= 248
    a[7] &= 0x3fffffffu;                               //        h[31] &= 63
    a[7] |= 0x40000000u;                               //        h[31] |= 64
    ge_p3 A;
    ge_scalarmult_base(A, a, btab);
    uint32_t abyte[8];
    ge_p3_encode(abyte, A);
    uint32_t r[8], rd[16];
    sha512_pre_msg(rd, prefix, 32, msg, mlen);         // r = SHA-512(prefix || M) mod L
    sc_reduce512(r, rd);
    ge_p3 Rp;
    ge_scalarmult_base(Rp, r, btab);
    uint32_t rb[8];
    ge_p3_encode(rb, Rp);
    uint32_t pre[16], kd[16], k[8], S[8];
#pragma unroll
    for (int q = 0; q < 8; q++) { pre[q] = rb[q]; pre[8 + q] = abyte[q]; }
    sha512_pre_msg(kd, pre, 64, msg, mlen);            // k = SHA-512(R || A || M) mod L
    sc_reduce512(k, kd);
    sc_muladd(S, k, a, r);                             // S = (r + k a) mod L
#pragma unroll
    for (int q = 0; q < 8; q++) { pk_out[q] = abyte[q]; sig_out[q] = rb[q]; sig_out[8 + q] = S[q]; }
}

// ---------------------------------------------------------------- Merkle root of one transaction
// MerkleTree.buildMerkleTree over cnt leaf digests (8 big-endian words each), in place.
// Returns false for an empty leaf list (MerkleTreeException).  root = 8 big-endian words.
__host__ __device__ inline bool cv_merkle_root_inplace(uint32_t *lvl, uint32_t cnt, uint32_t root[8]) {
    if (cnt == 0) {
#pragma unroll
        for (int q = 0; q < 8; q++) root[q] = 0;
        return false;
    }
    while (cnt > 1) {
        const uint32_t m = (cnt + 1) >> 1;
        for (uint32_t j = 0; j < m; j++) {
            uint32_t l[8], r[8], o[8];
            const uint32_t li = 2 * j, ri = (2 * j + 1 < cnt) ? 2 * j + 1 : cnt - 1;
#pragma unroll
            for (int q = 0; q < 8; q++) { l[q] = lvl[li * 8 + q]; r[q] = lvl[ri * 8 + q]; }
            sha256_node(o, l, r);
#pragma unroll
            for (int q = 0; q < 8; q++) lvl[j * 8 + q] = o[q];
        }
        cnt = m;
    }
#pragma unroll
    for (int q = 0; q < 8; q++) root[q] = lvl[q];
    return true;
}
