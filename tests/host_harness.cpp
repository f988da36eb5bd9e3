// host_harness.cpp — TEST INFRASTRUCTURE: runs the product's per-lane device code (corda_amd/csrc/
// cv_verify.h and friends, all __host__ __device__) on the CPU so its logic can be checked against
// the oracle without a GPU.  Built by tests/conftest.py into tests/_build/libcvhost.so.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../corda_amd/csrc/cv_verify.h"

static void words_from_bytes(uint32_t *w, const uint8_t *b, int nwords) {
    for (int i = 0; i < nwords; i++) memcpy(&w[i], b + 4 * i, 4);
}
static void bytes_from_words(uint8_t *b, const uint32_t *w, int nwords) {
    for (int i = 0; i < nwords; i++) memcpy(b + 4 * i, &w[i], 4);
}

extern "C" {

// verdict (0/1); *status = 0 ok / 1 bad key
int cvh_verify(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, uint32_t mlen, int *status) {
    uint32_t aw[8], rw[8], sw[8];
    words_from_bytes(aw, pk, 8);
    words_from_bytes(rw, sig, 8);
    words_from_bytes(sw, sig + 32, 8);
    bool key_ok = false;
    const bool ok = cv_verify_one(CV_BTAB_H, aw, rw, sw, msg, mlen, &key_ok);
    *status = key_ok ? 0 : 1;
    return ok ? 1 : 0;
}

// Keyed (per-key comb) verify of one signature: key prep + hash + comb + finish.
int cvh_verify_keyed(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, uint32_t mlen, int *status) {
    uint32_t aw[8], rw[8], sw[8];
    words_from_bytes(aw, pk, 8);
    words_from_bytes(rw, sig, 8);
    words_from_bytes(sw, sig + 32, 8);
    // 2 x 66 KB of key tables: heap, not thread_local TLS (large TLS blocks in a dlopen'ed library
    // crashed the multi-process tests that share the pytest process)
    std::vector<uint32_t> ktab_v(CV_KTAB_WORDS + 4), ext_v(CV_KTAB_WORDS + 4);
    uint32_t *ktab = reinterpret_cast<uint32_t *>((reinterpret_cast<uintptr_t>(ktab_v.data()) + 15) & ~(uintptr_t)15);
    uint32_t *ext = reinterpret_cast<uint32_t *>((reinterpret_cast<uintptr_t>(ext_v.data()) + 15) & ~(uintptr_t)15);
    uint32_t hs[CV_HS_WORDS];
    uint32_t Rrec[CV_R_WORDS] __attribute__((aligned(16)));
    const bool key_ok = cv_key_prep(aw, ext, ktab);
    cv_keyed_hs(aw, rw, sw, msg, mlen, hs);
    ge_p2 R;
    cv_comb_straus(CV_BCOMB_H, hs, ktab, R);
    fe_store(Rrec, R.X);
    fe_store(Rrec + 10, R.Y);
    fe_store(Rrec + 20, R.Z);
    uint32_t sigw[16];
    for (int q = 0; q < 8; q++) { sigw[q] = rw[q]; sigw[8 + q] = sw[q]; }
    const uint8_t okb = key_ok ? 1 : 0;
    *status = key_ok ? 0 : 1;
    return (int)(cv_verify_finish(Rrec, sigw, &okb, 1) & 1u);
}

// The GPU kernels' organisation on the host: prep + straus per signature, finish in lane chunks of
// CV_FIN_CHUNK consecutive signatures.  verdict[i] = 0/1, status[i] = 0 ok / 1 bad key.
void cvh_verify_batch(uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off,
                      const uint32_t *len, uint8_t *verdict, uint8_t *status) {
    uint32_t *hs = new uint32_t[(size_t)n * CV_HS_WORDS + 16];
    uint32_t *tab = static_cast<uint32_t *>(aligned_alloc(16, ((size_t)n * CV_TAB_WORDS + 4) * 4));
    uint32_t *R = static_cast<uint32_t *>(aligned_alloc(16, ((size_t)n * CV_R_WORDS + 4) * 4));
    uint8_t *ok = new uint8_t[n + 1];
    for (uint32_t i = 0; i < n; i++) {
        uint32_t aw[8], rw[8], sw[8];
        words_from_bytes(aw, pk + 32 * (size_t)i, 8);
        words_from_bytes(rw, sig + 64 * (size_t)i, 8);
        words_from_bytes(sw, sig + 64 * (size_t)i + 32, 8);
        ok[i] = cv_verify_prep(aw, rw, sw, arena + off[i], len[i], hs + (size_t)i * CV_HS_WORDS,
                               tab + (size_t)i * CV_TAB_WORDS) ? 1 : 0;
        status[i] = ok[i] ? 0 : 1;
        ge_p2 Rp;
        cv_verify_straus(CV_BTAB_H, hs + (size_t)i * CV_HS_WORDS, tab + (size_t)i * CV_TAB_WORDS, Rp);
        fe_store(R + (size_t)i * CV_R_WORDS, Rp.X);
        fe_store(R + (size_t)i * CV_R_WORDS + 10, Rp.Y);
        fe_store(R + (size_t)i * CV_R_WORDS + 20, Rp.Z);
    }
    for (uint32_t b = 0; b < n; b += CV_FIN_CHUNK) {
        const int cnt = (int)(n - b < CV_FIN_CHUNK ? n - b : CV_FIN_CHUNK);
        uint32_t sigw[16 * CV_FIN_CHUNK];
        words_from_bytes(sigw, sig + 64 * (size_t)b, 16 * cnt);
        const uint32_t bits = cv_verify_finish(R + (size_t)b * CV_R_WORDS, sigw, ok + b, cnt);
        for (int k = 0; k < cnt; k++) verdict[b + k] = (bits >> k) & 1u;
    }
    delete[] hs;
    free(tab);
    free(R);
    delete[] ok;
}

void cvh_sign(const uint8_t *seed, const uint8_t *msg, uint32_t mlen, uint8_t *pk, uint8_t *sig) {
    uint32_t sd[8], pw[8], sg[16];
    words_from_bytes(sd, seed, 8);
    cv_sign_one(CV_BTAB_H, sd, msg, mlen, pw, sg);
    bytes_from_words(pk, pw, 8);
    bytes_from_words(sig, sg, 16);
}

// field element round trips: in = 32 bytes (value < 2^255), ops on canonical encodings
void cvh_fe_mul(const uint8_t *a, const uint8_t *b, uint8_t *out) {
    uint32_t aw[8], bw[8], ow[8];
    words_from_bytes(aw, a, 8);
    words_from_bytes(bw, b, 8);
    fe fa, fb, fo;
    fe_from_words(fa, aw);
    fe_from_words(fb, bw);
    fe_mul(fo, fa, fb);
    fe_to_words(ow, fo);
    bytes_from_words(out, ow, 8);
}
void cvh_fe_sq(const uint8_t *a, uint8_t *out, int dbl) {
    uint32_t aw[8], ow[8];
    words_from_bytes(aw, a, 8);
    fe fa, fo;
    fe_from_words(fa, aw);
    if (dbl) fe_sq2(fo, fa); else fe_sq(fo, fa);
    fe_to_words(ow, fo);
    bytes_from_words(out, ow, 8);
}
void cvh_fe_invert(const uint8_t *a, uint8_t *out) {
    uint32_t aw[8], ow[8];
    words_from_bytes(aw, a, 8);
    fe fa, fo;
    fe_from_words(fa, aw);
    fe_invert(fo, fa);
    fe_to_words(ow, fo);
    bytes_from_words(out, ow, 8);
}
// mul of raw limb vectors (bounds stress): a, b = 10 int32 limbs each
void cvh_fe_mul_limbs(const uint32_t *a, const uint32_t *b, uint8_t *out) {
    fe fa, fb, fo;
    memcpy(fa.v, a, 40);
    memcpy(fb.v, b, 40);
    fe_mul(fo, fa, fb);
    uint32_t ow[8];
    fe_to_words(ow, fo);
    bytes_from_words(out, ow, 8);
}
// the interleaved forms used by the group formulas: 4 products / 4 squares (the third doubled)
void cvh_fe_mul4_limbs(const uint32_t *a, const uint32_t *b, uint8_t *out) {
    fe f[4], g[4], h[4];
    for (int m = 0; m < 4; m++) {
        memcpy(f[m].v, a + 10 * m, 40);
        memcpy(g[m].v, b + 10 * m, 40);
    }
    fe_mul_n<4>(h, f, g);
    for (int m = 0; m < 4; m++) {
        uint32_t ow[8];
        fe_to_words(ow, h[m]);
        bytes_from_words(out + 32 * m, ow, 8);
    }
}
void cvh_fe_sq4_limbs(const uint32_t *a, uint8_t *out) {
    fe f[4], h[4];
    for (int m = 0; m < 4; m++) memcpy(f[m].v, a + 10 * m, 40);
    fe_sq_n<4, 0x4>(h, f);
    for (int m = 0; m < 4; m++) {
        uint32_t ow[8];
        fe_to_words(ow, h[m]);
        bytes_from_words(out + 32 * m, ow, 8);
    }
}
void cvh_fe_sq_limbs(const uint32_t *a, uint8_t *out) {
    fe fa, fo;
    memcpy(fa.v, a, 40);
    fe_sq(fo, fa);
    uint32_t ow[8];
    fe_to_words(ow, fo);
    bytes_from_words(out, ow, 8);
}
void cvh_fe_to_bytes_limbs(const uint32_t *a, uint8_t *out) {
    fe fa;
    memcpy(fa.v, a, 40);
    uint32_t ow[8];
    fe_to_words(ow, fa);
    bytes_from_words(out, ow, 8);
}

void cvh_sc_reduce(const uint8_t *in64, uint8_t *out32) {
    uint32_t x[16], o[8];
    words_from_bytes(x, in64, 16);
    sc_reduce512(o, x);
    bytes_from_words(out32, o, 8);
}
void cvh_sc_muladd(const uint8_t *a, const uint8_t *b, const uint8_t *c, uint8_t *out) {
    uint32_t aw[8], bw[8], cw[8], o[8];
    words_from_bytes(aw, a, 8);
    words_from_bytes(bw, b, 8);
    words_from_bytes(cw, c, 8);
    sc_muladd(o, aw, bw, cw);
    bytes_from_words(out, o, 8);
}
int cvh_slide_drops(const uint8_t *s) {
    uint32_t w[8];
    words_from_bytes(w, s, 8);
    return slide_drops_carry(w) ? 1 : 0;
}
void cvh_effective_s(const uint8_t *s, uint8_t *out) {
    uint32_t w[8], o[8];
    words_from_bytes(w, s, 8);
    sc_effective_s(o, w);
    bytes_from_words(out, o, 8);
}
int cvh_digit16(const uint8_t *s, int k) {
    uint32_t w[8];
    words_from_bytes(w, s, 8);
    return digit16(w, k);
}
void cvh_digits65536(const uint8_t *s, uint32_t *out8) {
    uint32_t w[8];
    std::memcpy(w, s, 32);
    digits65536_pairs(out8, w);
}
// The tri form's window words (cv_hs_scalars<true, false>: rolled constant-shift digit recoding) against the
// definition — window word = -u digit | (+-v digit) << 5 | w-low digit << 10 | w-high digit << 15 (5 bits
// each, digit16's recoding, w's halves split at 2^128), plus the window count at word 64.  Returns the
// number of differing words of the 65.
int cvh_tri_digit_words_mismatch(const uint8_t *h32, const uint8_t *s32) {
    uint32_t h[8], s[8], hs[CV_HS_WORDS], dig[65], u[8], v[8], w[8];
    words_from_bytes(h, h32, 8);
    words_from_bytes(s, s32, 8);
    for (int i = 0; i < 8; i++) { hs[i] = h[i]; hs[8 + i] = s[i]; }
    cv_hs_scalars<true, false>(hs, dig, 1);
    bool v_neg;
    int nwin;
    sc_halfsize(u, v, v_neg, nwin, w, h, s);
    int bad = dig[64] != (uint32_t)nwin;
    for (int win = 0; win < 64; win++) {
        const int da = -digit16(u, win), dr = v_neg ? -digit16(v, win) : digit16(v, win);
        const int dlo = win < 32 ? digit16(w, win) : 0, dhi = win < 32 ? digit16(w, 32 + win) : 0;
        const uint32_t want = ((uint32_t)da & 0x1fu) | (((uint32_t)dr & 0x1fu) << 5) | (((uint32_t)dlo & 0x1fu) << 10) |
                              (((uint32_t)dhi & 0x1fu) << 15);
        bad += dig[win] != want;
    }
    return bad;
}
int cvh_digit256(const uint8_t *s, int k) {
    uint32_t w[8];
    words_from_bytes(w, s, 8);
    return digit256(w, k);
}
int cvh_digit256_row(const uint8_t *s, int j, int u) {
    uint32_t w[8];
    words_from_bytes(w, s, 8);
    return digit256_row(w, j, u);
}
void cvh_sha512(const uint8_t *pre, int npre, const uint8_t *msg, uint32_t mlen, uint8_t *out) {
    uint32_t p[16] = {0}, o[16];
    words_from_bytes(p, pre, npre / 4);
    sha512_pre_msg(o, p, npre, msg, mlen);
    bytes_from_words(out, o, 16);
}
void cvh_sha256(const uint8_t *msg, uint32_t n, uint8_t *out) {
    uint32_t o[8];
    sha256_bytes(o, msg, n);
    for (int i = 0; i < 8; i++) {
        const uint32_t v = cv_bswap32(o[i]);
        memcpy(out + 4 * i, &v, 4);
    }
}
// Merkle root over leaf digests (bytes, cnt x 32); returns 0 for empty
uint32_t cvh_tx_of_sig(uint32_t g, uint32_t nt, const uint32_t *tsb) { return cv_tx_of_sig(g, nt, tsb); }
int cvh_tx_all_valid(uint32_t b, uint32_t e, const uint64_t *bitmap) { return cv_tx_all_valid(b, e, bitmap) ? 1 : 0; }

int cvh_merkle_root(const uint8_t *leaves, uint32_t cnt, uint8_t *out) {
    uint32_t *lvl = new uint32_t[8 * (cnt ? cnt : 1)];
    for (uint32_t i = 0; i < 8 * cnt; i++) {
        uint32_t v;
        memcpy(&v, leaves + 4 * i, 4);
        lvl[i] = cv_bswap32(v);
    }
    uint32_t root[8];
    const bool ok = cv_merkle_root_inplace(lvl, cnt, root);
    for (int i = 0; i < 8; i++) {
        const uint32_t v = cv_bswap32(root[i]);
        memcpy(out + 4 * i, &v, 4);
    }
    delete[] lvl;
    return ok ? 1 : 0;
}

// Half-size-scalar verify of one signature (prep + hsprep + straus, identity test).  sc_out:
// CV_HS_DIGWORDS (73) words.
int cvh_verify_hs(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, uint32_t mlen, int *status,
                  uint32_t *sc_out) {
    uint32_t aw[8], rw[8], sw[8];
    words_from_bytes(aw, pk, 8);
    words_from_bytes(rw, sig, 8);
    words_from_bytes(sw, sig + 32, 8);
    bool key_ok = false;
    const bool ok = cv_verify_one_hs(CV_BCOMB_H, aw, rw, sw, msg, mlen, &key_ok, sc_out);
    *status = key_ok ? 0 : 1;
    return ok ? 1 : 0;
}

// sc_halfsize on (h, s) given as 32 LE bytes each; out = u (32 B) | |v| (32 B) | w (32 B).
int cvh_halfsize(const uint8_t *h, const uint8_t *s, uint8_t *out, int *v_neg, int *nwin) {
    uint32_t hw[8], sw[8], u[8], v[8], w[8];
    words_from_bytes(hw, h, 8);
    words_from_bytes(sw, s, 8);
    bool neg = false;
    int nw = 0;
    const bool ok = sc_halfsize(u, v, neg, nw, w, hw, sw);
    bytes_from_words(out, u, 8);
    bytes_from_words(out + 32, v, 8);
    bytes_from_words(out + 64, w, 8);
    *v_neg = neg ? 1 : 0;
    *nwin = nw;
    return ok ? 1 : 0;
}

// The device's reciprocal sequence in cv_qdiv on the host (0 = exact division), for the lattice tests.
void cvh_set_rcp_emulation(double rel_err) { cv_rcp_emulation = rel_err; }

// One quotient step of sc_halfsize's exact loop on (r0, r1) given as 32 LE bytes each (r0 >= r1 >= 2^128):
// returns q and r0 - q r1 in out (32 B).
uint32_t cvh_exact_step(const uint8_t *r0b, const uint8_t *r1b, uint8_t *out) {
    uint32_t r0[8], r1[8];
    words_from_bytes(r0, r0b, 8);
    words_from_bytes(r1, r1b, 8);
    const uint32_t q = cv_exact_quotient(r0, r1);
    cv_submul8(r0, r1, q);
    bytes_from_words(out, r0, 8);
    return q;
}

// PartialMerkleTree.verify of tree t of a flat batch (cv_pmt_verify); returns status, *verdict.
int cvh_pmt_verify(uint32_t b, uint32_t e, const uint8_t *kind, const uint32_t *left, const uint32_t *right,
                   const uint8_t *leaf_hash, const uint8_t *root, const uint8_t *check, uint32_t cb, uint32_t ce,
                   uint32_t *dig, uint8_t *flag, int *verdict) {
    bool v = false;
    const int st = cv_pmt_verify(b, e, kind, left, right, leaf_hash, root, check, cb, ce, dig, flag, v);
    *verdict = v ? 1 : 0;
    return st;
}

// Fused half-size prep (interleaved A/R decodes) + straus for one signature.
int cvh_verify_hs_fused(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, uint32_t mlen, int *status, int lat) {
    uint32_t aw[8], rw[8], sw[8];
    words_from_bytes(aw, pk, 8);
    words_from_bytes(rw, sig, 8);
    words_from_bytes(sw, sig + 32, 8);
    bool key_ok = false;
    const bool ok = lat ? cv_verify_one_hs_fused<true>(CV_BCOMB_H, aw, rw, sw, msg, mlen, &key_ok)
                        : cv_verify_one_hs_fused<false>(CV_BCOMB_H, aw, rw, sw, msg, mlen, &key_ok);
    *status = key_ok ? 0 : 1;
    return ok ? 1 : 0;
}

static int table_compare(const uint32_t *full, const uint32_t *split);
// The latency prep's split odd-multiple table (two lanes per point, ge_cached_multiples8_half) against
// the one-lane table, for the point a 32-byte encoding decodes to (as key: k*(-A); as R: k*R; the
// identity when it does not decode).  Returns the number of differing words of the 9-entry table.
int cvh_table_split_mismatch(const uint8_t *enc32, int is_r) {
    uint32_t w[8];
    words_from_bytes(w, enc32, 8);
    uint32_t full[CV_TAB_WORDS], split[CV_TAB_WORDS];
    for (int i = 0; i < CV_TAB_WORDS; i++) full[i] = 0xdeadbeefu, split[i] = 0x0badf00du;
    const bool ok1 = cv_hs_point_one<false>(w, is_r != 0, full);
    const bool ok2 = cv_hs_point_one<false>(w, is_r != 0, split, 0);
    const bool ok3 = cv_hs_point_one<false>(w, is_r != 0, split, 1);
    return ((ok1 != ok2 || ok1 != ok3) ? 1000 : 0) + table_compare(full, split);
}

// the same point in each entry (projective: the split tables reach 4P, 6P, 8P by additions, so their Z
// differs from the one-lane doublings'): (Y+X)/Z, (Y-X)/Z, 2dT/Z agree, and Z != 0
static int table_compare(const uint32_t *full, const uint32_t *split) {
    int bad = 0;
    for (int k = 0; k < 9; k++) {
        ge_cached a, b;
        ge_cached_load(a, full + 40 * k);
        ge_cached_load(b, split + 40 * k);
        const fe *fa[3] = {&a.YplusX, &a.YminusX, &a.T2d}, *fb[3] = {&b.YplusX, &b.YminusX, &b.T2d};
        for (int c = 0; c < 3; c++) {
            fe l, r;
            uint32_t lw[8], rw2[8];
            fe_mul(l, *fa[c], b.Z);
            fe_mul(r, *fb[c], a.Z);
            fe_to_words(lw, l);
            fe_to_words(rw2, r);
            for (int q = 0; q < 8; q++) bad += lw[q] != rw2[q];
        }
        uint32_t zw[8];
        fe_to_words(zw, b.Z);
        bool zero = true;
        for (int q = 0; q < 8; q++) zero = zero && zw[q] == 0;
        bad += zero;   // Z != 0
    }
    return bad;
}

}  // extern "C"
