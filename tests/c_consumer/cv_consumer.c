/* cv_consumer.c — the drop-in boundary driven from plain C99, the way a JNI / JNA / cgo binding drives it: only
 * include/cordaverify.h and the shared library, no Python, no torch.  tests/test_c_consumer.py compiles it with
 * gcc -std=c99 -pedantic -Werror and runs it on a fixture it writes from the golden corpus.
 *
 *   cv_consumer FIXTURE        exit 0: every check passed; 3: no GPU (the host-only checks passed); 1: a check failed
 *
 * Fixture (little-endian): "CVF1", u64 n, u64 arena_bytes, pk[n][32], sig[n][64], off[n] u64, len[n] u32,
 * verdict[n] u8, status[n] u8, arena[arena_bytes].
 *
 * What it checks, each against the reference behaviour the header's entry point replaces:
 *  - host-only entry points: cv_version, cv_strerror, cv_msg_extent, cv_tx_verdicts (SignedTransaction.kt:58-72's
 *    per-transaction AND), and cv_open failing with CV_E_NO_DEVICE rather than falling back;
 *  - with a GPU: cv_ed25519_verify_batch (CryptoUtilities.kt:90-96, one verdict bit and one status byte per record)
 *    against the corpus' expected verdicts, the batch repeated to several sizes (whole and ragged bitmap words);
 *    the _ex arena bound (CV_E_ARGS one byte short); the _async form + cv_wait; inputs in cv_host_alloc memory. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cordaverify.h"

static int failures = 0;
#define CHECK(c, ...)                                                   \
    do {                                                                \
        if (!(c)) {                                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);       \
            fprintf(stderr, __VA_ARGS__);                               \
            fputc('\n', stderr);                                        \
            failures++;                                                 \
        }                                                               \
    } while (0)

struct batch {
    size_t n;
    uint64_t arena_bytes;
    uint8_t *pk, *sig, *verdict, *status, *arena;
    uint64_t *off;
    uint32_t *len;
};

static void *xmalloc(size_t b) {
    void *p = malloc(b ? b : 1);
    if (!p) {
        fprintf(stderr, "out of memory\n");
        exit(1);
    }
    return p;
}

static int read_all(FILE *f, void *dst, size_t bytes) { return fread(dst, 1, bytes, f) == bytes; }

static int load_fixture(const char *path, struct batch *b) {
    FILE *f = fopen(path, "rb");
    char magic[4];
    uint64_t n;
    int ok;
    if (!f) return 0;
    ok = read_all(f, magic, 4) && memcmp(magic, "CVF1", 4) == 0 && read_all(f, &n, 8) && read_all(f, &b->arena_bytes, 8);
    if (!ok) {
        fclose(f);
        return 0;
    }
    b->n = (size_t)n;
    b->pk = xmalloc(b->n * 32);
    b->sig = xmalloc(b->n * 64);
    b->off = xmalloc(b->n * 8);
    b->len = xmalloc(b->n * 4);
    b->verdict = xmalloc(b->n);
    b->status = xmalloc(b->n);
    b->arena = xmalloc((size_t)b->arena_bytes);
    ok = read_all(f, b->pk, b->n * 32) && read_all(f, b->sig, b->n * 64) && read_all(f, b->off, b->n * 8) &&
         read_all(f, b->len, b->n * 4) && read_all(f, b->verdict, b->n) && read_all(f, b->status, b->n) &&
         read_all(f, b->arena, (size_t)b->arena_bytes);
    fclose(f);
    return ok;
}

/* the corpus repeated to m records (record i = corpus record i mod n; the arena is shared) */
static void repeat(const struct batch *src, size_t m, struct batch *dst) {
    size_t i;
    *dst = *src;
    dst->n = m;
    dst->pk = xmalloc(m * 32);
    dst->sig = xmalloc(m * 64);
    dst->off = xmalloc(m * 8);
    dst->len = xmalloc(m * 4);
    dst->verdict = xmalloc(m);
    dst->status = xmalloc(m);
    for (i = 0; i < m; i++) {
        const size_t j = i % src->n;
        memcpy(dst->pk + 32 * i, src->pk + 32 * j, 32);
        memcpy(dst->sig + 64 * i, src->sig + 64 * j, 64);
        dst->off[i] = src->off[j];
        dst->len[i] = src->len[j];
        dst->verdict[i] = src->verdict[j];
        dst->status[i] = src->status[j];
    }
}

static void free_repeat(struct batch *b) {
    free(b->pk);
    free(b->sig);
    free(b->off);
    free(b->len);
    free(b->verdict);
    free(b->status);
}

/* bit i of word i/64 = record i's verdict; bits past n must be 0; status byte per record */
static int compare(const char *what, const struct batch *b, const uint64_t *bm, const uint8_t *st) {
    size_t i, bad = 0;
    const size_t words = (b->n + 63) / 64;
    for (i = 0; i < b->n; i++) {
        const int bit = (int)((bm[i / 64] >> (i % 64)) & 1u);
        if (bit != b->verdict[i] || (st && st[i] != b->status[i])) {
            if (bad < 5)
                fprintf(stderr, "  %s: record %zu verdict %d (expected %d) status %d (expected %d)\n", what, i, bit,
                        b->verdict[i], st ? st[i] : -1, b->status[i]);
            bad++;
        }
    }
    if (b->n % 64) CHECK((bm[words - 1] >> (b->n % 64)) == 0, "%s: bits past n set", what);
    CHECK(bad == 0, "%s: %zu of %zu records differ", what, bad, b->n);
    return bad == 0;
}

static void host_only_checks(const struct batch *b) {
    uint64_t ext = 0;
    size_t i;
    const char *v = cv_version();
    CHECK(v && strstr(v, "gfx950"), "cv_version: %s", v ? v : "(null)");
    CHECK(cv_strerror(CV_OK) && strcmp(cv_strerror(CV_OK), "ok") == 0, "cv_strerror(CV_OK)");
    CHECK(cv_strerror(CV_E_ARGS) != NULL, "cv_strerror(CV_E_ARGS)");
    for (i = 0; i < b->n; i++)
        if (b->off[i] + b->len[i] > ext) ext = b->off[i] + b->len[i];
    CHECK(cv_msg_extent(b->n, b->off, b->len) == ext, "cv_msg_extent");
    CHECK(cv_msg_extent(0, NULL, NULL) == 0, "cv_msg_extent(0)");
    {
        /* three transactions over 130 signatures: [0, 64) all valid, [64, 66) one invalid, [66, 130) valid */
        uint64_t bm[3] = {~0ull, ~0ull ^ 2ull, 3ull};
        const uint32_t begin[4] = {0, 64, 66, 130};
        uint8_t ok[3] = {9, 9, 9};
        CHECK(cv_tx_verdicts(3, bm, begin, ok) == CV_OK, "cv_tx_verdicts rc");
        CHECK(ok[0] == 1 && ok[1] == 0 && ok[2] == 1, "cv_tx_verdicts %d %d %d", ok[0], ok[1], ok[2]);
    }
}

static void verify_checks(cv_ctx *ctx, const struct batch *corpus) {
    const size_t sizes[4] = {1, 64, corpus->n, 3 * corpus->n + 17};
    int s;
    for (s = 0; s < 4; s++) {
        struct batch b;
        size_t words;
        uint64_t *bm;
        uint8_t *st;
        char what[64];
        int rc;
        repeat(corpus, sizes[s], &b);
        words = (b.n + 63) / 64;
        bm = xmalloc(words * 8);
        st = xmalloc(b.n);
        memset(bm, 0xa5, words * 8);
        rc = cv_ed25519_verify_batch(ctx, b.n, b.pk, b.sig, b.arena, b.off, b.len, bm, st);
        snprintf(what, sizeof what, "verify_batch n=%zu", b.n);
        CHECK(rc == CV_OK, "%s rc %d (%s)", what, rc, cv_strerror(rc));
        if (rc == CV_OK) compare(what, &b, bm, st);

        /* the arena bound: exact extent passes, one byte short is refused before any read */
        {
            const uint64_t ext = cv_msg_extent(b.n, b.off, b.len);
            memset(bm, 0, words * 8);
            rc = cv_ed25519_verify_batch_ex(ctx, b.n, b.pk, b.sig, b.arena, ext, b.off, b.len, bm, NULL, NULL);
            CHECK(rc == CV_OK, "verify_batch_ex at the extent rc %d", rc);
            if (rc == CV_OK) compare("verify_batch_ex", &b, bm, NULL);
            if (ext > 0) {
                rc = cv_ed25519_verify_batch_ex(ctx, b.n, b.pk, b.sig, b.arena, ext - 1, b.off, b.len, bm, NULL, NULL);
                CHECK(rc == CV_E_ARGS, "verify_batch_ex one byte short rc %d (expected CV_E_ARGS)", rc);
            }
        }
        /* asynchronous form: submit two, wait in reverse order */
        {
            uint64_t *bm2 = xmalloc(words * 8);
            uint64_t t1 = 0, t2 = 0;
            memset(bm, 0, words * 8);
            memset(bm2, 0, words * 8);
            rc = cv_ed25519_verify_batch_async(ctx, b.n, b.pk, b.sig, b.arena, b.off, b.len, bm, NULL, &t1);
            CHECK(rc == CV_OK, "async submit 1 rc %d", rc);
            rc = cv_ed25519_verify_batch_async(ctx, b.n, b.pk, b.sig, b.arena, b.off, b.len, bm2, st, &t2);
            CHECK(rc == CV_OK, "async submit 2 rc %d", rc);
            CHECK(cv_wait(ctx, t2) == CV_OK, "cv_wait 2");
            CHECK(cv_wait(ctx, t1) == CV_OK, "cv_wait 1");
            CHECK(cv_wait(ctx, t1) == CV_E_ARGS, "a ticket is waited at most once");
            compare("async 1", &b, bm, NULL);
            compare("async 2", &b, bm2, st);
            free(bm2);
        }
        free(bm);
        free(st);
        free_repeat(&b);
    }

    /* every input array in pinned memory from cv_host_alloc (the engine DMAs straight out of them) */
    {
        const struct batch *b = corpus;
        const size_t words = (b->n + 63) / 64;
        void *p[6] = {0};
        const size_t bytes[6] = {b->n * 32, b->n * 64, (size_t)b->arena_bytes, b->n * 8, b->n * 4, words * 8};
        int k, rc = CV_OK;
        for (k = 0; k < 6 && rc == CV_OK; k++) rc = cv_host_alloc(ctx, bytes[k], &p[k]);
        CHECK(rc == CV_OK, "cv_host_alloc rc %d", rc);
        if (rc == CV_OK) {
            memcpy(p[0], b->pk, bytes[0]);
            memcpy(p[1], b->sig, bytes[1]);
            memcpy(p[2], b->arena, bytes[2]);
            memcpy(p[3], b->off, bytes[3]);
            memcpy(p[4], b->len, bytes[4]);
            memset(p[5], 0, bytes[5]);
            rc = cv_ed25519_verify_batch(ctx, b->n, p[0], p[1], p[2], p[3], p[4], p[5], NULL);
            CHECK(rc == CV_OK, "pinned verify rc %d", rc);
            if (rc == CV_OK) compare("pinned inputs", b, p[5], NULL);
        }
        for (k = 0; k < 6; k++)
            if (p[k]) cv_host_free(ctx, p[k]);
    }
}

int main(int argc, char **argv) {
    struct batch corpus;
    cv_ctx *ctx = NULL;
    int rc;
    if (argc != 2 || !load_fixture(argv[1], &corpus)) {
        fprintf(stderr, "usage: cv_consumer FIXTURE (a CVF1 file)\n");
        return 1;
    }
    host_only_checks(&corpus);
    rc = cv_open(0, &ctx);
    if (rc == CV_E_NO_DEVICE) {
        CHECK(ctx == NULL, "cv_open without a device left a context");
        printf("host-only checks: %s; cv_open: %s\n", failures ? "FAILED" : "ok", cv_strerror(rc));
        return failures ? 1 : 3;
    }
    CHECK(rc == CV_OK && ctx != NULL, "cv_open rc %d (%s)", rc, cv_strerror(rc));
    if (rc != CV_OK) return 1;
    printf("devices: %d\n", cv_device_count(ctx));
    verify_checks(ctx, &corpus);
    cv_close(ctx);
    printf("%s (%zu corpus records)\n", failures ? "FAILED" : "all checks passed", corpus.n);
    return failures ? 1 : 0;
}
