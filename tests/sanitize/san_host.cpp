// san_host.cpp — TEST INFRASTRUCTURE: the host-only logic of the C-ABI library (corda_amd/csrc/cv_api.cpp)
// built with AddressSanitizer + UndefinedBehaviorSanitizer (or ThreadSanitizer) and exercised without a
// GPU.  cv_api.cpp is included whole so its file-local functions are reachable; the kernel launchers it
// calls (cv_launch.h) are stubs that never run.  Checked here:
//   dedupe_keys          key dedupe of cv_ed25519_verify_batch (pools, early out, limits)
//   WorkerPool/par_copy  the packing thread pool and its pinned-staging copies (piece boundaries, empty jobs)
//   stage_plan/_pack     staging layout of a record range (arena range and compact gather forms)
//   pipe_cuts            the host pipeline's sub-chunk plan (64-aligned, covering, balanced tail)
//   for_each_shard       shard ranges over k devices, one thread each
//   cv_tx_verdicts       per-transaction AND
// Exit status 0 = every check passed; sanitizer reports abort the run (halt_on_error).
#include "../../corda_amd/csrc/cv_api.cpp"

#include <cstdio>
#include <cstdlib>

extern "C" {
// launcher stubs: nothing in this test reaches the device
hipError_t cvk_verify(uint32_t, const uint8_t *, const uint8_t *, const uint8_t *, const uint64_t *, const uint32_t *,
                      uint64_t *, uint8_t *, uint32_t *, uint32_t *, uint32_t *, uint8_t *, uint32_t *, uint32_t,
                      hipStream_t, hipEvent_t *, const CvkSplit *) { return hipErrorNoDevice; }
hipError_t cvk_sign(uint32_t, const uint8_t *, const uint8_t *, const uint64_t *, const uint32_t *, uint8_t *, uint8_t *,
                    hipStream_t) { return hipErrorNoDevice; }
hipError_t cvk_pmt_verify(uint32_t, const uint8_t *, const uint32_t *, const uint32_t *, const uint8_t *, const uint32_t *,
                          const uint8_t *, const uint8_t *, const uint32_t *, uint32_t *, uint8_t *, uint8_t *, uint8_t *,
                          hipStream_t) { return hipErrorNoDevice; }
hipError_t cvk_merkle(uint32_t, uint32_t, const uint8_t *, const uint64_t *, const uint32_t *, const uint32_t *, uint32_t *,
                      uint8_t *, uint8_t *, hipStream_t) { return hipErrorNoDevice; }
hipError_t cvk_calibrate(uint32_t, int, uint32_t, void *, hipStream_t) { return hipErrorNoDevice; }
hipError_t cvk_prep_probe(uint32_t, const uint8_t *, const uint8_t *, const uint8_t *, const uint64_t *, const uint32_t *,
                          uint32_t *, uint32_t *, uint32_t, uint64_t *, hipStream_t) { return hipErrorNoDevice; }
hipError_t cvk_mad_clock(uint32_t, uint32_t, uint64_t *, hipStream_t) { return hipErrorNoDevice; }
uint32_t cvk_get_tri_max(void) { return 4096; }
int cvk_tri_zc_ok(uint32_t, uint32_t) { return 0; }
hipError_t cvk_verify_tri_zc(uint32_t, const uint8_t *, const uint8_t *, const uint8_t *, const uint64_t *,
                             const uint32_t *, uint8_t *, uint8_t *, uint32_t *, uint8_t *, uint32_t *, uint32_t,
                             hipStream_t, const void *, void *, size_t) {
    return hipErrorNoDevice;
}
hipError_t cvk_prepare(hipStream_t) { return hipErrorNoDevice; }
hipError_t cvk_keyprep(uint32_t, const uint8_t *, const uint32_t *, uint32_t *, uint32_t *, uint8_t *, hipStream_t) {
    return hipErrorNoDevice;
}
hipError_t cvk_verify_keyed(uint32_t, const uint8_t *, const uint32_t *, const uint32_t *, const uint32_t *,
                            const uint8_t *, const uint8_t *, const uint8_t *, const uint64_t *, const uint32_t *,
                            uint64_t *, uint8_t *, uint32_t *, uint32_t *, uint8_t *, uint32_t, hipStream_t, hipEvent_t *) {
    return hipErrorNoDevice;
}
}

static int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                         \
        }                                                                     \
    } while (0)

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

static void test_dedupe() {
    for (size_t n : {0ul, 1ul, 63ul, 64ul, 65ul, 1000ul, 1025ul, 5000ul, 70000ul, (size_t)kAutoKeyedMax,
                     (size_t)kAutoKeyedMax + 1}) {
        for (size_t pool : {1ul, 7ul, 64ul, 300ul, 100000ul}) {
            std::vector<uint8_t> keys_pool(32 * pool);
            for (auto &b : keys_pool) b = (uint8_t)rnd();
            std::vector<uint8_t> pk(32 * std::max<size_t>(n, 1));
            for (size_t i = 0; i < n; i++) std::memcpy(&pk[32 * i], &keys_pool[32 * (rnd() % pool)], 32);
            std::vector<uint8_t> keys;
            std::vector<uint32_t> idx;
            const bool took = dedupe_keys(n, pk.data(), keys, idx);
            if (n < 64 || n > kAutoKeyedMax) CHECK(!took);
            if (!took) continue;
            const size_t nk = keys.size() / 32;
            CHECK(idx.size() == n);
            CHECK(8 * nk <= n);
            for (size_t i = 0; i < n; i++) {
                CHECK(idx[i] < nk);
                if (idx[i] < nk) CHECK(std::memcmp(&keys[32 * idx[i]], &pk[32 * i], 32) == 0);
            }
            for (size_t a = 0; a + 1 < nk && a < 64; a++)     // distinct keys are distinct
                CHECK(std::memcmp(&keys[32 * a], &keys[32 * (a + 1)], 32) != 0);
        }
    }
    // keys that differ in one byte only must not collide in the dedupe
    const size_t n = 4096;
    std::vector<uint8_t> pk(32 * n, 0xAB);
    for (size_t i = 0; i < n; i++) pk[32 * i + 31] = (uint8_t)(i / 16);   // 16 per key, 256 keys
    std::vector<uint8_t> keys;
    std::vector<uint32_t> idx;
    CHECK(dedupe_keys(n, pk.data(), keys, idx));
    CHECK(keys.size() / 32 == 256);
}

static void test_pool() {
    // every task of every run executes exactly once, across many back-to-back runs (TSan: no races in
    // the generation handshake)
    for (int helpers : {0, 1, 3, 7}) {
        WorkerPool pool(helpers);
        std::vector<std::atomic<int>> hits(97);
        for (int r = 0; r < 400; r++) {
            const size_t nt = (size_t)(r % 97) + 1;
            for (size_t i = 0; i < nt; i++) hits[i].store(0);
            pool.run(nt, [&](size_t i) { hits[i].fetch_add(1); });
            for (size_t i = 0; i < nt; i++) CHECK(hits[i].load() == 1);
        }
    }
}

static void test_par_copy() {
    for (int threads : {1, 2, 3, 4, 8, 13}) {
        for (int rep = 0; rep < 6; rep++) {
            std::vector<std::vector<uint8_t>> src(5), dst(5);
            std::vector<CopyJob> jobs;
            for (int j = 0; j < 5; j++) {
                const size_t len = rep == 0 ? 0 : (rnd() % 3) * (512 * 1024) + rnd() % 100000;
                src[j].resize(len + 1);
                dst[j].assign(len + 1, 0);
                for (auto &b : src[j]) b = (uint8_t)rnd();
                jobs.push_back({dst[j].data(), src[j].data(), len});
            }
            WorkerPool pool(threads - 1);
            par_copy(jobs, &pool);
            CHECK(pool.threads() == threads);
            for (int j = 0; j < 5; j++) {
                CHECK(std::memcmp(dst[j].data(), src[j].data(), jobs[j].len) == 0);
                CHECK(dst[j][jobs[j].len] == 0);              // nothing written past the job
            }
        }
    }
}

static void test_stage(bool scattered, size_t n) {
    std::vector<uint32_t> len(n);
    std::vector<uint64_t> off(n);
    size_t arena_size = scattered ? (32u << 20) : n * 700 + 64;
    std::vector<uint8_t> arena(arena_size);
    for (auto &b : arena) b = (uint8_t)rnd();
    uint64_t pos = 5;
    for (size_t i = 0; i < n; i++) {
        len[i] = (uint32_t)(rnd() % 701);
        if (scattered) {
            off[i] = rnd() % (arena_size - 701);
        } else {
            off[i] = pos;
            pos += len[i] + rnd() % 3;
        }
    }
    std::vector<uint8_t> pk(32 * n), sig(64 * n);
    for (auto &b : pk) b = (uint8_t)rnd();
    for (auto &b : sig) b = (uint8_t)rnd();
    for (size_t b : {0ul, 64ul, 1000ul}) {
        for (size_t e : {b + 1, b + 64, n}) {
            if (e > n || e <= b) continue;
            WorkerPool pool(2);
            const Stage st = stage_plan(b, e, off.data(), len.data(), (e - b) % 2 ? &pool : nullptr);
            const Stage st1 = stage_plan(b, e, off.data(), len.data());
            CHECK(st.lo == st1.lo && st.hi == st1.hi && st.total == st1.total && st.compact == st1.compact);
            if (e - b >= 64) CHECK(st.compact == scattered);
            std::vector<uint8_t> h(st.total + 64, 0xEE);
            stage_pack(st, h.data(), b, pk.data(), sig.data(), arena.data(), off.data(), len.data(), &pool, [] {});
            CHECK(h[st.total] == 0xEE);                                    // nothing past the staging
            CHECK(std::memcmp(h.data() + st.o_pk, &pk[32 * b], 32 * (e - b)) == 0);
            CHECK(std::memcmp(h.data() + st.o_sig, &sig[64 * b], 64 * (e - b)) == 0);
            const uint64_t *hoff = reinterpret_cast<const uint64_t *>(h.data() + st.o_off);
            const uint32_t *hlen = reinterpret_cast<const uint32_t *>(h.data() + st.o_len);
            for (size_t i = b; i < e; i++) {
                CHECK(hlen[i - b] == len[i]);
                // the device reads arena_dev - lo + off: here the staging arena part stands for arena_dev
                const uint64_t rel = hoff[i - b] - st.lo;
                CHECK(rel + len[i] <= st.hi - st.lo);
                CHECK(std::memcmp(h.data() + st.o_ar + rel, &arena[off[i]], len[i]) == 0);
                if (!st.compact) CHECK(hoff[i - b] % 16 == off[i] % 16);      // alignment kept
            }
            for (int k = 0; k < 16; k++) CHECK(h[st.o_ar + (st.hi - st.lo) + k] == 0);
        }
    }
}

static void test_pipe_cuts() {
    for (size_t b : {0ul, 64ul, 128000ul}) {
        for (size_t n : {1ul, 63ul, 64ul, 65ul, 131073ul, 1000000ul, 4394307ul}) {
            for (size_t first : {64ul, 100ul, 65536ul}) {
                for (size_t C : {64ul, 1000ul, 262144ul}) {
                    if (n / std::max<size_t>(C, 64) > 200000) continue;
                    const auto cut = pipe_cuts(b, b + n, first, C);
                    CHECK(cut.front() == b && cut.back() == b + n);
                    for (size_t j = 0; j + 1 < cut.size(); j++) {
                        CHECK(cut[j + 1] > cut[j]);
                        if (j + 2 < cut.size()) CHECK((cut[j + 1] - b) % 64 == 0);
                        CHECK(cut[j + 1] - cut[j] <= std::max(first, std::max<size_t>(C / 64 * 64, 64)));
                    }
                }
            }
        }
    }
}

static void test_shards() {
    for (size_t ndev : {1ul, 2ul, 3ul, 8ul}) {
        cv_ctx ctx;
        ctx.devs.resize(ndev);
        for (size_t k = 0; k < ndev; k++) ctx.devs[k].ordinal = (int)k;
        for (size_t n : {1ul, 64ul, 65ul, 1000ul, 100003ul}) {
            std::vector<std::vector<std::pair<size_t, size_t>>> got(ndev);
            std::mutex mu;
            const int rc = for_each_shard(&ctx, n, [&](Device &d, size_t b, size_t e, int threads) {
                std::lock_guard<std::mutex> g(mu);
                got[(size_t)d.ordinal].push_back({b, e});
                return threads >= 1 ? CV_OK : CV_E_ARGS;
            });
            CHECK(rc == CV_OK);
            std::vector<std::pair<size_t, size_t>> all;
            for (auto &v : got) all.insert(all.end(), v.begin(), v.end());
            std::sort(all.begin(), all.end());
            size_t p = 0;
            for (auto &r : all) {
                CHECK(r.first == p);
                CHECK(r.first % 64 == 0);
                p = r.second;
            }
            CHECK(p == n);
        }
        for (Device &d : ctx.devs) d.stream = nullptr;
        ctx.devs.clear();
    }
}

static void test_tx_verdicts() {
    for (int rep = 0; rep < 50; rep++) {
        const size_t ntx = rnd() % 300 + 1;
        std::vector<uint32_t> begin(ntx + 1, 0);
        for (size_t t = 0; t < ntx; t++) begin[t + 1] = begin[t] + (uint32_t)(rnd() % 5);
        const size_t n = begin[ntx];
        std::vector<uint64_t> bm((n + 63) / 64 + 1);
        for (auto &w : bm) w = (rnd() % 4) ? ~0ull : rnd();
        std::vector<uint8_t> ok(ntx, 7);
        CHECK(cv_tx_verdicts(ntx, bm.data(), begin.data(), ok.data()) == CV_OK);
        for (size_t t = 0; t < ntx; t++) {
            bool want = begin[t + 1] > begin[t];
            for (uint32_t i = begin[t]; i < begin[t + 1]; i++) want = want && ((bm[i / 64] >> (i % 64)) & 1);
            CHECK(ok[t] == (want ? 1 : 0));
        }
    }
    uint32_t bad[3] = {0, 5, 2};
    uint64_t w = ~0ull;
    uint8_t ok[2];
    CHECK(cv_tx_verdicts(2, &w, bad, ok) == CV_E_ARGS);
    CHECK(cv_tx_verdicts(0, nullptr, nullptr, nullptr) == CV_OK);
}

static void test_abi_guards() {
    cv_ctx *ctx = nullptr;
    CHECK(cv_open(0, nullptr) == CV_E_ARGS);
    uint64_t bm[1];
    CHECK(cv_ed25519_verify_batch(nullptr, 1, nullptr, nullptr, nullptr, nullptr, nullptr, bm, nullptr) == CV_E_ARGS);
    CHECK(cv_strerror(CV_E_OOM) != nullptr && cv_strerror(12345) != nullptr);
    std::vector<uint8_t> pk(32 * 100);
    std::vector<uint32_t> idx(100);
    size_t nk = 99;
    CHECK(cv_diag_dedupe_keys(100, pk.data(), idx.data(), &nk) == 1 && nk == 1);
    (void)ctx;
}

int main(int argc, char **argv) {
    const bool threads_only = argc > 1 && std::strcmp(argv[1], "--threads") == 0;
    test_pool();
    test_par_copy();
    test_shards();
    if (!threads_only) {
        test_dedupe();
        test_stage(false, 3001);
        test_stage(true, 3001);
        test_stage(false, 140001);   // several range-scan slices
        test_pipe_cuts();
        test_tx_verdicts();
        test_abi_guards();
    }
    if (g_fail) {
        std::fprintf(stderr, "san_host: %d checks failed\n", g_fail);
        return 1;
    }
    std::printf("san_host: all checks passed%s\n", threads_only ? " (thread tests)" : "");
    return 0;
}
