// san_host.cpp — TEST INFRASTRUCTURE: the host-only logic of the C-ABI library (corda_amd/csrc/cv_api.cpp)
// built with AddressSanitizer + UndefinedBehaviorSanitizer (or ThreadSanitizer) and exercised without a
// GPU.  cv_api.cpp is included whole so its file-local functions are reachable; the kernel launchers it
// calls (cv_launch.h) are stubs that never run.  Checked here:
//   dedupe_keys          key dedupe of cv_ed25519_verify_batch (pools, gate, slices on a pool, first-seen order)
//   WorkerPool/par_copy  the packing thread pool and its pinned-staging copies (piece boundaries, empty jobs)
//   stage_plan/_pack     staging layout of a record range (arena range and compact gather forms)
//   pipe_cuts            the host pipeline's sub-chunk plan (64-aligned, covering, balanced tail)
//   dispatch             routing: shard ranges over k devices, per-device exclusion, concurrent callers
//   mstage_plan/_pack    Merkle staging of a transaction range (non-monotone offsets, empty txs, compact)
//   cv_tx_verdicts       per-transaction AND
// Exit status 0 = every check passed; sanitizer reports abort the run (halt_on_error).
#include "../../corda_amd/csrc/cv_api.cpp"

#include <cstdio>
#include <cstdlib>

extern "C" {
// launcher stubs: nothing in this test reaches the device
hipError_t cvk_verify(const CvkPlan *, uint32_t, const uint8_t *, const uint8_t *, const uint8_t *, const uint64_t *,
                      const uint32_t *, uint64_t *, uint8_t *, uint32_t *, uint8_t *, uint32_t *, uint32_t, hipStream_t,
                      hipEvent_t *, const CvkSplit *, const CvkPrepOverlap *) { return hipErrorNoDevice; }
hipError_t cvk_sign(uint32_t, const uint8_t *, const uint8_t *, const uint64_t *, const uint32_t *, uint8_t *, uint8_t *,
                    hipStream_t) { return hipErrorNoDevice; }
hipError_t cvk_pmt_verify(uint32_t, const uint8_t *, const uint32_t *, const uint32_t *, const uint8_t *, const uint32_t *,
                          const uint8_t *, const uint8_t *, const uint32_t *, uint32_t *, uint8_t *, uint8_t *, uint8_t *,
                          hipStream_t) { return hipErrorNoDevice; }
hipError_t cvk_merkle(uint32_t, uint32_t, uint32_t, const uint8_t *, const uint64_t *, const uint32_t *, const uint32_t *,
                      uint32_t *, uint8_t *, uint8_t *, hipStream_t) { return hipErrorNoDevice; }
hipError_t cvk_tx_sig_refs(uint32_t, uint32_t, uint32_t, uint32_t, const uint32_t *, uint64_t *, uint32_t *, hipStream_t) {
    return hipErrorNoDevice;
}
hipError_t cvk_tx_verdicts(uint32_t, uint32_t, const uint32_t *, const uint8_t *, const uint64_t *, uint8_t *, hipStream_t) {
    return hipErrorNoDevice;
}
hipError_t cvk_calibrate(uint32_t, int, uint32_t, void *, hipStream_t) { return hipErrorNoDevice; }
hipError_t cvk_mad_clock(uint32_t, uint32_t, uint64_t *, hipStream_t) { return hipErrorNoDevice; }
int cvk_tri_zc_ok(const CvkPlan *, uint32_t, uint32_t) { return 0; }
hipError_t cvk_verify_tri_zc(const CvkPlan *, uint32_t, const uint8_t *, const uint8_t *, const uint8_t *, const uint64_t *,
                             const uint32_t *, uint8_t *, uint8_t *, uint32_t *, uint8_t *, uint32_t *, uint32_t,
                             hipStream_t, const void *, void *, size_t) {
    return hipErrorNoDevice;
}
hipError_t cvk_prepare(hipStream_t) { return hipErrorNoDevice; }
hipError_t cvk_keyprep(uint32_t, const uint8_t *, const uint32_t *, uint32_t *, uint32_t *, uint8_t *, hipStream_t) {
    return hipErrorNoDevice;
}
hipError_t cvk_verify_keyed(const CvkPlan *, uint32_t, const uint8_t *, const uint32_t *, const uint32_t *, const uint32_t *,
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
    for (size_t n : {0ul, 1ul, 63ul, 64ul, 65ul, 1000ul, 1025ul, 5000ul, 70000ul, 300001ul}) {
        for (size_t pool : {1ul, 7ul, 64ul, 300ul, 100000ul}) {
            std::vector<uint8_t> keys_pool(32 * pool);
            for (auto &b : keys_pool) b = (uint8_t)rnd();
            std::vector<uint8_t> pk(32 * std::max<size_t>(n, 1));
            for (size_t i = 0; i < n; i++) std::memcpy(&pk[32 * i], &keys_pool[32 * (rnd() % pool)], 32);
            for (int threads : {1, 4}) {
                std::unique_ptr<WorkerPool> wp(threads > 1 ? new WorkerPool(threads - 1) : nullptr);
                std::vector<uint8_t> keys;
                std::vector<uint32_t> idx;
                const bool took = dedupe_keys(n, pk.data(), keys, idx, wp.get());
                if (n < 64) CHECK(!took);
                if (n >= 64 && pool * 8 <= n / 2 && pool <= 300) CHECK(took);   // clearly repeated: keyed
                if (!took) continue;
                const size_t nk = keys.size() / 32;
                CHECK(idx.size() == n);
                CHECK(8 * nk <= n);
                for (size_t i = 0; i < n; i++) {
                    CHECK(idx[i] < nk);
                    if (idx[i] < nk) CHECK(std::memcmp(&keys[32 * idx[i]], &pk[32 * i], 32) == 0);
                }
                // distinct keys are distinct, in first-seen order
                std::vector<uint8_t> seen(nk, 0);
                uint32_t next = 0;
                for (size_t i = 0; i < n; i++)
                    if (idx[i] < nk && !seen[idx[i]]) {
                        CHECK(idx[i] == next);
                        seen[idx[i]] = 1;
                        next++;
                    }
            }
        }
    }
    // keys that differ in one byte only must not collide in the dedupe
    const size_t n = 4096;
    std::vector<uint8_t> pk(32 * n, 0xAB);
    for (size_t i = 0; i < n; i++) pk[32 * i + 31] = (uint8_t)(i / 16);   // 16 per key, 256 keys
    std::vector<uint8_t> keys;
    std::vector<uint32_t> idx;
    CHECK(dedupe_keys(n, pk.data(), keys, idx, nullptr));
    CHECK(keys.size() / 32 == 256);
    // the gate: a large distinct-keyed batch is declined, a pooled one accepted
    std::vector<uint8_t> big(32 * 200000);
    for (auto &b : big) b = (uint8_t)rnd();
    CHECK(!dedupe_gate(200000, big.data()));
    for (size_t i = 0; i < 200000; i++) std::memcpy(&big[32 * i], &big[32 * (rnd() % 1000)], 32);
    CHECK(dedupe_gate(200000, big.data()));
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
            const Stage stk = stage_plan(b, e, off.data(), len.data(), nullptr, true);
            CHECK(stk.keyed && stk.o_kidx == 0 && stk.o_sig == al16((e - b) * 4) && stk.lo == st.lo && stk.hi == st.hi);
            CHECK(st.lo == st1.lo && st.hi == st1.hi && st.total == st1.total && st.compact == st1.compact);
            if (e - b >= 64) CHECK(st.compact == scattered);
            std::vector<uint8_t> h(st.total + 64, 0xEE);
            stage_pack(st, h.data(), b, pk.data(), nullptr, sig.data(), arena.data(), off.data(), len.data(), &pool, [] {});
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

// Merkle staging of transactions [t0, t1): leaf offsets not monotone (the arena holds the leaves in reverse
// order, with gaps), empty transactions, the compact (scattered) form
static void test_mstage(bool scattered) {
    const size_t ntx = 700;
    std::vector<uint32_t> txb(ntx + 1, 0);
    for (size_t t = 0; t < ntx; t++) txb[t + 1] = txb[t] + (uint32_t)(t % 9 == 0 ? 0 : rnd() % 8);
    const size_t nl = txb[ntx];
    std::vector<uint32_t> len(nl);
    std::vector<uint64_t> off(nl);
    const size_t arena_size = scattered ? (16u << 20) : nl * 800 + 64;
    std::vector<uint8_t> arena(arena_size);
    for (auto &b : arena) b = (uint8_t)rnd();
    uint64_t pos = arena_size - 8;
    for (size_t i = 0; i < nl; i++) {
        len[i] = (uint32_t)(rnd() % 700);
        if (scattered) {
            off[i] = rnd() % (arena_size - 701);
        } else {
            pos -= len[i] + rnd() % 5;
            off[i] = pos;                                    // decreasing offsets
        }
    }
    WorkerPool pool(2);
    for (size_t t0 : {0ul, 1ul, 350ul}) {
        for (size_t t1 : {t0 + 1, t0 + 9, ntx}) {
            if (t1 > ntx || t1 <= t0) continue;
            const MStage st = mstage_plan(t0, t1, txb.data(), off.data(), len.data(), &pool);
            CHECK(st.l0 == txb[t0] && st.l1 == txb[t1]);
            std::vector<uint8_t> h(st.total + 64, 0xEE);
            mstage_pack(st, h.data(), txb.data(), arena.data(), off.data(), len.data(), &pool);
            CHECK(h[st.total] == 0xEE);
            const uint64_t *hoff = reinterpret_cast<const uint64_t *>(h.data() + st.o_off);
            const uint32_t *hlen = reinterpret_cast<const uint32_t *>(h.data() + st.o_len);
            const uint32_t *htx = reinterpret_cast<const uint32_t *>(h.data() + st.o_txb);
            for (size_t t = t0; t <= t1; t++) CHECK(htx[t - t0] == txb[t]);
            for (size_t i = st.l0; i < st.l1; i++) {
                CHECK(hlen[i - st.l0] == len[i]);
                const uint64_t rel = hoff[i - st.l0] - st.lo;
                CHECK(rel + len[i] <= st.hi - st.lo);
                CHECK(std::memcmp(h.data() + st.o_ar + rel, &arena[off[i]], len[i]) == 0);
            }
            if (st.l1 - st.l0 > 64) CHECK(st.compact == scattered);
        }
    }
}

// Routing: shards of every call cover [0, n) exactly (starts at multiples of 64), a device never runs two
// shards at once (its lock), and the load counts return to zero; threads > 1: concurrent callers
// (VERDICT r3 item 3 — 4 threads x 200 interleaved calls on a 4-device context, host logic only; under
// ThreadSanitizer in san_host_tsan).
static void test_dispatch(size_t ndev, int nthreads, int calls) {
    cv_ctx ctx;
    for (size_t k = 0; k < ndev; k++) {
        ctx.devs.emplace_back(new Device());
        ctx.devs.back()->ordinal = (int)k;
    }
    ctx.opt[CV_OPT_SHARD_MIN].store(1024);
    ctx.opt[CV_OPT_SPREAD_MIN].store(65536);
    std::vector<std::atomic<int>> busy(ndev);
    std::atomic<int> fails{0};
    auto caller = [&](int t) {
        uint64_t x = 0x1234567ull + (uint64_t)t * 7919;
        for (int c = 0; c < calls; c++) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            static const size_t sizes[] = {1, 64, 100, 1024, 4096, 5000, 9000, 40000, 70001};
            const size_t n = sizes[(x >> 33) % 9];
            std::mutex mu;
            std::vector<std::pair<size_t, size_t>> got;
            const Opts o = ctx.opts();
            const int rc = dispatch(&ctx, o, n, 64, [&](Device &d, size_t b, size_t e, int threads) {
                const size_t k = dev_index(&ctx, d);
                if (busy[k].exchange(1) != 0) fails++;          // two shards on one device at once
                std::this_thread::yield();
                {
                    std::lock_guard<std::mutex> g(mu);
                    got.push_back({b, e});
                }
                busy[k].store(0);
                return threads >= 1 ? CV_OK : CV_E_ARGS;
            });
            if (rc != CV_OK) fails++;
            std::sort(got.begin(), got.end());
            size_t p = 0;
            for (auto &r : got) {
                if (r.first != p || r.first % 64) fails++;
                p = r.second;
            }
            if (p != n) fails++;
            if (n <= 1024 && got.size() != 1) fails++;          // small batches go whole to one device
            if (n >= 65536 && ndev > 1 && got.size() != ndev) fails++;   // throughput batches spread
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++) th.emplace_back(caller, t);
    for (auto &t : th) t.join();
    CHECK(fails.load() == 0);
    for (auto &d : ctx.devs) CHECK(d->load.load() == 0);
    for (auto &d : ctx.devs) d->stream = nullptr;
    ctx.devs.clear();
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

// a pipelined call whose finish fails reports the error to its own cv_wait, also when a later call
// reusing its output (pipe_out) or an error path's drain ran the finish; finished tickets pruned from the live
// map keep their result.  Device ordinal 4095 does not exist, so every finish fails at hipSetDevice.
static void test_failed_finish_reaches_waiter() {
    cv_ctx ctx;
    ctx.devs.emplace_back(new Device());
    Device &d = *ctx.devs[0];
    d.ordinal = 4095;
    d.out[0].pending = true;
    d.out[0].ticketed = true;                              // (as the async entry points mark a ticketed call)
    d.out[0].gen = 1;
    const uint64_t t1 = ticket_add(&ctx, {Part{0, 0, 1}});
    d.out_next = 0;
    {
        int k = -1;
        std::unique_lock<std::mutex> lk;
        PipeOut &po = pipe_out(d, &k, lk);                 // a later call takes output 0: finishes call 1
        CHECK(k == 0 && !po.pending);
        po.pending = true;
        po.ticketed = true;
        po.gen = 2;
    }
    const uint64_t t2 = ticket_add(&ctx, {Part{0, 0, 2}});
    CHECK(cv_wait(&ctx, t1) == CV_E_HIP);                  // call 1's error, although its output was reused
    CHECK(cv_wait(&ctx, t2) == CV_E_HIP);                  // call 2 finishes (and fails) in its own wait
    CHECK(cv_wait(&ctx, t1) == CV_E_ARGS);                 // a ticket is waited once
    // 100 calls, each output reused by the next: once 64 tickets are live the finished ones are pruned with
    // their result, and every one of them still reports its error
    std::vector<uint64_t> tk;
    for (uint64_t g = 10; g < 110; g++) {
        int k = -1;
        std::unique_lock<std::mutex> lk;
        PipeOut &po = pipe_out(d, &k, lk);
        po.pending = true;
        po.ticketed = true;
        po.gen = g;
        lk.unlock();
        tk.push_back(ticket_add(&ctx, {Part{0, (uint64_t)k, g}}));
    }
    CHECK(ctx.tickets.size() < 64 && !ctx.tickets_done.empty());
    for (uint64_t t : tk) CHECK(cv_wait(&ctx, t) == CV_E_HIP);
    CHECK(ctx.tickets.empty() && ctx.tickets_done.empty());
    // a ticketed call's failure is not evicted by later failing SYNCHRONOUS calls on the same output
    // (they return their error themselves and record nothing): 200 of them, then the ticket still reports its own
    {
        int k = -1;
        std::unique_lock<std::mutex> lk;
        PipeOut &po = pipe_out(d, &k, lk);
        po.pending = true;
        po.ticketed = true;
        po.gen = 500;
        lk.unlock();
        const uint64_t ta = ticket_add(&ctx, {Part{0, (uint64_t)k, 500}});
        size_t before = 0;
        for (PipeOut &o : d.out) before += o.failed.size();
        for (uint64_t g = 501; g < 701; g++) {
            std::unique_lock<std::mutex> lk2;
            int k2 = -1;
            PipeOut &p2 = pipe_out(d, &k2, lk2);              // finishes (and fails) the call before on this output
            p2.pending = true;                              // an unticketed (synchronous) call
            p2.gen = g;
            CHECK(pipe_finish(d, p2) == CV_E_HIP);
        }
        size_t recorded = 0;
        for (PipeOut &o : d.out) recorded += o.failed.size();
        CHECK(recorded == before + 1);                      // call 500's; the synchronous failures were not recorded
        CHECK(cv_wait(&ctx, ta) == CV_E_HIP);
    }
    ctx.devs.clear();
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
    for (size_t ndev : {1ul, 2ul, 3ul, 8ul}) test_dispatch(ndev, 1, 60);
    test_dispatch(4, 4, 200);        // 4 threads x 200 interleaved calls, 4 devices
    if (!threads_only) {
        test_dedupe();
        test_stage(false, 3001);
        test_stage(true, 3001);
        test_stage(false, 140001);   // several range-scan slices
        test_mstage(false);
        test_mstage(true);
        test_pipe_cuts();
        test_tx_verdicts();
        test_failed_finish_reaches_waiter();
        test_abi_guards();
    }
    if (g_fail) {
        std::fprintf(stderr, "san_host: %d checks failed\n", g_fail);
        return 1;
    }
    std::printf("san_host: all checks passed%s\n", threads_only ? " (thread tests)" : "");
    return 0;
}
