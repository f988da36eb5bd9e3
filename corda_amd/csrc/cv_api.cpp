// cv_api.cpp — the C-ABI (include/cordaverify.h): contexts, per-device workspaces, host-buffer
// batches sharded over the context's GPUs (one host thread + one HIP stream per device), and the
// device-resident entry points used by bench.py.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstring>
#include <chrono>
#include <mutex>
#include <random>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/cordaverify.h"

extern "C" {
hipError_t cvk_verify(uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off,
                      const uint32_t *len, uint64_t *bitmap, uint8_t *status, uint32_t *ws_hs, uint32_t *ws_tab,
                      uint32_t *ws_R, uint8_t *ws_ok, uint32_t *ws_dig, uint32_t ws_cap, hipStream_t stream,
                      hipEvent_t *ev);
hipError_t cvk_sign(uint32_t n, const uint8_t *seed, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                    uint8_t *pk, uint8_t *sig, hipStream_t stream);
hipError_t cvk_pmt_verify(uint32_t ntrees, const uint8_t *kind, const uint32_t *left, const uint32_t *right,
                          const uint8_t *leaf_hash, const uint32_t *tree_begin, const uint8_t *root, const uint8_t *check,
                          const uint32_t *check_begin, uint32_t *dig, uint8_t *flag, uint8_t *verdict, uint8_t *status,
                          hipStream_t stream);
hipError_t cvk_merkle(uint32_t ntx, uint32_t nleaves, const uint8_t *arena, const uint64_t *leaf_off,
                      const uint32_t *leaf_len, const uint32_t *tx_begin, uint32_t *leaf_digest, uint8_t *ids,
                      uint8_t *status, hipStream_t stream);
hipError_t cvk_calibrate(uint32_t iters, int which, uint32_t blocks, void *scratch, hipStream_t stream);
hipError_t cvk_prep_probe(uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off,
                          const uint32_t *len, uint32_t *ws_dig, uint32_t *ws_tab, uint32_t ws_cap, uint64_t *stamps,
                          hipStream_t stream);
hipError_t cvk_mad_clock(uint32_t iters, uint32_t blocks, uint64_t *out, hipStream_t stream);
uint32_t cvk_get_tri_max(void);
hipError_t cvk_prepare(hipStream_t stream);
hipError_t cvk_keyprep(uint32_t nk, const uint8_t *keys, const uint32_t *slots, uint32_t *scratch, uint32_t *ktab_pool,
                       uint8_t *kok_pool, hipStream_t stream);
hipError_t cvk_verify_keyed(uint32_t n, const uint8_t *keys, const uint32_t *key_index, const uint32_t *slot_of_key,
                            const uint32_t *ktab_pool, const uint8_t *kok_pool, const uint8_t *sig,
                            const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint64_t *bitmap,
                            uint8_t *status, uint32_t *ws_hs, uint32_t *ws_R, uint8_t *ws_ok, uint32_t ws_cap,
                            hipStream_t stream, hipEvent_t *ev);
}

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return e;
        }
        cap = want;
        return hipSuccess;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Pinned (page-locked) host staging buffer: the host-buffer API packs a call's inputs into it so one
// DMA moves them (pageable hipMemcpyAsync stages every copy through the runtime's own buffers — five
// input copies cost ~0.1 ms of a 0.4-0.7 ms notary batch, tools/notary_probe.py).
struct PinBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e != hipSuccess) {
            p = nullptr;
            return e;
        }
        cap = want;
        return hipSuccess;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Device-resident per-key comb tables (keyed verify), content-addressed by the
// 32 key bytes.  A key's tables are computed once (cv_keyprep_kernel) and reused by every later
// batch on that device; when the pool is full it is emptied (epoch reset) before new keys go in.
// Key bytes come from untrusted submitters (and invalid keys are deduped before decoding), so the
// host hash tables hash all 32 bytes with a per-process random seed: a batch of keys that share some
// bytes cannot pile into one probe chain.  64-bit multiply-xorshift mixing of the four words, each
// folded with its own seed (a keyed hash in the wyhash / murmur-finaliser family: not cryptographic,
// only unpredictable to the submitter).
static uint64_t key_seed(int k) {
    static const std::array<uint64_t, 5> seeds = [] {
        std::random_device rd;
        std::array<uint64_t, 5> s{};
        for (auto &x : s) x = ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
        return s;
    }();
    return seeds[k];
}
static inline uint64_t mix64(uint64_t x) {
    x ^= x >> 32;
    x *= 0xd6e8feb86659fd93ull;
    x ^= x >> 32;
    x *= 0xd6e8feb86659fd93ull;
    x ^= x >> 32;
    return x;
}
static inline uint64_t key_hash32(const uint8_t *k) {
    uint64_t w[4];
    std::memcpy(w, k, 32);
    uint64_t h = key_seed(4);
    for (int i = 0; i < 4; i++) h = mix64(h ^ (w[i] + key_seed(i)) * 0x9E3779B97F4A7C15ull) + (uint64_t)i;
    return h;
}
struct KeyHash {
    size_t operator()(const std::array<uint8_t, 32> &k) const { return (size_t)key_hash32(k.data()); }
};
struct KeyCache {
    DevBuf ktab, kok, keys, slots, slot_of_key, key_index, scratch;
    uint32_t cap = 0;
    std::unordered_map<std::array<uint8_t, 32>, uint32_t, KeyHash> map;
    uint64_t hits = 0, misses = 0, resets = 0;
};

struct Device {
    int ordinal = 0;
    hipStream_t stream = nullptr;
    DevBuf pk, sig, arena, off, len, bitmap, status, seed, tx_begin, digest, ids;
    DevBuf packed;                       // host-buffer verify: pk | sig | off | len | arena in one block
    PinBuf pin_in, pin_out;              // its pinned host staging (inputs; bitmap | status)
    DevBuf pmt;                          // partial Merkle trees: inputs, outputs and workspace, packed
    DevBuf ws_hs, ws_tab, ws_R, ws_ok, ws_dig;   // verify workspace per signature: hs 64 B, 2 tables 2 x 1440 B,
                                         // R record 128 B, ok 1 B, half-size digits 260 B
    uint32_t ws_cap = 0;
    KeyCache kc;
    // the last stream that used the shared workspace / key pool, and an event after its use
    hipStream_t ws_last = nullptr;
    hipEvent_t ws_ev = nullptr;
};

// key-table pool capacity per device (keys); 66 KB of tables per key (1.1 GB at the default; the pool
// grows to a call's distinct keys when they exceed it)
constexpr uint32_t kDefaultKeyCap = 1u << 14;
constexpr size_t kKtabBytes = 16512 * 4;  // CV_KTAB_WORDS: 4 comb rows x 129 affine entries x 128 B
constexpr size_t kTabBytes = 9 * 40 * 4;  // CV_TAB_WORDS: k*P, k = 0..8, cached form (cv_verify.h)
// cv_ed25519_verify_batch dedupes keys on the host up to this batch size, and takes the keyed
// (per-key comb) path when the batch has at least eight signatures per distinct key on average (a key's
// 66 KB of tables cost about as much as 7 plain verifies to build; cached keys cost nothing)
constexpr size_t kAutoKeyedMax = 1u << 18;

// Verify workspace capacity: batches above it run in chunks of this many signatures (~13.4 GB of
// workspace at 2^22; same-box A/B at 8M signatures: 2^21 73.2, 2^22 72.4, 2^23 72.4 ms -- fewer
// chunk tails to drain; whole-round chunks of 1,966,080 were slower, 73.4 ms).
constexpr uint32_t kVerifyChunk = 1u << 22;

hipError_t ensure_verify_ws(Device &d, size_t n) {
    uint32_t want = (uint32_t)std::min<size_t>(kVerifyChunk, (n + 511) / 512 * 512);
    if (want <= d.ws_cap) return hipSuccess;
    hipError_t e;
    if ((e = d.ws_hs.ensure((size_t)want * 64)) != hipSuccess) return e;
    if ((e = d.ws_tab.ensure((size_t)want * 2 * kTabBytes)) != hipSuccess) return e;   // k*(-A), k*R
    if ((e = d.ws_R.ensure((size_t)want * 128)) != hipSuccess) return e;
    if ((e = d.ws_ok.ensure((size_t)want)) != hipSuccess) return e;
    if ((e = d.ws_dig.ensure((size_t)want * 73 * 4)) != hipSuccess) return e;   // CV_HS_DIGWORDS
    d.ws_cap = want;
    return hipSuccess;
}

// Every use of a device's shared state (the verify workspace, the key pool) is ordered across
// streams: a launch group enqueued on stream s first waits for the previous group when that ran on
// another stream (ws_begin), and marks its own end (ws_end).  Device-pointer calls may therefore be
// made on any streams; they serialise on the workspace instead of racing on it.  Callers hold
// ctx->mu around ws_begin .. ws_end.
hipError_t ws_begin(Device &d, hipStream_t s) {
    hipError_t e = hipSuccess;
    if (!d.ws_ev && (e = hipEventCreateWithFlags(&d.ws_ev, hipEventDisableTiming)) != hipSuccess) return e;
    if (d.ws_last && d.ws_last != s) e = hipStreamWaitEvent(s, d.ws_ev, 0);
    return e;
}
hipError_t ws_end(Device &d, hipStream_t s) {
    d.ws_last = s;
    return hipEventRecord(d.ws_ev, s);
}

hipError_t launch_verify(Device &d, uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                         const uint64_t *off, const uint32_t *len, uint64_t *bitmap, uint8_t *status, hipStream_t s,
                         hipEvent_t *ev = nullptr) {
    hipError_t e = ensure_verify_ws(d, n);
    if (e == hipSuccess) e = ws_begin(d, s);
    if (e != hipSuccess) return e;
    e = cvk_verify(n, pk, sig, arena, off, len, bitmap, status, d.ws_hs.as<uint32_t>(), d.ws_tab.as<uint32_t>(),
                   d.ws_R.as<uint32_t>(), d.ws_ok.as<uint8_t>(), d.ws_dig.as<uint32_t>(), d.ws_cap, s, ev);
    const hipError_t e2 = ws_end(d, s);
    return e != hipSuccess ? e : e2;
}

int hip_rc(hipError_t e) {
    if (e == hipSuccess) return CV_OK;
    if (e == hipErrorOutOfMemory) return CV_E_OOM;
    return CV_E_HIP;
}

#define CV_TRY(expr)                        \
    do {                                    \
        hipError_t e_ = (expr);             \
        if (e_ != hipSuccess) return hip_rc(e_); \
    } while (0)

}  // namespace

struct cv_ctx {
    std::vector<Device> devs;
    std::mutex mu;
    uint32_t key_cap = kDefaultKeyCap;
};

extern "C" {

const char *cv_version(void) { return "cordaverify-mi355x 0.1 (gfx950)"; }

const char *cv_strerror(int code) {
    switch (code) {
        case CV_OK: return "ok";
        case CV_E_NO_DEVICE: return "no HIP device matches the device mask";
        case CV_E_HIP: return "HIP runtime error";
        case CV_E_ARGS: return "invalid argument";
        case CV_E_OOM: return "device out of memory";
        case CV_E_TOO_LARGE: return "batch shard exceeds 2^32-1 records";
        default: return "unknown error";
    }
}

// Test knob (internal, not in the header): every device of the next cv_open appears k times in the
// context — k independent Device slots (own stream, buffers, workspace, key pool) on one GPU — so the
// multi-device host path (for_each_shard: one thread per slot, 64-aligned shard ranges, per-slot
// dedupe and key pools) runs and is tested on a one-GPU box.  0 / 1 = off.
static int g_virtual_devices = 1;
void cvk_set_virtual_devices(int k) { g_virtual_devices = (k >= 1 && k <= 16) ? k : 1; }

int cv_open(uint32_t device_mask, cv_ctx **out) {
    if (!out) return CV_E_ARGS;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return CV_E_NO_DEVICE;
    cv_ctx *ctx = new (std::nothrow) cv_ctx();
    if (!ctx) return CV_E_OOM;
    for (int d = 0; d < count && d < 32; d++) {
        if (device_mask && !(device_mask & (1u << d))) continue;
        for (int v = 0; v < g_virtual_devices; v++) {
            Device dev;
            dev.ordinal = d;
            if (hipSetDevice(d) != hipSuccess ||
                hipStreamCreateWithFlags(&dev.stream, hipStreamNonBlocking) != hipSuccess) {
                cv_close(ctx);
                return CV_E_HIP;
            }
            ctx->devs.push_back(dev);
            // Per-device basepoint rows (16.8 MB, built once per process): eager, so the first
            // verify is not charged for them and no later call synchronises to build them.
            if (v == 0 && cvk_prepare(dev.stream) != hipSuccess) {
                cv_close(ctx);
                return CV_E_HIP;
            }
        }
    }
    if (ctx->devs.empty()) {
        delete ctx;
        return CV_E_NO_DEVICE;
    }
    *out = ctx;
    return CV_OK;
}

void cv_close(cv_ctx *ctx) {
    if (!ctx) return;
    for (Device &d : ctx->devs) {
        (void)hipSetDevice(d.ordinal);
        if (d.stream) (void)hipStreamSynchronize(d.stream);
        for (DevBuf *b : {&d.pk, &d.sig, &d.arena, &d.off, &d.len, &d.bitmap, &d.status, &d.seed, &d.tx_begin,
                          &d.digest, &d.ids, &d.pmt, &d.ws_hs, &d.ws_tab, &d.ws_R, &d.ws_ok, &d.ws_dig, &d.kc.ktab, &d.kc.kok,
                          &d.kc.keys, &d.kc.slots, &d.kc.slot_of_key, &d.kc.key_index, &d.kc.scratch})
            b->release();
        d.packed.release();
        d.pin_in.release();
        d.pin_out.release();
        if (d.ws_ev) (void)hipEventDestroy(d.ws_ev);
        if (d.stream) (void)hipStreamDestroy(d.stream);
    }
    delete ctx;
}

int cv_device_count(const cv_ctx *ctx) { return ctx ? (int)ctx->devs.size() : 0; }

static Device *find_dev(cv_ctx *ctx, int device) {
    for (Device &d : ctx->devs)
        if (d.ordinal == device) return &d;
    return nullptr;
}

// ---------------------------------------------------------------- verify (host buffers)
// One shard [b, e) of a batch on one device.  b is a multiple of 64, so the shard's bitmap words
// are whole words of the caller's bitmap.  The inputs are packed into the device's pinned staging
// buffer (pk | sig | off rebased to the shard's arena range | len | arena bytes, 16-B aligned parts),
// moved by one DMA (two above 1 MB: the first overlaps packing the second part) into one device
// block, verified, and the bitmap (+ status) come back by one DMA.
static inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// Host copies into the pinned staging buffer.  A large batch is packed by a few threads (one core
// copies ~10 GB/s, below what the DMA takes): each segment is cut into >= 512 KB pieces dealt out
// round-robin; `extra` runs on the calling thread meanwhile.
extern "C++" {
struct CopyJob {
    void *dst;
    const void *src;
    size_t len;
};
template <class F> static void par_copy(const std::vector<CopyJob> &jobs, F extra) {
    constexpr size_t kPiece = 512 * 1024;
    constexpr int kThreads = 4;
    size_t total = 0;
    for (const CopyJob &j : jobs) total += j.len;
    if (total < 2 * kPiece) {
        for (const CopyJob &j : jobs)
            if (j.len) std::memcpy(j.dst, j.src, j.len);
        extra();
        return;
    }
    std::vector<CopyJob> pieces;
    for (const CopyJob &j : jobs)
        for (size_t o = 0; o < j.len; o += kPiece)
            pieces.push_back({static_cast<uint8_t *>(j.dst) + o, static_cast<const uint8_t *>(j.src) + o,
                              std::min(kPiece, j.len - o)});
    auto work = [&pieces](int t) {
        for (size_t k = (size_t)t; k < pieces.size(); k += kThreads)
            std::memcpy(pieces[k].dst, pieces[k].src, pieces[k].len);
    };
    std::thread th[kThreads - 1];
    for (int t = 1; t < kThreads; t++) th[t - 1] = std::thread(work, t);
    extra();
    work(0);
    for (auto &x : th) x.join();
}
}  // extern "C++"
static int verify_shard(Device &d, size_t b, size_t e, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                        const uint64_t *off, const uint32_t *len, uint64_t *bitmap, uint8_t *status) {
    const size_t n = e - b;
    if (n == 0) return CV_OK;
    if (n > 0xffffffffull) return CV_E_TOO_LARGE;
    CV_TRY(hipSetDevice(d.ordinal));
    // arena sub-range used by this shard; offsets are rebased to it
    uint64_t lo = UINT64_MAX, hi = 0;
    for (size_t i = b; i < e; i++) {
        lo = std::min<uint64_t>(lo, off[i]);
        hi = std::max<uint64_t>(hi, off[i] + len[i]);
    }
    if (hi < lo) hi = lo;
    const size_t words = (n + 63) / 64;
    const size_t o_pk = 0, o_sig = al16(n * 32), o_off = o_sig + al16(n * 64), o_len = o_off + al16(n * 8);
    const size_t o_ar = o_len + al16(n * 4), total = o_ar + al16(hi - lo + 16);
    const size_t o_bm = 0, o_st = al16(words * 8), total_out = o_st + al16(n);
    CV_TRY(d.pin_in.ensure(total));
    CV_TRY(d.pin_out.ensure(total_out));
    CV_TRY(d.packed.ensure(total));
    CV_TRY(d.bitmap.ensure(total_out));
    hipStream_t s = d.stream;
    // the staging buffers are reused by the next call: the previous call synchronised at its end
    uint8_t *h = d.pin_in.as<uint8_t>();
    uint64_t *hoff = reinterpret_cast<uint64_t *>(h + o_off);
    uint8_t *dv = d.packed.as<uint8_t>();
    // Two-stage staging above 1 MB of keys + signatures: they are packed and their DMA is issued
    // first, so it runs while the offsets, lengths and message bytes are packed (notary 65,536:
    // 1.29-1.34 -> 1.21-1.25 ms p50); below, one DMA (a second DMA's ~6 us would cost more than it hides).
    const bool two_stage = o_off >= ((size_t)1 << 20);
    par_copy({{h + o_pk, pk + b * 32, n * 32}, {h + o_sig, sig + b * 64, n * 64}}, [] {});
    if (two_stage) CV_TRY(hipMemcpyAsync(dv, h, o_off, hipMemcpyHostToDevice, s));
    par_copy({{h + o_len, len + b, n * 4},
              {h + o_ar, hi > lo ? arena + lo : nullptr, (size_t)(hi - lo)}},
             [&] {
                 for (size_t i = 0; i < n; i++) hoff[i] = off[b + i] - lo;
             });
    std::memset(h + o_ar + (hi - lo), 0, 16);
    if (two_stage)
        CV_TRY(hipMemcpyAsync(dv + o_off, h + o_off, total - o_off, hipMemcpyHostToDevice, s));
    else
        CV_TRY(hipMemcpyAsync(dv, h, total, hipMemcpyHostToDevice, s));
    uint8_t *dout = d.bitmap.as<uint8_t>();
    CV_TRY(launch_verify(d, (uint32_t)n, dv + o_pk, dv + o_sig, dv + o_ar, reinterpret_cast<const uint64_t *>(dv + o_off),
                         reinterpret_cast<const uint32_t *>(dv + o_len), reinterpret_cast<uint64_t *>(dout + o_bm),
                         status ? dout + o_st : nullptr, s));
    CV_TRY(hipMemcpyAsync(d.pin_out.p, dout, status ? o_st + n : words * 8, hipMemcpyDeviceToHost, s));
    CV_TRY(hipStreamSynchronize(s));
    std::memcpy(bitmap + b / 64, d.pin_out.as<uint8_t>() + o_bm, words * 8);
    if (status) std::memcpy(status + b, d.pin_out.as<uint8_t>() + o_st, n);
    return CV_OK;
}

}  // extern "C"

// Shards [0, n) over the context's devices (contiguous ranges, multiples of 64) and runs fn per shard.
template <class F> static int for_each_shard(cv_ctx *ctx, size_t n, F fn) {
    const size_t ndev = ctx->devs.size();
    size_t per = (n + ndev - 1) / ndev;
    per = (per + 63) / 64 * 64;
    if (ndev == 1 || n <= 64) return fn(ctx->devs[0], 0, n);
    std::vector<int> rc(ndev, CV_OK);
    std::vector<std::thread> th;
    for (size_t k = 0; k < ndev; k++) {
        const size_t b = std::min(n, k * per), e = std::min(n, b + per);
        if (b >= e) continue;
        th.emplace_back([&, k, b, e] { rc[k] = fn(ctx->devs[k], b, e); });
    }
    for (auto &t : th) t.join();
    for (int r : rc)
        if (r != CV_OK) return r;
    return CV_OK;
}

// ---------------------------------------------------------------- keyed verify (per-key comb tables)
// Makes the keys k (used[k] != 0, or all when used == nullptr) of keys[0..nk) resident in d's key
// pool and fills slot_of_key[k]; one keyprep launch on s computes the tables of the new ones.
static int key_resolve(Device &d, uint32_t cap, size_t nk, const uint8_t *keys, const uint8_t *used,
                       std::vector<uint32_t> &slot_of_key, hipStream_t s) {
    KeyCache &kc = d.kc;
    size_t nused = 0;
    for (size_t k = 0; k < nk; k++) nused += used ? (used[k] != 0) : 1;
    const size_t need = std::max<size_t>(cap, nused);
    if (kc.cap < need) {                      // (re)allocate the pool; resident tables are dropped
        if (need > 0xffffffffull / 2) return CV_E_TOO_LARGE;
        CV_TRY(hipStreamSynchronize(s));
        kc.ktab.release();
        kc.kok.release();
        CV_TRY(kc.ktab.ensure(need * kKtabBytes));
        CV_TRY(kc.kok.ensure(need));
        kc.cap = (uint32_t)need;
        kc.map.clear();
    }
    if (kc.map.size() + nused > kc.cap) {     // epoch reset: every key of this call gets a fresh slot
        kc.map.clear();
        kc.resets++;
    }
    std::vector<uint8_t> miss_keys;
    std::vector<uint32_t> miss_slots;
    std::array<uint8_t, 32> key;
    slot_of_key.assign(nk, 0);
    for (size_t k = 0; k < nk; k++) {
        if (used && !used[k]) continue;
        std::memcpy(key.data(), keys + 32 * k, 32);
        auto it = kc.map.find(key);
        if (it != kc.map.end()) {
            slot_of_key[k] = it->second;
            kc.hits++;
            continue;
        }
        const uint32_t slot = (uint32_t)kc.map.size();
        kc.map.emplace(key, slot);
        slot_of_key[k] = slot;
        miss_keys.insert(miss_keys.end(), key.begin(), key.end());
        miss_slots.push_back(slot);
        kc.misses++;
    }
    if (!miss_slots.empty()) {
        const size_t m = miss_slots.size();
        CV_TRY(kc.keys.ensure(m * 32));
        CV_TRY(kc.slots.ensure(m * 4));
        CV_TRY(kc.scratch.ensure(m * kKtabBytes));
        CV_TRY(hipMemcpyAsync(kc.keys.p, miss_keys.data(), m * 32, hipMemcpyHostToDevice, s));
        CV_TRY(hipMemcpyAsync(kc.slots.p, miss_slots.data(), m * 4, hipMemcpyHostToDevice, s));
        CV_TRY(cvk_keyprep((uint32_t)m, kc.keys.as<uint8_t>(), kc.slots.as<uint32_t>(), kc.scratch.as<uint32_t>(),
                           kc.ktab.as<uint32_t>(), kc.kok.as<uint8_t>(), s));
    }
    return CV_OK;
}

// One shard [b, e) of a keyed host-buffer batch on one device (b a multiple of 64).
static int verify_shard_keyed(uint32_t cap, Device &d, size_t b, size_t e, size_t nkeys, const uint8_t *keys,
                              const uint32_t *key_index, const uint8_t *sig, const uint8_t *arena,
                              const uint64_t *off, const uint32_t *len, uint64_t *bitmap, uint8_t *status) {
    const size_t n = e - b;
    if (n == 0) return CV_OK;
    if (n > 0xffffffffull || nkeys > 0xffffffffull) return CV_E_TOO_LARGE;
    CV_TRY(hipSetDevice(d.ordinal));
    std::vector<uint8_t> used(nkeys, 0);
    uint64_t lo = UINT64_MAX, hi = 0;
    for (size_t i = b; i < e; i++) {
        if (key_index[i] >= nkeys) return CV_E_ARGS;
        used[key_index[i]] = 1;
        lo = std::min<uint64_t>(lo, off[i]);
        hi = std::max<uint64_t>(hi, off[i] + len[i]);
    }
    if (hi < lo) hi = lo;
    hipStream_t s = d.stream;
    CV_TRY(ws_begin(d, s));
    std::vector<uint32_t> sok;
    int rc = key_resolve(d, cap, nkeys, keys, used.data(), sok, s);
    if (rc != CV_OK) return rc;
    const size_t words = (n + 63) / 64;
    KeyCache &kc = d.kc;
    CV_TRY(d.pk.ensure(nkeys * 32));
    CV_TRY(kc.slot_of_key.ensure(nkeys * 4));
    CV_TRY(kc.key_index.ensure(n * 4));
    CV_TRY(d.sig.ensure(n * 64));
    CV_TRY(d.arena.ensure(hi - lo + 16));
    CV_TRY(d.off.ensure(n * 8));
    CV_TRY(d.len.ensure(n * 4));
    CV_TRY(d.bitmap.ensure(words * 8));
    CV_TRY(d.status.ensure(n));
    CV_TRY(hipMemcpyAsync(d.pk.p, keys, nkeys * 32, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(kc.slot_of_key.p, sok.data(), nkeys * 4, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(kc.key_index.p, key_index + b, n * 4, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(d.sig.p, sig + b * 64, n * 64, hipMemcpyHostToDevice, s));
    if (hi > lo) CV_TRY(hipMemcpyAsync(d.arena.p, arena + lo, hi - lo, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(d.off.p, off + b, n * 8, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(d.len.p, len + b, n * 4, hipMemcpyHostToDevice, s));
    CV_TRY(ensure_verify_ws(d, n));
    CV_TRY(cvk_verify_keyed((uint32_t)n, d.pk.as<uint8_t>(), kc.key_index.as<uint32_t>(), kc.slot_of_key.as<uint32_t>(),
                            kc.ktab.as<uint32_t>(), kc.kok.as<uint8_t>(), d.sig.as<uint8_t>(),
                            d.arena.as<uint8_t>() - lo, d.off.as<uint64_t>(), d.len.as<uint32_t>(),
                            d.bitmap.as<uint64_t>(), status ? d.status.as<uint8_t>() : nullptr, d.ws_hs.as<uint32_t>(),
                            d.ws_R.as<uint32_t>(), d.ws_ok.as<uint8_t>(), d.ws_cap, s, nullptr));
    CV_TRY(ws_end(d, s));
    CV_TRY(hipMemcpyAsync(bitmap + b / 64, d.bitmap.p, words * 8, hipMemcpyDeviceToHost, s));
    if (status) CV_TRY(hipMemcpyAsync(status + b, d.status.p, n, hipMemcpyDeviceToHost, s));
    CV_TRY(hipStreamSynchronize(s));
    return CV_OK;
}

// Host-side key dedupe for the plain entry point: keys[] = distinct key bytes, key_index[i] = its
// index.  Returns false when the batch does not repeat keys enough for the keyed path to pay (it
// gives up as soon as more than n/8 distinct keys have been seen).  Flat open addressing on the
// seeded hash of all 32 key bytes (key_hash32), no per-key allocation.
static bool dedupe_keys(size_t n, const uint8_t *pk, std::vector<uint8_t> &keys, std::vector<uint32_t> &key_index) {
    if (n < 64 || n > kAutoKeyedMax) return false;
    // Cheap early out for batches of (nearly) distinct keys: when the first 256 signatures already
    // carry more than 192 distinct keys the batch is taken as distinct-keyed without hashing the
    // rest (a performance guess only: both paths return the same verdicts).
    if (n > 1024) {
        constexpr int kS = 256;
        uint32_t tag[2 * kS];
        std::fill(tag, tag + 2 * kS, UINT32_MAX);
        int distinct = 0;
        for (int i = 0; i < kS; i++) {
            const uint8_t *k = pk + 32 * (size_t)i;
            uint32_t bkt = key_hash32(k) & (2 * kS - 1);
            for (;;) {
                if (tag[bkt] == UINT32_MAX) {
                    tag[bkt] = (uint32_t)i;
                    distinct++;
                    break;
                }
                if (std::memcmp(pk + 32 * (size_t)tag[bkt], k, 32) == 0) break;
                bkt = (bkt + 1) & (2 * kS - 1);
            }
        }
        if (distinct > 3 * kS / 4) return false;
    }
    size_t cap = 64;
    while (cap < 2 * n) cap <<= 1;
    std::vector<uint32_t> first(cap, UINT32_MAX);   // bucket -> first signature with that key
    std::vector<uint32_t> uid(cap, 0);              // bucket -> distinct-key index
    key_index.resize(n);
    uint32_t nuniq = 0;
    std::vector<uint32_t> uniq_sig;
    uniq_sig.reserve(n / 2 + 1);
    for (size_t i = 0; i < n; i++) {
        const uint8_t *k = pk + 32 * i;
        size_t bkt = (size_t)key_hash32(k) & (cap - 1);
        for (;;) {
            const uint32_t f = first[bkt];
            if (f == UINT32_MAX) {
                first[bkt] = (uint32_t)i;
                uid[bkt] = nuniq;
                key_index[i] = nuniq++;
                uniq_sig.push_back((uint32_t)i);
                if (8 * (size_t)nuniq > n) return false;   // fewer than eight signatures per key
                break;
            }
            if (std::memcmp(pk + 32 * (size_t)f, k, 32) == 0) {
                key_index[i] = uid[bkt];
                break;
            }
            bkt = (bkt + 1) & (cap - 1);
        }
    }
    keys.resize(32 * (size_t)nuniq);
    for (uint32_t u = 0; u < nuniq; u++) std::memcpy(keys.data() + 32 * (size_t)u, pk + 32 * (size_t)uniq_sig[u], 32);
    return true;
}

extern "C" {

// Diagnostic: the host-side key dedupe of cv_ed25519_verify_batch on its own (no device needed).
int cv_diag_dedupe_keys(size_t n, const uint8_t *pk, uint32_t *key_index, size_t *nkeys) {
    if (!pk || !key_index || !nkeys) return CV_E_ARGS;
    std::vector<uint8_t> keys;
    std::vector<uint32_t> idx;
    if (!dedupe_keys(n, pk, keys, idx)) {
        *nkeys = 0;
        return 0;
    }
    std::memcpy(key_index, idx.data(), n * sizeof(uint32_t));
    *nkeys = keys.size() / 32;
    return 1;
}

int cv_ed25519_verify_batch(cv_ctx *ctx, size_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg_arena,
                            const uint64_t *msg_off, const uint32_t *msg_len, uint64_t *verdict_bitmap,
                            uint8_t *status) {
    if (!ctx) return CV_E_ARGS;
    if (n == 0) return CV_OK;
    if (!pk || !sig || !msg_off || !msg_len || !verdict_bitmap) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    std::vector<uint8_t> keys;
    std::vector<uint32_t> key_index;
    // Batches the tri-chain latency form takes (n <= 4,096) stay on the plain path whatever their keys:
    // there the per-signature chain is the latency, and the tri chain (128 doublings spread over four
    // quads, decodes beside the scalars) beats the keyed comb chain (hash, 60 quad doublings + 96
    // additions, then the inversion): notary batch of 4,096 with 64 signers 0.47 vs 0.34 ms distinct.
    if (n > cvk_get_tri_max() && dedupe_keys(n, pk, keys, key_index)) {
        const size_t nk = keys.size() / 32;
        return for_each_shard(ctx, n, [&](Device &d, size_t b, size_t e) {
            return verify_shard_keyed(ctx->key_cap, d, b, e, nk, keys.data(), key_index.data(), sig, msg_arena, msg_off,
                                      msg_len, verdict_bitmap, status);
        });
    }
    return for_each_shard(ctx, n, [&](Device &d, size_t b, size_t e) {
        return verify_shard(d, b, e, pk, sig, msg_arena, msg_off, msg_len, verdict_bitmap, status);
    });
}

int cv_ed25519_verify_batch_keyed(cv_ctx *ctx, size_t n, size_t nkeys, const uint8_t *keys, const uint32_t *key_index,
                                  const uint8_t *sig, const uint8_t *msg_arena, const uint64_t *msg_off,
                                  const uint32_t *msg_len, uint64_t *verdict_bitmap, uint8_t *status) {
    if (!ctx) return CV_E_ARGS;
    if (n == 0) return CV_OK;
    if (!keys || !key_index || !sig || !msg_off || !msg_len || !verdict_bitmap || nkeys == 0) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    return for_each_shard(ctx, n, [&](Device &d, size_t b, size_t e) {
        return verify_shard_keyed(ctx->key_cap, d, b, e, nkeys, keys, key_index, sig, msg_arena, msg_off, msg_len,
                                  verdict_bitmap, status);
    });
}

int cv_key_cache_reserve(cv_ctx *ctx, size_t max_keys) {
    if (!ctx || max_keys == 0 || max_keys > 0x7fffffffull) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    ctx->key_cap = (uint32_t)max_keys;
    return CV_OK;
}

int cv_key_cache_stats(cv_ctx *ctx, int device, uint64_t *out4) {
    if (!ctx || !out4) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    Device *d = find_dev(ctx, device);
    if (!d) return CV_E_ARGS;
    out4[0] = d->kc.map.size();
    out4[1] = d->kc.cap;
    out4[2] = d->kc.hits;
    out4[3] = d->kc.misses;
    return CV_OK;
}

// ---------------------------------------------------------------- sign (host buffers)
static int sign_shard(Device &d, size_t b, size_t e, const uint8_t *seed, const uint8_t *arena, const uint64_t *off,
                      const uint32_t *len, uint8_t *pk, uint8_t *sig) {
    const size_t n = e - b;
    if (n == 0) return CV_OK;
    if (n > 0xffffffffull) return CV_E_TOO_LARGE;
    CV_TRY(hipSetDevice(d.ordinal));
    uint64_t lo = UINT64_MAX, hi = 0;
    for (size_t i = b; i < e; i++) {
        lo = std::min<uint64_t>(lo, off[i]);
        hi = std::max<uint64_t>(hi, off[i] + len[i]);
    }
    if (hi < lo) hi = lo;
    CV_TRY(d.seed.ensure(n * 32));
    CV_TRY(d.arena.ensure(hi - lo + 16));
    CV_TRY(d.off.ensure(n * 8));
    CV_TRY(d.len.ensure(n * 4));
    CV_TRY(d.pk.ensure(n * 32));
    CV_TRY(d.sig.ensure(n * 64));
    hipStream_t s = d.stream;
    CV_TRY(hipMemcpyAsync(d.seed.p, seed + b * 32, n * 32, hipMemcpyHostToDevice, s));
    if (hi > lo) CV_TRY(hipMemcpyAsync(d.arena.p, arena + lo, hi - lo, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(d.off.p, off + b, n * 8, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(d.len.p, len + b, n * 4, hipMemcpyHostToDevice, s));
    CV_TRY(cvk_sign((uint32_t)n, d.seed.as<uint8_t>(), d.arena.as<uint8_t>() - lo, d.off.as<uint64_t>(),
                    d.len.as<uint32_t>(), d.pk.as<uint8_t>(), d.sig.as<uint8_t>(), s));
    CV_TRY(hipMemcpyAsync(pk + b * 32, d.pk.p, n * 32, hipMemcpyDeviceToHost, s));
    CV_TRY(hipMemcpyAsync(sig + b * 64, d.sig.p, n * 64, hipMemcpyDeviceToHost, s));
    CV_TRY(hipStreamSynchronize(s));
    return CV_OK;
}

int cv_ed25519_sign_batch(cv_ctx *ctx, size_t n, const uint8_t *seed, const uint8_t *msg_arena,
                          const uint64_t *msg_off, const uint32_t *msg_len, uint8_t *pk_out, uint8_t *sig_out) {
    if (!ctx) return CV_E_ARGS;
    if (n == 0) return CV_OK;
    if (!seed || !msg_off || !msg_len || !pk_out || !sig_out) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    return for_each_shard(ctx, n, [&](Device &d, size_t b, size_t e) {
        return sign_shard(d, b, e, seed, msg_arena, msg_off, msg_len, pk_out, sig_out);
    });
}

// ---------------------------------------------------------------- Merkle (host buffers)
int cv_merkle_tx_ids_ex(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                        const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, uint8_t *ids, uint8_t *tx_status) {
    if (!ctx) return CV_E_ARGS;
    if (ntx == 0) return CV_OK;
    if (!tx_leaf_begin || !ids) return CV_E_ARGS;
    const size_t nleaves = tx_leaf_begin[ntx];
    if (tx_leaf_begin[0] != 0) return CV_E_ARGS;
    for (size_t t = 0; t < ntx; t++)
        if (tx_leaf_begin[t + 1] < tx_leaf_begin[t]) return CV_E_ARGS;
    if (nleaves && (!leaf_off || !leaf_len)) return CV_E_ARGS;
    if (ntx > 0xfffffffeull || nleaves > 0xffffffffull) return CV_E_TOO_LARGE;
    std::lock_guard<std::mutex> g(ctx->mu);
    Device &d = ctx->devs[0];
    CV_TRY(hipSetDevice(d.ordinal));
    uint64_t hi = 0;
    for (size_t i = 0; i < nleaves; i++) hi = std::max<uint64_t>(hi, leaf_off[i] + leaf_len[i]);
    CV_TRY(d.arena.ensure(hi + 16));
    CV_TRY(d.off.ensure(nleaves * 8 + 8));
    CV_TRY(d.len.ensure(nleaves * 4 + 4));
    CV_TRY(d.tx_begin.ensure((ntx + 1) * 4));
    CV_TRY(d.digest.ensure(nleaves * 32 + 32));
    CV_TRY(d.ids.ensure(ntx * 32));
    CV_TRY(d.status.ensure(ntx));
    hipStream_t s = d.stream;
    if (hi) CV_TRY(hipMemcpyAsync(d.arena.p, leaf_arena, hi, hipMemcpyHostToDevice, s));
    if (nleaves) {
        CV_TRY(hipMemcpyAsync(d.off.p, leaf_off, nleaves * 8, hipMemcpyHostToDevice, s));
        CV_TRY(hipMemcpyAsync(d.len.p, leaf_len, nleaves * 4, hipMemcpyHostToDevice, s));
    }
    CV_TRY(hipMemcpyAsync(d.tx_begin.p, tx_leaf_begin, (ntx + 1) * 4, hipMemcpyHostToDevice, s));
    CV_TRY(cvk_merkle((uint32_t)ntx, (uint32_t)nleaves, d.arena.as<uint8_t>(), d.off.as<uint64_t>(),
                      d.len.as<uint32_t>(), d.tx_begin.as<uint32_t>(), d.digest.as<uint32_t>(), d.ids.as<uint8_t>(),
                      d.status.as<uint8_t>(), s));
    CV_TRY(hipMemcpyAsync(ids, d.ids.p, ntx * 32, hipMemcpyDeviceToHost, s));
    if (tx_status) CV_TRY(hipMemcpyAsync(tx_status, d.status.p, ntx, hipMemcpyDeviceToHost, s));
    CV_TRY(hipStreamSynchronize(s));
    return CV_OK;
}

int cv_partial_merkle_verify(cv_ctx *ctx, size_t ntrees, size_t nnodes, const uint8_t *kind, const uint32_t *left,
                             const uint32_t *right, const uint8_t *leaf_hash, const uint32_t *tree_begin,
                             const uint8_t *root, size_t ncheck, const uint8_t *check, const uint32_t *check_begin,
                             uint8_t *verdict, uint8_t *status) {
    if (!ctx) return CV_E_ARGS;
    if (ntrees == 0) return CV_OK;
    if (!tree_begin || !check_begin || !root || !verdict) return CV_E_ARGS;
    if (nnodes && (!kind || !left || !right || !leaf_hash)) return CV_E_ARGS;
    if (ncheck && !check) return CV_E_ARGS;
    if (ntrees > 0xfffffffeull || nnodes > 0xfffffffeull || ncheck > 0xfffffffeull) return CV_E_TOO_LARGE;
    // the ranges must be well formed for the kernel to stay inside the buffers
    if (tree_begin[0] != 0 || tree_begin[ntrees] != nnodes || check_begin[0] != 0 || check_begin[ntrees] != ncheck)
        return CV_E_ARGS;
    for (size_t t = 0; t < ntrees; t++)
        if (tree_begin[t + 1] < tree_begin[t] || check_begin[t + 1] < check_begin[t]) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    Device &d = ctx->devs[0];
    CV_TRY(hipSetDevice(d.ordinal));
    auto up16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t o_kind = 0, o_left = up16(o_kind + nnodes), o_right = up16(o_left + 4 * nnodes);
    const size_t o_hash = up16(o_right + 4 * nnodes), o_tb = up16(o_hash + 32 * nnodes);
    const size_t o_root = up16(o_tb + 4 * (ntrees + 1)), o_check = up16(o_root + 32 * ntrees);
    const size_t o_cb = up16(o_check + 32 * ncheck), o_verdict = up16(o_cb + 4 * (ntrees + 1));
    const size_t o_status = up16(o_verdict + ntrees), o_dig = up16(o_status + ntrees);
    const size_t o_flag = up16(o_dig + 32 * nnodes), total = up16(o_flag + nnodes + 1);
    CV_TRY(d.pmt.ensure(total));
    uint8_t *base = d.pmt.as<uint8_t>();
    hipStream_t s = d.stream;
    if (nnodes) {
        CV_TRY(hipMemcpyAsync(base + o_kind, kind, nnodes, hipMemcpyHostToDevice, s));
        CV_TRY(hipMemcpyAsync(base + o_left, left, 4 * nnodes, hipMemcpyHostToDevice, s));
        CV_TRY(hipMemcpyAsync(base + o_right, right, 4 * nnodes, hipMemcpyHostToDevice, s));
        CV_TRY(hipMemcpyAsync(base + o_hash, leaf_hash, 32 * nnodes, hipMemcpyHostToDevice, s));
    }
    CV_TRY(hipMemcpyAsync(base + o_tb, tree_begin, 4 * (ntrees + 1), hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(base + o_root, root, 32 * ntrees, hipMemcpyHostToDevice, s));
    if (ncheck) CV_TRY(hipMemcpyAsync(base + o_check, check, 32 * ncheck, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(base + o_cb, check_begin, 4 * (ntrees + 1), hipMemcpyHostToDevice, s));
    CV_TRY(cvk_pmt_verify((uint32_t)ntrees, base + o_kind, reinterpret_cast<uint32_t *>(base + o_left),
                          reinterpret_cast<uint32_t *>(base + o_right), base + o_hash,
                          reinterpret_cast<uint32_t *>(base + o_tb), base + o_root, base + o_check,
                          reinterpret_cast<uint32_t *>(base + o_cb), reinterpret_cast<uint32_t *>(base + o_dig),
                          base + o_flag, base + o_verdict, base + o_status, s));
    CV_TRY(hipMemcpyAsync(verdict, base + o_verdict, ntrees, hipMemcpyDeviceToHost, s));
    if (status) CV_TRY(hipMemcpyAsync(status, base + o_status, ntrees, hipMemcpyDeviceToHost, s));
    CV_TRY(hipStreamSynchronize(s));
    return CV_OK;
}

int cv_merkle_tx_ids(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                     const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, uint8_t *ids) {
    return cv_merkle_tx_ids_ex(ctx, ntx, leaf_arena, leaf_off, leaf_len, tx_leaf_begin, ids, nullptr);
}

int cv_tx_verdicts(size_t ntx, const uint64_t *bitmap, const uint32_t *tx_sig_begin, uint8_t *tx_ok) {
    if (ntx == 0) return CV_OK;
    if (!bitmap || !tx_sig_begin || !tx_ok) return CV_E_ARGS;
    for (size_t t = 0; t < ntx; t++) {
        const uint32_t b = tx_sig_begin[t], e = tx_sig_begin[t + 1];
        if (e < b) return CV_E_ARGS;
        bool ok = e > b;
        for (uint32_t i = b; i < e && ok; i++) ok = (bitmap[i >> 6] >> (i & 63)) & 1u;
        tx_ok[t] = ok ? 1 : 0;
    }
    return CV_OK;
}

// ---------------------------------------------------------------- device-resident API
int cv_ed25519_verify_device(cv_ctx *ctx, int device, size_t n, const void *d_pk, const void *d_sig,
                             const void *d_arena, const void *d_off, const void *d_len, void *d_bitmap,
                             void *d_status, void *stream) {
    if (!ctx) return CV_E_ARGS;
    if (n == 0) return CV_OK;
    if (n > 0xffffffffull) return CV_E_TOO_LARGE;
    Device *d = find_dev(ctx, device);
    if (!d || !d_pk || !d_sig || !d_arena || !d_off || !d_len || !d_bitmap) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);            // enqueue only; ordered on the workspace (ws_begin)
    CV_TRY(hipSetDevice(d->ordinal));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : d->stream;
    CV_TRY(launch_verify(*d, (uint32_t)n, static_cast<const uint8_t *>(d_pk), static_cast<const uint8_t *>(d_sig),
                         static_cast<const uint8_t *>(d_arena), static_cast<const uint64_t *>(d_off),
                         static_cast<const uint32_t *>(d_len), static_cast<uint64_t *>(d_bitmap),
                         static_cast<uint8_t *>(d_status), s));
    return CV_OK;
}

int cv_ed25519_verify_device_timed(cv_ctx *ctx, int device, size_t n, const void *d_pk, const void *d_sig,
                                   const void *d_arena, const void *d_off, const void *d_len, void *d_bitmap,
                                   void *stream, float *phase_ms) {
    if (!ctx || !phase_ms) return CV_E_ARGS;
    phase_ms[0] = phase_ms[1] = phase_ms[2] = 0.f;
    if (n == 0) return CV_OK;
    if (n > 0xffffffffull) return CV_E_TOO_LARGE;
    Device *d = find_dev(ctx, device);
    if (!d || !d_pk || !d_sig || !d_arena || !d_off || !d_len || !d_bitmap) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    CV_TRY(hipSetDevice(d->ordinal));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : d->stream;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    hipError_t e = hipSuccess;
    for (int k = 0; k < 4 && e == hipSuccess; k++) e = hipEventCreate(&ev[k]);
    // one workspace chunk at a time (chunk starts are multiples of 64: whole bitmap words)
    for (size_t c0 = 0; c0 < n && e == hipSuccess; c0 += kVerifyChunk) {
        const size_t m = std::min<size_t>(kVerifyChunk, n - c0);
        e = launch_verify(*d, (uint32_t)m, static_cast<const uint8_t *>(d_pk) + c0 * 32,
                          static_cast<const uint8_t *>(d_sig) + c0 * 64, static_cast<const uint8_t *>(d_arena),
                          static_cast<const uint64_t *>(d_off) + c0, static_cast<const uint32_t *>(d_len) + c0,
                          static_cast<uint64_t *>(d_bitmap) + c0 / 64, nullptr, s, ev);
        if (e == hipSuccess) e = hipEventSynchronize(ev[3]);
        for (int k = 0; k < 3 && e == hipSuccess; k++) {
            float ms = 0.f;
            e = hipEventElapsedTime(&ms, ev[k], ev[k + 1]);
            phase_ms[k] += ms;
        }
    }
    for (hipEvent_t x : ev)
        if (x) (void)hipEventDestroy(x);
    return hip_rc(e);
}

int cv_ed25519_verify_device_keyed(cv_ctx *ctx, int device, size_t n, size_t nkeys, const void *d_keys,
                                   const void *d_key_index, const void *d_sig, const void *d_arena, const void *d_off,
                                   const void *d_len, void *d_bitmap, void *d_status, void *stream, float *phase_ms) {
    if (!ctx) return CV_E_ARGS;
    if (n == 0) return CV_OK;
    if (n > 0xffffffffull || nkeys > 0xffffffffull) return CV_E_TOO_LARGE;
    Device *d = find_dev(ctx, device);
    if (!d || nkeys == 0 || !d_keys || !d_key_index || !d_sig || !d_arena || !d_off || !d_len || !d_bitmap)
        return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    CV_TRY(hipSetDevice(d->ordinal));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : d->stream;
    // the key bytes come to the host (32 B per distinct key) to resolve them against the pool
    std::vector<uint8_t> hkeys(nkeys * 32);
    CV_TRY(hipMemcpyAsync(hkeys.data(), d_keys, nkeys * 32, hipMemcpyDeviceToHost, s));
    CV_TRY(hipStreamSynchronize(s));
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    hipError_t e = hipSuccess;
    if (phase_ms)
        for (int k = 0; k < 5 && e == hipSuccess; k++) e = hipEventCreate(&ev[k]);
    if (e == hipSuccess && phase_ms) e = hipEventRecord(ev[0], s);
    if (e == hipSuccess) e = ws_begin(*d, s);
    std::vector<uint32_t> sok;
    int rc = e == hipSuccess ? key_resolve(*d, ctx->key_cap, nkeys, hkeys.data(), nullptr, sok, s) : hip_rc(e);
    KeyCache &kc = d->kc;
    if (rc == CV_OK) rc = hip_rc(kc.slot_of_key.ensure(nkeys * 4));
    if (rc == CV_OK) rc = hip_rc(hipMemcpyAsync(kc.slot_of_key.p, sok.data(), nkeys * 4, hipMemcpyHostToDevice, s));
    if (rc == CV_OK) rc = hip_rc(ensure_verify_ws(*d, n));
    if (rc == CV_OK)
        rc = hip_rc(cvk_verify_keyed((uint32_t)n, static_cast<const uint8_t *>(d_keys),
                                     static_cast<const uint32_t *>(d_key_index), kc.slot_of_key.as<uint32_t>(),
                                     kc.ktab.as<uint32_t>(), kc.kok.as<uint8_t>(), static_cast<const uint8_t *>(d_sig),
                                     static_cast<const uint8_t *>(d_arena), static_cast<const uint64_t *>(d_off),
                                     static_cast<const uint32_t *>(d_len), static_cast<uint64_t *>(d_bitmap),
                                     static_cast<uint8_t *>(d_status), d->ws_hs.as<uint32_t>(), d->ws_R.as<uint32_t>(),
                                     d->ws_ok.as<uint8_t>(), d->ws_cap, s, phase_ms ? ev + 1 : nullptr));
    if (d->ws_ev) {
        const hipError_t e2 = ws_end(*d, s);
        if (rc == CV_OK) rc = hip_rc(e2);
    }
    if (rc == CV_OK && phase_ms) {
        e = hipEventSynchronize(ev[4]);
        for (int k = 0; k < 4 && e == hipSuccess; k++) e = hipEventElapsedTime(&phase_ms[k], ev[k], ev[k + 1]);
        rc = hip_rc(e);
    }
    for (hipEvent_t x : ev)
        if (x) (void)hipEventDestroy(x);
    return rc;
}

int cv_ed25519_sign_device(cv_ctx *ctx, int device, size_t n, const void *d_seed, const void *d_arena,
                           const void *d_off, const void *d_len, void *d_pk, void *d_sig, void *stream) {
    if (!ctx) return CV_E_ARGS;
    if (n == 0) return CV_OK;
    if (n > 0xffffffffull) return CV_E_TOO_LARGE;
    Device *d = find_dev(ctx, device);
    if (!d || !d_seed || !d_arena || !d_off || !d_len || !d_pk || !d_sig) return CV_E_ARGS;
    CV_TRY(hipSetDevice(d->ordinal));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : d->stream;
    CV_TRY(cvk_sign((uint32_t)n, static_cast<const uint8_t *>(d_seed), static_cast<const uint8_t *>(d_arena),
                    static_cast<const uint64_t *>(d_off), static_cast<const uint32_t *>(d_len),
                    static_cast<uint8_t *>(d_pk), static_cast<uint8_t *>(d_sig), s));
    return CV_OK;
}

int cv_merkle_tx_ids_device(cv_ctx *ctx, int device, size_t ntx, size_t nleaves, const void *d_arena,
                            const void *d_leaf_off, const void *d_leaf_len, const void *d_tx_leaf_begin,
                            void *d_workspace, void *d_ids, void *d_tx_status, void *stream) {
    if (!ctx) return CV_E_ARGS;
    if (ntx == 0) return CV_OK;
    if (ntx > 0xfffffffeull || nleaves > 0xffffffffull) return CV_E_TOO_LARGE;
    Device *d = find_dev(ctx, device);
    if (!d || !d_tx_leaf_begin || !d_ids || (nleaves && (!d_arena || !d_leaf_off || !d_leaf_len || !d_workspace)))
        return CV_E_ARGS;
    CV_TRY(hipSetDevice(d->ordinal));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : d->stream;
    CV_TRY(cvk_merkle((uint32_t)ntx, (uint32_t)nleaves, static_cast<const uint8_t *>(d_arena),
                      static_cast<const uint64_t *>(d_leaf_off), static_cast<const uint32_t *>(d_leaf_len),
                      static_cast<const uint32_t *>(d_tx_leaf_begin), static_cast<uint32_t *>(d_workspace),
                      static_cast<uint8_t *>(d_ids), static_cast<uint8_t *>(d_tx_status), s));
    return CV_OK;
}

int cv_synchronize(cv_ctx *ctx, int device) {
    if (!ctx) return CV_E_ARGS;
    Device *d = find_dev(ctx, device);
    if (!d) return CV_E_ARGS;
    CV_TRY(hipSetDevice(d->ordinal));
    CV_TRY(hipStreamSynchronize(d->stream));
    return CV_OK;
}

// ---------------------------------------------------------------- calibration
int cv_calibrate(cv_ctx *ctx, int device, double *mad_per_s, double *femul_per_s) {
    if (!ctx) return CV_E_ARGS;
    Device *d = find_dev(ctx, device);
    if (!d) return CV_E_ARGS;
    CV_TRY(hipSetDevice(d->ordinal));
    hipDeviceProp_t prop;
    CV_TRY(hipGetDeviceProperties(&prop, d->ordinal));
    const uint32_t blocks = (uint32_t)prop.multiProcessorCount * 8;   // 8 waves per SIMD worth of work
    void *scratch = nullptr;
    CV_TRY(hipMalloc(&scratch, 64));
    hipEvent_t e0, e1;
    CV_TRY(hipEventCreate(&e0));
    CV_TRY(hipEventCreate(&e1));
    double rates[2] = {0, 0};
    for (int which = 0; which < 2; which++) {
        const uint32_t iters = which == 0 ? 20000 : 2000;
        CV_TRY(cvk_calibrate(iters / 10, which, blocks, scratch, d->stream));   // warm-up
        CV_TRY(hipEventRecord(e0, d->stream));
        CV_TRY(cvk_calibrate(iters, which, blocks, scratch, d->stream));
        CV_TRY(hipEventRecord(e1, d->stream));
        CV_TRY(hipEventSynchronize(e1));
        float ms = 0;
        CV_TRY(hipEventElapsedTime(&ms, e0, e1));
        const double per_thread = which == 0 ? 128.0 * iters : 4.0 * iters;
        rates[which] = per_thread * blocks * 256.0 / (ms * 1e-3);
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(scratch);
    if (mad_per_s) *mad_per_s = rates[0];
    if (femul_per_s) *femul_per_s = rates[1];
    return CV_OK;
}

// Roofline peak on a cycle basis (diagnostic): out[0] = chip-wide v_mad_u64_u32 rate (MAC/s),
// out[1] = shader clock during the run (GHz, s_memtime over s_memrealtime in block 0),
// out[2] = cycles per mad wave-instruction per SIMD at that clock, out[3] = SIMD count,
// out[4] = the MAC ceiling at the 2.4 GHz peak clock for that cycle count (MAC/s).
int cv_calibrate_cycles(cv_ctx *ctx, int device, double *out) {
    if (!ctx || !out) return CV_E_ARGS;
    Device *d = find_dev(ctx, device);
    if (!d) return CV_E_ARGS;
    CV_TRY(hipSetDevice(d->ordinal));
    hipDeviceProp_t prop;
    CV_TRY(hipGetDeviceProperties(&prop, d->ordinal));
    const uint32_t blocks = (uint32_t)prop.multiProcessorCount * 8, iters = 20000;
    uint64_t *buf = nullptr;
    CV_TRY(hipMalloc(&buf, 64));
    hipEvent_t e0, e1;
    CV_TRY(hipEventCreate(&e0));
    CV_TRY(hipEventCreate(&e1));
    hipError_t e = cvk_mad_clock(iters / 10, blocks, buf, d->stream);
    if (e == hipSuccess) e = hipEventRecord(e0, d->stream);
    if (e == hipSuccess) e = cvk_mad_clock(iters, blocks, buf, d->stream);
    if (e == hipSuccess) e = hipEventRecord(e1, d->stream);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0.f;
    uint64_t clk[2] = {0, 0};
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess) e = hipMemcpy(clk, buf, 16, hipMemcpyDeviceToHost);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(buf);
    if (e != hipSuccess) return hip_rc(e);
    const double simds = 4.0 * prop.multiProcessorCount;
    const double rate = 128.0 * iters * blocks * 256.0 / (ms * 1e-3);
    const double ghz = clk[1] ? (double)clk[0] / ((double)clk[1] / 100e6) / 1e9 : 0.0;
    const double wave_instr_per_s = rate / 64.0;
    const double cyc = ghz > 0 ? simds * ghz * 1e9 / wave_instr_per_s : 0.0;
    out[0] = rate;
    out[1] = ghz;
    out[2] = cyc;
    out[3] = simds;
    out[4] = cyc > 0 ? simds * 2.4e9 * 64.0 / cyc : 0.0;
    return CV_OK;
}

// Per-phase shader cycles of the fused prep kernel (diagnostic build of the same code, one chunk):
// out[k] = mean cycles per wave of phase k (hash, lattice, digits, decode A+R, tables), out[5] =
// their sum, out[6] = waves measured, out[7] = the SHA-512 part of the hash phase.  The workspace is the device's verify workspace.
int cv_diag_prep_phases(cv_ctx *ctx, int device, size_t n, const void *d_pk, const void *d_sig, const void *d_arena,
                        const void *d_off, const void *d_len, double *out) {
    if (!ctx || !out || n == 0) return CV_E_ARGS;
    if (n > kVerifyChunk) return CV_E_TOO_LARGE;
    Device *d = find_dev(ctx, device);
    if (!d || !d_pk || !d_sig || !d_arena || !d_off || !d_len) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    CV_TRY(hipSetDevice(d->ordinal));
    CV_TRY(ensure_verify_ws(*d, n));
    const size_t waves = (n + 63) / 64;
    uint64_t *st = nullptr;
    CV_TRY(hipMalloc(&st, waves * 64));
    CV_TRY(ws_begin(*d, d->stream));
    hipError_t e = cvk_prep_probe((uint32_t)n, static_cast<const uint8_t *>(d_pk), static_cast<const uint8_t *>(d_sig),
                                  static_cast<const uint8_t *>(d_arena), static_cast<const uint64_t *>(d_off),
                                  static_cast<const uint32_t *>(d_len), d->ws_dig.as<uint32_t>(), d->ws_tab.as<uint32_t>(),
                                  d->ws_cap, st, d->stream);
    if (e == hipSuccess) e = ws_end(*d, d->stream);
    std::vector<uint64_t> h(waves * 8);
    if (e == hipSuccess) e = hipStreamSynchronize(d->stream);
    if (e == hipSuccess) e = hipMemcpy(h.data(), st, waves * 64, hipMemcpyDeviceToHost);
    (void)hipFree(st);
    if (e != hipSuccess) return hip_rc(e);
    double sum[6] = {0, 0, 0, 0, 0, 0};
    for (size_t w = 0; w < waves; w++)
        for (int k = 0; k < 6; k++) sum[k] += (double)h[w * 8 + k];
    out[5] = 0;
    for (int k = 0; k < 5; k++) {
        out[k] = sum[k] / (double)waves;
        out[5] += out[k];
    }
    out[6] = (double)waves;
    out[7] = sum[5] / (double)waves;
    return CV_OK;
}

}  // extern "C"
