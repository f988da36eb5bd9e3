// cv_api.cpp — the C-ABI (include/cordaverify.h): contexts, per-device verify workspace slots, host-buffer
// batches sharded over the context's GPUs (one host thread per device) and pipelined through pinned
// staging, and the device-resident entry points used by bench.py.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <chrono>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/cordaverify.h"
#include "cv_launch.h"

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
    void *dev = nullptr;   // the device's address of p (hipHostGetDevicePointer)
    size_t cap = 0;
    unsigned flags = hipHostMallocDefault;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = dev = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
        hipError_t e = hipHostMalloc(&p, want, flags);
        if (e == hipSuccess && (e = hipHostGetDevicePointer(&dev, p, 0)) != hipSuccess) (void)hipHostFree(p);
        if (e != hipSuccess) {
            p = dev = nullptr;
            return e;
        }
        cap = want;
        return hipSuccess;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
    template <class T> T *dev_as() const { return static_cast<T *>(dev); }
    void release() {
        if (p) (void)hipHostFree(p);
        p = dev = nullptr;
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
    // the last stream that used the pool, and an event after that use (pool_begin / pool_end)
    hipStream_t last = nullptr;
    hipEvent_t ev = nullptr;
    PinBuf pin;                    // pinned staging of the device-API keyed call's slot_of_key upload
    hipEvent_t pin_ev = nullptr;   // recorded after that upload
    bool pin_busy = false;
};

// One verify workspace (per signature: hs 64 B, 2 tables 2 x 1440 B, R record 128 B, ok 1 B, half-size
// digits 292 B) with what orders its use across streams, its drain-overlap helper, and the host
// pipeline's staging for the sub-chunks that run on it.  A device has kSlots of them: device-API
// calls on different streams take different slots and run concurrently; the host-buffer pipeline
// deals its sub-chunks round-robin over the slots (each slot's stream: H2D -> verify -> D2H).
struct Slot {
    DevBuf ws_hs, ws_tab, ws_R, ws_ok, ws_dig;
    uint32_t ws_cap = 0;
    hipStream_t last = nullptr;   // the stream of the last launch group on this workspace
    hipEvent_t ev = nullptr;      // recorded after that group
    uint64_t stamp = 0;           // last use (least-recently-used choice)
    CvkSplit split;               // drain-overlap helper stream + events (created on first need)
    hipStream_t stream = nullptr; // the slot's own stream (slot 0: the device stream)
    PinBuf pin_in;                // host-buffer staging of one (sub-)chunk: pk | sig | off | len | arena
    DevBuf packed;                // its device copy
    hipEvent_t h2d = nullptr;     // recorded after the last DMA out of pin_in
    bool h2d_pending = false;
};
constexpr int kSlots = 4;
constexpr int kRing = 6;   // input blocks of the host pipeline (more than slots: copies run ahead of kernels)
constexpr int kOuts = 2;   // host pipeline calls in flight per device (cv_ed25519_verify_batch_async)

// The verdict output of one pipelined host call on one device: bitmap words | status bytes on the
// device, their pinned host copy, and the event after that copy.  pending: enqueued, not yet copied
// into the caller's arrays (pipe_finish does that); gen counts the calls that used this slot.
struct PipeOut {
    DevBuf dout;
    PinBuf hout;
    hipEvent_t done = nullptr;           // (unused since the host-side join; kept for cv_close)
    hipEvent_t slot_done[kSlots] = {};   // after this call's last launch group on each slot stream
    bool slot_used[kSlots] = {};
    bool pending = false;
    uint64_t gen = 0;
    uint64_t *bitmap = nullptr;
    uint8_t *status = nullptr;
    size_t b = 0, n = 0, o_st = 0;
};

// A fixed set of host threads for index-parallel jobs (the host-buffer path's packing and range scans):
// run(ntasks, fn) calls fn(i) for every i in [0, ntasks) on the helpers and the calling thread and
// returns when all are done.  Created once per device, so a pipelined call does not pay a thread start
// per sub-chunk (round-3 probe: ~14 thread starts per sub-chunk held C5's host path at 11 GB/s).
class WorkerPool {
  public:
    explicit WorkerPool(int helpers) {
        for (int t = 0; t < helpers; t++) th_.emplace_back([this] { loop(); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int threads() const { return (int)th_.size() + 1; }
    void run(size_t ntasks, const std::function<void(size_t)> &fn) {
        if (ntasks == 0) return;
        if (th_.empty() || ntasks == 1) {
            for (size_t i = 0; i < ntasks; i++) fn(i);
            return;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &fn;
            ntasks_ = ntasks;
            next_.store(0);
            busy_ = th_.size();
            gen_++;
        }
        cv_.notify_all();
        drain(fn, ntasks);
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return busy_ == 0; });
        job_ = nullptr;
    }

  private:
    void drain(const std::function<void(size_t)> &fn, size_t ntasks) {
        for (size_t i; (i = next_.fetch_add(1)) < ntasks;) fn(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(size_t)> *job;
            size_t ntasks;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                job = job_;
                ntasks = ntasks_;
            }
            drain(*job, ntasks);
            {
                std::lock_guard<std::mutex> g(mu_);
                if (--busy_ == 0) done_cv_.notify_one();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t)> *job_ = nullptr;
    size_t ntasks_ = 0, busy_ = 0;
    std::atomic<size_t> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

struct Device {
    int ordinal = 0;
    hipStream_t stream = nullptr;
    DevBuf pk, sig, arena, off, len, bitmap, status, seed, tx_begin, digest, ids;
    PinBuf pin_out;                      // host-buffer verify outputs: bitmap | status
    // zero-copy notary path (verify_shard_small_zc): fine-grained pinned host memory the kernels read
    // (packed records) and store into (verdict nibbles | status) over PCIe
    PinBuf zc_in, zc_out;
    DevBuf pmt;                          // partial Merkle trees: inputs, outputs and workspace, packed
    Slot slot[kSlots];
    uint64_t clock = 0;
    KeyCache kc;
    std::unique_ptr<WorkerPool> pool;    // host packing threads (created on the first large host batch)
    // The host pipeline's input ring (verify_shard_pipe): sub-chunk j's records go into device block
    // j % kRing by the ONE copy stream (so every H2D copy runs on one DMA queue, never as a blit kernel
    // beside the verify kernels), packed first into pinned staging block j % kRing when the caller's
    // arrays are pageable.  in_ready[q]: after block q's copies (copy stream); in_free[q]: after the
    // verify that read it (its slot stream).
    hipStream_t copy = nullptr;
    hipStream_t outs = nullptr;          // the pipeline's verdict copies (pipe_finish)
    PipeOut out[kOuts];                  // the pipeline's verdict outputs, one per call in flight
    int out_next = 0;
    DevBuf inblk[kRing];
    PinBuf instage[kRing];
    hipEvent_t in_ready[kRing] = {}, in_free[kRing] = {};
    bool in_used[kRing] = {}, stage_busy[kRing] = {};
    int ring_next = 0;                   // the ring block the next sub-chunk takes
    WorkerPool &workers(int threads) {
        if (!pool || pool->threads() != threads) {
            pool.reset();
            pool.reset(new WorkerPool(threads - 1));
        }
        return *pool;
    }
};

// key-table pool capacity per device (keys); 66 KB of tables per key (1.1 GB at the default; the pool
// grows to a call's distinct keys when they exceed it)
constexpr uint32_t kDefaultKeyCap = 1u << 14;
constexpr size_t kKtabBytes = 16512 * 4;  // CV_KTAB_WORDS: 4 comb rows x 129 affine entries x 128 B
constexpr size_t kTabBytes = 9 * 40 * 4;  // CV_TAB_WORDS: k*P, k = 0..8, cached form (cv_verify.h)
// new keys' tables are computed in launches of at most this many keys (bounded keyprep scratch: 270 MB)
constexpr size_t kKeyprepBatch = 4096;
// cv_ed25519_verify_batch dedupes keys on the host up to this batch size, and takes the keyed
// (per-key comb) path when the batch has at least eight signatures per distinct key on average (a key's
// 66 KB of tables cost about as much as 7 plain verifies to build; cached keys cost nothing)
constexpr size_t kAutoKeyedMax = 1u << 18;

// Verify workspace capacity: batches above it run in chunks of this many signatures (~13.4 GB of
// workspace at 2^22; same-box A/B at 8M signatures: 2^21 73.2, 2^22 72.4, 2^23 72.4 ms -- fewer
// chunk tails to drain; whole-round chunks of 1,966,080 were slower, 73.4 ms).
constexpr uint32_t kVerifyChunk = 1u << 22;

// Host-buffer pipeline (verify_shard_pipe): shards above g_pipe_min signatures are cut into a first
// sub-chunk of g_pipe_first (short, so the GPU starts early) and then sub-chunks of g_pipe_chunk (the
// last two balanced), dealt round-robin over the device's slots; g_pack_threads host threads pack each
// sub-chunk into pinned staging while the earlier ones transfer and verify.
static size_t g_pipe_min = 131072, g_pipe_first = 32768, g_pipe_chunk = 262144;
static int g_pack_threads = 8;
// small-form batches of at least this many signatures pack their staging on the device's worker pool
static size_t g_small_pool_min = 16384;
// compute slots the pipeline deals its sub-chunks over (2..kSlots).  2: with GPU_MAX_HW_QUEUES = 4
// (HIP's default) the null stream, the device stream, one more slot stream and the copy stream each get
// a hardware queue; a third slot stream shares one — with the copy stream, whose copies then waited
// behind that slot's Straus kernel (2.4 ms stalls, profiles/r03e_timeline_pinned_nofill.txt)
static int g_pipe_slots = 2;
static int g_pipe_ramp = 1;    // sub-chunk sizes double from g_pipe_first up to g_pipe_chunk
static size_t g_async_chunk = 262144;   // sub-chunks of cv_ed25519_verify_batch_async (no ramp)
// host-side time of the pipelined path, seconds (cvk_pipe_stats): range scans, packing, waits for a
// slot's staging, enqueue (HIP calls), the final synchronisation; and calls / sub-chunks
struct PipeStats {
    double plan = 0, pack = 0, wait = 0, enq = 0, sync = 0;
    uint64_t calls = 0, chunks = 0, direct = 0;
};
// 1 = pinned caller arrays are DMAed in place (stage_direct); 0 = always pack (A/B knob)
static int g_direct_dma = 1;
static size_t g_direct_small_min = 16384;   // the small path's direct-DMA threshold (signatures)
// 1 = cv_open creates the host pipeline's streams (slot 1, copy, verdict copy) right after the device
// stream; 0 = on first use (A/B knob, read by cv_open)
static int g_eager_streams = 1;
// tri-form batches from host buffers: 0 = DMA in / copy out (verify_shard_small), 1 = zero-copy (the prep
// reads the pinned staging over PCIe, verdicts stored into pinned host memory), 2 = zero-copy out with a
// gather kernel moving the staging into device memory first (verify_shard_small_zc), 3 = auto: 2 from
// 2,048 signatures, 1 below (same-box A/B, profiles/r03p_notary_zc_gather_ab.log: 4,096 0.289 ms p50 with
// the gather against 0.291-0.298 without; 256 0.251 against 0.249)
static int g_small_zc = 3;
// host-side time of the zero-copy path, seconds (cvk_small_stats): range scan + setup (buffers,
// workspace), packing, launches, the synchronisation (≈ the kernels), the bitmap assembly; and calls
static double g_small_t[5];
static uint64_t g_small_calls;
static PipeStats g_pipe_stats;
static std::mutex g_pipe_stats_mu;
static inline double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

hipError_t slot_events(Slot &sl) {
    hipError_t e = hipSuccess;
    if (!sl.ev && (e = hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming)) != hipSuccess) return e;
    if (!sl.h2d && (e = hipEventCreateWithFlags(&sl.h2d, hipEventDisableTiming)) != hipSuccess) return e;
    return e;
}

// the slot's own stream (created on first use; slot 0 shares the device stream)
hipError_t slot_stream(Device &d, int k, hipStream_t *out) {
    Slot &sl = d.slot[k];
    if (!sl.stream) {
        if (k == 0)
            sl.stream = d.stream;
        else {
            const hipError_t e = hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking);
            if (e != hipSuccess) {
                sl.stream = nullptr;
                return e;
            }
        }
    }
    *out = sl.stream;
    return hipSuccess;
}

// the drain-overlap helper of a slot (created on the first large device-API call that may split)
hipError_t slot_split(Device &d, Slot &sl) {
    if (sl.split.s2) return hipSuccess;
    CvkSplit x;
    hipError_t e = hipDeviceGetAttribute(&x.cus, hipDeviceAttributeMultiprocessorCount, d.ordinal);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&x.start, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&x.prep1, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&x.done2, hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&x.s2, hipStreamNonBlocking);
    if (e != hipSuccess) {
        for (hipEvent_t v : {x.start, x.prep1, x.done2})
            if (v) (void)hipEventDestroy(v);
        return e;
    }
    sl.split = x;
    return hipSuccess;
}

// The workspace slot for a launch group on stream s: the slot s used last (no cross-stream wait),
// else the least recently used one (ws_begin then waits for that slot's previous group).
Slot &pick_slot(Device &d, hipStream_t s) {
    for (Slot &sl : d.slot)
        if (sl.last == s) return sl;
    Slot *best = &d.slot[0];
    for (Slot &sl : d.slot)
        if (sl.stamp < best->stamp) best = &sl;
    return *best;
}

// Grows a slot's workspace to n signatures (capped at one chunk).  The old buffers may still be read
// by a queued group, so that group is waited for first; ws_cap stays 0 until all five buffers exist
// (a failed growth leaves a slot that the next call grows again, never a null workspace with a
// stale capacity).
hipError_t ensure_verify_ws(Slot &sl, size_t n) {
    uint32_t want = (uint32_t)std::min<size_t>(kVerifyChunk, (n + 511) / 512 * 512);
    if (want <= sl.ws_cap) return hipSuccess;
    hipError_t e;
    if (sl.last && sl.ev && (e = hipEventSynchronize(sl.ev)) != hipSuccess) return e;
    sl.ws_cap = 0;
    if ((e = sl.ws_hs.ensure((size_t)want * 64)) != hipSuccess) return e;
    if ((e = sl.ws_tab.ensure((size_t)want * 2 * kTabBytes)) != hipSuccess) return e;   // k*(-A), k*R
    if ((e = sl.ws_R.ensure((size_t)want * 128)) != hipSuccess) return e;
    if ((e = sl.ws_ok.ensure((size_t)want)) != hipSuccess) return e;
    if ((e = sl.ws_dig.ensure((size_t)want * 73 * 4)) != hipSuccess) return e;   // CV_HS_DIGWORDS
    sl.ws_cap = want;
    return hipSuccess;
}

// Every use of a shared device resource (a workspace slot, the key pool) is ordered across streams:
// a launch group enqueued on stream s first waits for the previous group when that ran on another
// stream (ws_begin), and marks its own end (ws_end).  Device-pointer calls may therefore be made on any
// streams; two streams that hold different slots run concurrently, and a stream that takes over a slot
// waits for it instead of racing on it.  Callers hold ctx->mu around ws_begin .. ws_end.
hipError_t ws_begin(Device &d, Slot &sl, hipStream_t s) {
    hipError_t e = slot_events(sl);
    if (e != hipSuccess) return e;
    sl.stamp = ++d.clock;
    if (sl.last && sl.last != s) e = hipStreamWaitEvent(s, sl.ev, 0);
    return e;
}
hipError_t ws_end(Slot &sl, hipStream_t s) {
    sl.last = s;
    return hipEventRecord(sl.ev, s);
}
hipError_t pool_begin(KeyCache &kc, hipStream_t s) {
    hipError_t e = hipSuccess;
    if (!kc.ev && (e = hipEventCreateWithFlags(&kc.ev, hipEventDisableTiming)) != hipSuccess) return e;
    if (kc.last && kc.last != s) e = hipStreamWaitEvent(s, kc.ev, 0);
    return e;
}
hipError_t pool_end(KeyCache &kc, hipStream_t s) {
    kc.last = s;
    return hipEventRecord(kc.ev, s);
}

// One verify launch group on slot sl, stream s.  split: the drain-overlap sub-chunks may be used.
hipError_t launch_verify(Device &d, Slot &sl, uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                         const uint64_t *off, const uint32_t *len, uint64_t *bitmap, uint8_t *status, hipStream_t s,
                         hipEvent_t *ev, bool split) {
    hipError_t e = ensure_verify_ws(sl, n);
    if (e == hipSuccess) e = ws_begin(d, sl, s);
    if (e != hipSuccess) return e;
    if (split && n >= 131072) (void)slot_split(d, sl);   // without a helper the chunk runs whole
    e = cvk_verify(n, pk, sig, arena, off, len, bitmap, status, sl.ws_hs.as<uint32_t>(), sl.ws_tab.as<uint32_t>(),
                   sl.ws_R.as<uint32_t>(), sl.ws_ok.as<uint8_t>(), sl.ws_dig.as<uint32_t>(), sl.ws_cap, s, ev,
                   split && sl.split.s2 ? &sl.split : nullptr);
    const hipError_t e2 = ws_end(sl, s);
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

// Runs fn at scope exit unless dismissed (error paths that must drain queued DMAs out of pinned
// staging before a later call reuses or frees it).
template <class F> struct OnExit {
    F fn;
    bool armed = true;
    ~OnExit() {
        if (armed) fn();
    }
};
template <class F> OnExit<F> on_exit(F fn) { return OnExit<F>{fn}; }

}  // namespace

struct cv_ctx {
    std::vector<Device> devs;
    std::mutex mu;
    uint32_t key_cap = kDefaultKeyCap;
    // cv_ed25519_verify_batch_async: ticket -> (device index, output slot, that slot's gen) per shard
    uint64_t next_ticket = 0;
    std::unordered_map<uint64_t, std::vector<std::array<uint64_t, 3>>> tickets;
};

extern "C" {

const char *cv_version(void) { return "cordaverify-mi355x 0.2 (gfx950)"; }

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

// Tuning knob (internal): the host-buffer pipeline's shard threshold, first and steady sub-chunk sizes
// (signatures; 0 keeps the current value) and packing threads.
void cvk_set_direct_dma(int v) { g_direct_dma = v ? 1 : 0; }
void cvk_set_direct_small_min(int n) { g_direct_small_min = n > 0 ? (size_t)n : 16384; }
void cvk_set_small_zc(int v) { g_small_zc = (v >= 0 && v <= 3) ? v : 3; }
void cvk_set_eager_streams(int v) { g_eager_streams = v ? 1 : 0; }
// out[6] = plan+setup, pack, launch, sync, assemble (seconds, summed) and calls; reset clears them
void cvk_small_stats(double *out, int reset) {
    std::lock_guard<std::mutex> g(g_pipe_stats_mu);
    if (out) {
        for (int k = 0; k < 5; k++) out[k] = g_small_t[k];
        out[5] = (double)g_small_calls;
    }
    if (reset) {
        for (double &t : g_small_t) t = 0;
        g_small_calls = 0;
    }
}
void cvk_set_small_pool_min(int n) { g_small_pool_min = n > 0 ? (size_t)n : 16384; }
void cvk_set_pipe_slots(int k) { g_pipe_slots = (k >= 2 && k <= kSlots) ? k : 2; }
void cvk_set_pipe_ramp(int v) { g_pipe_ramp = v ? 1 : 0; }
void cvk_set_async_chunk(int m) { g_async_chunk = m >= 64 ? (size_t)m / 64 * 64 : 262144; }
void cvk_set_pipe(size_t min_n, size_t first, size_t chunk, int threads) {
    if (min_n) g_pipe_min = min_n;
    if (first) g_pipe_first = std::max<size_t>(64, first / 64 * 64);
    if (chunk) g_pipe_chunk = std::max<size_t>(64, chunk / 64 * 64);
    if (threads > 0) g_pack_threads = std::min(threads, 64);
}

// Diagnostic knob: out[7] = {plan, pack, wait, enqueue, sync seconds, calls, sub-chunks} of the
// pipelined host path since the last reset.
void cvk_pipe_stats(double *out, int reset) {
    std::lock_guard<std::mutex> g(g_pipe_stats_mu);
    const PipeStats &p = g_pipe_stats;
    if (out) {
        out[0] = p.plan;
        out[1] = p.pack;
        out[2] = p.wait;
        out[3] = p.enq;
        out[4] = p.sync;
        out[5] = (double)p.calls;
        out[6] = (double)p.chunks;
    }
    if (reset) g_pipe_stats = PipeStats{};
}
// max(off[i] + len[i]) over n records (0 for n = 0): the arena bytes a batch reaches, for the Python
// mirror's bounds check; slices of 2^20 records on up to 8 threads.
uint64_t cvk_msg_end(size_t n, const uint64_t *off, const uint32_t *len) {
    if (!n || !off || !len) return 0;
    constexpr size_t kSlice = 1u << 20;
    const size_t ns = (n + kSlice - 1) / kSlice;
    std::vector<uint64_t> part(ns, 0);
    auto scan = [&](size_t k) {
        uint64_t hi = 0;
        const size_t i1 = std::min(n, (k + 1) * kSlice);
        for (size_t i = k * kSlice; i < i1; i++) hi = std::max<uint64_t>(hi, off[i] + len[i]);
        part[k] = hi;
    };
    const size_t nt = std::min<size_t>(ns, 8);
    if (nt <= 1) {
        scan(0);
    } else {
        std::atomic<size_t> next{0};
        std::vector<std::thread> th;
        for (size_t t = 0; t < nt; t++)
            th.emplace_back([&] {
                for (size_t k; (k = next.fetch_add(1)) < ns;) scan(k);
            });
        for (auto &t : th) t.join();
    }
    return *std::max_element(part.begin(), part.end());
}
// sub-chunks of the pipelined path that were DMAed straight from pinned caller arrays (since the last reset)
double cvk_pipe_direct_chunks(void) {
    std::lock_guard<std::mutex> g(g_pipe_stats_mu);
    return (double)g_pipe_stats.direct;
}

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
            ctx->devs.push_back(std::move(dev));
            // The host pipeline's concurrently busy streams — slot 0 (the device stream), slot 1, the copy
            // stream and the verdict-copy stream — are created back to back here, before any helper
            // stream, so the runtime spreads them over distinct hardware queues (GPU_MAX_HW_QUEUES = 4 by
            // default).  Created lazily, after the device API's split helpers or a caller's own streams,
            // the copy stream could share a queue with a compute stream and its copies wait behind that
            // stream's kernels.
            if (g_eager_streams) {
                Device &dd = ctx->devs.back();
                hipStream_t s1 = nullptr;
                if (slot_stream(dd, 1, &s1) != hipSuccess ||
                    hipStreamCreateWithFlags(&dd.copy, hipStreamNonBlocking) != hipSuccess ||
                    hipStreamCreateWithFlags(&dd.outs, hipStreamNonBlocking) != hipSuccess) {
                    cv_close(ctx);
                    return CV_E_HIP;
                }
            }
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
        (void)hipDeviceSynchronize();
        for (DevBuf *b : {&d.pk, &d.sig, &d.arena, &d.off, &d.len, &d.bitmap, &d.status, &d.seed, &d.tx_begin,
                          &d.digest, &d.ids, &d.pmt, &d.kc.ktab, &d.kc.kok, &d.kc.keys, &d.kc.slots,
                          &d.kc.slot_of_key, &d.kc.key_index, &d.kc.scratch})
            b->release();
        d.pin_out.release();
        d.zc_in.release();
        d.zc_out.release();
        for (int k = 0; k < kSlots; k++) {
            Slot &sl = d.slot[k];
            for (DevBuf *b : {&sl.ws_hs, &sl.ws_tab, &sl.ws_R, &sl.ws_ok, &sl.ws_dig, &sl.packed}) b->release();
            sl.pin_in.release();
            for (hipEvent_t v : {sl.ev, sl.h2d, sl.split.start, sl.split.prep1, sl.split.done2})
                if (v) (void)hipEventDestroy(v);
            if (sl.split.s2) (void)hipStreamDestroy(sl.split.s2);
            if (k > 0 && sl.stream) (void)hipStreamDestroy(sl.stream);
        }
        for (PipeOut &o : d.out) {
            o.dout.release();
            o.hout.release();
            if (o.done) (void)hipEventDestroy(o.done);
            for (hipEvent_t v : o.slot_done)
                if (v) (void)hipEventDestroy(v);
        }
        if (d.outs) (void)hipStreamDestroy(d.outs);
        for (int q = 0; q < kRing; q++) {
            d.inblk[q].release();
            d.instage[q].release();
            for (hipEvent_t v : {d.in_ready[q], d.in_free[q]})
                if (v) (void)hipEventDestroy(v);
        }
        if (d.copy) (void)hipStreamDestroy(d.copy);
        d.kc.pin.release();
        if (d.kc.ev) (void)hipEventDestroy(d.kc.ev);
        if (d.kc.pin_ev) (void)hipEventDestroy(d.kc.pin_ev);
        if (d.stream) (void)hipStreamDestroy(d.stream);
    }
    delete ctx;
}

int cv_device_count(const cv_ctx *ctx) { return ctx ? (int)ctx->devs.size() : 0; }

int cv_host_alloc(cv_ctx *ctx, size_t bytes, void **out) {
    if (!ctx || !out || bytes == 0) return CV_E_ARGS;
    *out = nullptr;
    CV_TRY(hipSetDevice(ctx->devs[0].ordinal));
    void *p = nullptr;
    const hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e != hipSuccess) return e == hipErrorOutOfMemory ? CV_E_OOM : CV_E_HIP;
    *out = p;
    return CV_OK;
}

void cv_host_free(cv_ctx *ctx, void *p) {
    (void)ctx;
    if (p) (void)hipHostFree(p);
}

static Device *find_dev(cv_ctx *ctx, int device) {
    for (Device &d : ctx->devs)
        if (d.ordinal == device) return &d;
    return nullptr;
}

}  // extern "C"

// ---------------------------------------------------------------- verify (host buffers)
static inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// Host copies into pinned staging.  A large copy is done by the device's worker pool (one core copies
// ~10-12 GB/s, below what the DMA takes): each segment is cut into 256 KB pieces the workers take in
// turn.  Copies below 1 MB stay on the calling thread (a notary batch: waking workers costs more).
struct CopyJob {
    void *dst;
    const void *src;
    size_t len;
};
static void par_copy(const std::vector<CopyJob> &jobs, WorkerPool *pool) {
    constexpr size_t kPiece = 256 * 1024;
    size_t total = 0;
    for (const CopyJob &j : jobs) total += j.len;
    if (!pool || pool->threads() <= 1 || total < 4 * kPiece) {
        for (const CopyJob &j : jobs)
            if (j.len) std::memcpy(j.dst, j.src, j.len);
        return;
    }
    std::vector<CopyJob> pieces;
    pieces.reserve(total / kPiece + jobs.size());
    for (const CopyJob &j : jobs)
        for (size_t o = 0; o < j.len; o += kPiece)
            pieces.push_back({static_cast<uint8_t *>(j.dst) + o, static_cast<const uint8_t *>(j.src) + o,
                              std::min(kPiece, j.len - o)});
    pool->run(pieces.size(), [&pieces](size_t k) { std::memcpy(pieces[k].dst, pieces[k].src, pieces[k].len); });
}

// Staging layout of records [b, e): pk | sig | off | len | arena, 16-B aligned parts.  The arena part is
// the byte range [lo, hi) the records' messages span, with lo rounded down to 16 so the device arena
// pointer keeps every message's alignment; the kernels get arena_dev - lo and the caller's offsets
// unchanged.  When the messages are scattered (the range is more than twice their bytes + 1 MB), they
// are gathered back to back instead and the offsets rewritten ("compact").
struct Stage {
    size_t n = 0, o_pk = 0, o_sig = 0, o_off = 0, o_len = 0, o_ar = 0, total = 0;
    uint64_t lo = 0, hi = 0;
    bool compact = false;
};
static Stage stage_plan(size_t b, size_t e, const uint64_t *off, const uint32_t *len, WorkerPool *pool = nullptr) {
    Stage st;
    st.n = e - b;
    // the range scan, in slices of 64K records over the pool
    constexpr size_t kSlice = 65536;
    const size_t nslices = (st.n + kSlice - 1) / kSlice;
    struct R {
        uint64_t lo = UINT64_MAX, hi = 0, bytes = 0;
    };
    std::vector<R> part(std::max<size_t>(nslices, 1));
    auto scan = [&](size_t k) {
        R r;
        const size_t i1 = std::min(e, b + (k + 1) * kSlice);
        for (size_t i = b + k * kSlice; i < i1; i++) {
            r.lo = std::min<uint64_t>(r.lo, off[i]);
            r.hi = std::max<uint64_t>(r.hi, off[i] + len[i]);
            r.bytes += len[i];
        }
        part[k] = r;
    };
    if (pool && nslices > 1)
        pool->run(nslices, scan);
    else
        for (size_t k = 0; k < nslices; k++) scan(k);
    uint64_t lo = UINT64_MAX, hi = 0, bytes = 0;
    for (const R &r : part) {
        lo = std::min(lo, r.lo);
        hi = std::max(hi, r.hi);
        bytes += r.bytes;
    }
    if (hi < lo) lo = hi = 0;
    lo &= ~(uint64_t)15;
    st.compact = hi - lo > 2 * bytes + (1u << 20);
    st.lo = st.compact ? 0 : lo;
    st.hi = st.compact ? bytes : hi;
    const size_t n = st.n;
    st.o_pk = 0;
    st.o_sig = al16(n * 32);
    st.o_off = st.o_sig + al16(n * 64);
    st.o_len = st.o_off + al16(n * 8);
    st.o_ar = st.o_len + al16(n * 4);
    st.total = st.o_ar + al16(st.hi - st.lo + 16);
    return st;
}
// Packs records [b, e) into h by the plan (keys + signatures first: `first_part` runs after them, so
// their DMA can start while the rest is packed).
template <class F>
static void stage_pack(const Stage &st, uint8_t *h, size_t b, const uint8_t *pk, const uint8_t *sig,
                       const uint8_t *arena, const uint64_t *off, const uint32_t *len, WorkerPool *pool, F first_part) {
    const size_t n = st.n;
    par_copy({{h + st.o_pk, pk + b * 32, n * 32}, {h + st.o_sig, sig + b * 64, n * 64}}, pool);
    first_part();
    uint64_t *hoff = reinterpret_cast<uint64_t *>(h + st.o_off);
    uint8_t *har = h + st.o_ar;
    if (st.compact) {
        par_copy({{h + st.o_len, len + b, n * 4}}, nullptr);
        uint64_t pos = 0;
        for (size_t i = 0; i < n; i++) {
            hoff[i] = pos;
            if (len[b + i]) std::memcpy(har + pos, arena + off[b + i], len[b + i]);
            pos += len[b + i];
        }
    } else {
        par_copy({{h + st.o_off, off + b, n * 8}, {h + st.o_len, len + b, n * 4},
                  {har, st.hi > st.lo ? arena + st.lo : nullptr, (size_t)(st.hi - st.lo)}},
                 pool);
    }
    std::memset(har + (st.hi - st.lo), 0, 16);
}

// Is [p, p + bytes) page-locked host memory (hipHostMalloc / hipHostRegister)?  Both ends are looked
// up; a failed lookup (pageable memory) clears the runtime's last-error state so no later
// hipGetLastError reports it.
static bool host_pinned(const void *p, size_t bytes) {
    if (!p || bytes == 0) return p != nullptr;
    const uint8_t *q[2] = {static_cast<const uint8_t *>(p), static_cast<const uint8_t *>(p) + bytes - 1};
    for (const uint8_t *x : q) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, x) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (a.type != hipMemoryTypeHost) return false;
    }
    return true;
}
// Direct form of a stage: the record arrays of [b, e) and the arena range all pinned (and the arena
// not compacted), so they can be DMAed from where they are.
static bool stage_direct(const Stage &st, size_t b, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                         const uint64_t *off, const uint32_t *len) {
    if (!g_direct_dma || st.compact) return false;
    const size_t n = st.n;
    return host_pinned(pk + b * 32, n * 32) && host_pinned(sig + b * 64, n * 64) && host_pinned(off + b, n * 8) &&
           host_pinned(len + b, n * 4) && (st.hi == st.lo || host_pinned(arena + st.lo, st.hi - st.lo));
}
// The stage's DMAs straight from the caller's pinned arrays into the device block dv (the layout of
// stage_pack).  The 16 bytes after the arena part keep whatever the block held: the kernels read a
// message only through dword windows clamped to its last byte and mask the bytes past it, so those
// bytes never reach a verdict — and a fill there would be a blit KERNEL on the copy queue, which waits
// for a free CU slot behind the running verify waves (it held the C2 copy stream for 2.5 ms,
// profiles/r03d_timeline_pinned.txt).
static hipError_t stage_dma_direct(const Stage &st, uint8_t *dv, size_t b, const uint8_t *pk, const uint8_t *sig,
                                   const uint8_t *arena, const uint64_t *off, const uint32_t *len, hipStream_t s) {
    const size_t n = st.n;
    hipError_t e = hipMemcpyAsync(dv + st.o_pk, pk + b * 32, n * 32, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(dv + st.o_sig, sig + b * 64, n * 64, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(dv + st.o_off, off + b, n * 8, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(dv + st.o_len, len + b, n * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && st.hi > st.lo)
        e = hipMemcpyAsync(dv + st.o_ar, arena + st.lo, st.hi - st.lo, hipMemcpyHostToDevice, s);
    return e;
}

// Zero-copy form of the small path for tri-chain batches (n <= cvk_get_tri_max(): the notary batches).
// The records are packed into fine-grained pinned host memory that the fused prep kernel reads over
// PCIe, and the kernels store the status bytes and one verdict byte per wave (4 bits) into pinned host
// memory: no DMA in, no copy out.  Measured on the box, notary 4,096 (profiles/r03j_timeline_notary4096.txt),
// the DMA path paid 19.8 us of H2D + 11.6 us from the DMA's completion to the prep's start + 9.6 us for
// the verdict copy (a blit kernel after the Straus kernel).
static int verify_shard_small_zc(Device &d, const Stage &st, size_t b, const uint8_t *pk, const uint8_t *sig,
                                 const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint64_t *bitmap,
                                 uint8_t *status, WorkerPool *pool, double t_plan, bool gather) {
    double t[6];
    t[0] = t_plan;
    const size_t n = st.n, words = (n + 63) / 64, nnib = words * 16, waves = (n + 3) / 4;
    Slot &sl = d.slot[0];
    hipStream_t s = nullptr;
    CV_TRY(slot_stream(d, 0, &s));
    CV_TRY(slot_events(sl));
    d.zc_in.flags = d.zc_out.flags = hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable;
    CV_TRY(d.zc_in.ensure(st.total));
    CV_TRY(d.zc_out.ensure(al16(nnib) + al16(n)));
    CV_TRY(ensure_verify_ws(sl, n));
    if (!cvk_tri_zc_ok((uint32_t)n, sl.ws_cap)) return CV_E_HIP;   // (cannot happen: checked by the caller)
    uint8_t *h = d.zc_in.as<uint8_t>();
    if (gather) CV_TRY(sl.packed.ensure(al16(st.total)));
    const uint8_t *dv = gather ? sl.packed.as<uint8_t>() : d.zc_in.dev_as<uint8_t>();
    t[1] = now_s();
    stage_pack(st, h, b, pk, sig, arena, off, len, pool, [] {});
    uint8_t *nib = d.zc_out.as<uint8_t>();
    std::memset(nib + waves, 0, nnib - waves);   // bytes of waves past the batch: no wave stores them
    t[2] = now_s();
    auto drain = on_exit([s] { (void)hipStreamSynchronize(s); });   // error paths: no kernel outlives the call
    CV_TRY(ws_begin(d, sl, s));
    const hipError_t e = cvk_verify_tri_zc(
        (uint32_t)n, dv + st.o_pk, dv + st.o_sig, dv + st.o_ar - st.lo, reinterpret_cast<const uint64_t *>(dv + st.o_off),
        reinterpret_cast<const uint32_t *>(dv + st.o_len), d.zc_out.dev_as<uint8_t>(),
        status ? d.zc_out.dev_as<uint8_t>() + al16(nnib) : nullptr, sl.ws_tab.as<uint32_t>(), sl.ws_ok.as<uint8_t>(),
        sl.ws_dig.as<uint32_t>(), sl.ws_cap, s, gather ? d.zc_in.dev : nullptr, gather ? sl.packed.p : nullptr,
        gather ? al16(st.total) : 0);
    const hipError_t e2 = ws_end(sl, s);
    CV_TRY(e);
    CV_TRY(e2);
    t[3] = now_s();
    CV_TRY(hipStreamSynchronize(s));
    drain.armed = false;
    t[4] = now_s();
    for (size_t w = 0; w < words; w++) {
        uint64_t x = 0;
        for (int j = 0; j < 16; j++) x |= (uint64_t)(nib[16 * w + j] & 15u) << (4 * j);
        bitmap[b / 64 + w] = x;
    }
    if (status) std::memcpy(status + b, nib + al16(nnib), n);
    t[5] = now_s();
    {
        std::lock_guard<std::mutex> g(g_pipe_stats_mu);
        for (int k = 0; k < 5; k++) g_small_t[k] += t[k + 1] - t[k];
        g_small_calls++;
    }
    return CV_OK;
}

// One shard [b, e) of a batch on one device, small form (the notary-sized batches): packed into slot 0's
// pinned staging, moved by one DMA (two above 1 MB: the first overlaps packing the second part) into
// one device block, verified, and the bitmap (+ status) come back by one DMA.  b is a multiple of 64,
// so the shard's bitmap words are whole words of the caller's bitmap.
static int verify_shard_small(Device &d, size_t b, size_t e, const uint8_t *pk, const uint8_t *sig,
                              const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint64_t *bitmap,
                              uint8_t *status, int threads) {
    const size_t n = e - b;
    WorkerPool *pool = n >= g_small_pool_min ? &d.workers(threads) : nullptr;
    const double t_plan = now_s();
    const Stage st = stage_plan(b, e, off, len, pool);
    if (g_small_zc && cvk_tri_zc_ok((uint32_t)n, (uint32_t)n))
        return verify_shard_small_zc(d, st, b, pk, sig, arena, off, len, bitmap, status, pool, t_plan,
                                     g_small_zc == 2 || (g_small_zc == 3 && n >= 2048));
    const size_t words = (n + 63) / 64;
    const size_t o_bm = 0, o_st = al16(words * 8), total_out = o_st + al16(n);
    Slot &sl = d.slot[0];
    hipStream_t s = nullptr;
    CV_TRY(slot_stream(d, 0, &s));
    // the staging of a previous call may still be in a DMA only if that call failed half way (it
    // drains its queue on every error path below), so this wait is normally free
    if (sl.h2d_pending) {
        CV_TRY(hipEventSynchronize(sl.h2d));
        sl.h2d_pending = false;
    }
    CV_TRY(slot_events(sl));
    CV_TRY(sl.pin_in.ensure(st.total));
    CV_TRY(d.pin_out.ensure(total_out));
    CV_TRY(sl.packed.ensure(st.total));
    CV_TRY(d.bitmap.ensure(total_out));
    uint8_t *h = sl.pin_in.as<uint8_t>();
    uint8_t *dv = sl.packed.as<uint8_t>();
    auto drain = on_exit([s] { (void)hipStreamSynchronize(s); });   // error paths: no DMA outlives the call
    // Two-stage staging above 1 MB of keys + signatures: they are packed and their DMA is issued
    // first, so it runs while the offsets, lengths and message bytes are packed (notary 65,536:
    // 1.29-1.34 -> 1.21-1.25 ms p50); below, one DMA (a second DMA's ~6 us would cost more than it hides).
    const bool two_stage = st.o_off >= ((size_t)1 << 20);
    // below g_direct_small_min signatures one packed DMA beats five direct ones even from pinned
    // arrays (notary 4,096: 0.328 ms p50 packed vs 0.342 direct; 65,536: 1.28 vs 1.10,
    // profiles/r03h_bench.json)
    if (n >= g_direct_small_min && stage_direct(st, b, pk, sig, arena, off, len)) {
        // pinned caller arrays: no packing, the DMAs read them where they are
        CV_TRY(stage_dma_direct(st, dv, b, pk, sig, arena, off, len, s));
    } else {
        hipError_t e1 = hipSuccess;
        stage_pack(st, h, b, pk, sig, arena, off, len, pool, [&] {
            if (two_stage) e1 = hipMemcpyAsync(dv, h, st.o_off, hipMemcpyHostToDevice, s);
        });
        CV_TRY(e1);
        if (two_stage)
            CV_TRY(hipMemcpyAsync(dv + st.o_off, h + st.o_off, st.total - st.o_off, hipMemcpyHostToDevice, s));
        else
            CV_TRY(hipMemcpyAsync(dv, h, st.total, hipMemcpyHostToDevice, s));
    }
    uint8_t *dout = d.bitmap.as<uint8_t>();
    CV_TRY(launch_verify(d, sl, (uint32_t)n, dv + st.o_pk, dv + st.o_sig, dv + st.o_ar - st.lo,
                         reinterpret_cast<const uint64_t *>(dv + st.o_off), reinterpret_cast<const uint32_t *>(dv + st.o_len),
                         reinterpret_cast<uint64_t *>(dout + o_bm), status ? dout + o_st : nullptr, s, nullptr, true));
    CV_TRY(hipMemcpyAsync(d.pin_out.p, dout, status ? o_st + n : words * 8, hipMemcpyDeviceToHost, s));
    CV_TRY(hipStreamSynchronize(s));
    drain.armed = false;
    std::memcpy(bitmap + b / 64, d.pin_out.as<uint8_t>() + o_bm, words * 8);
    if (status) std::memcpy(status + b, d.pin_out.as<uint8_t>() + o_st, n);
    return CV_OK;
}

// The pipeline's sub-chunk boundaries of [b, e): [first, C, C, ..., the last two balanced]; every
// boundary but e is b + a multiple of 64 (whole bitmap words per sub-chunk).
// With ramp, the sizes after the first double (first, 2 first, 4 first, ...) until they reach C: each
// sub-chunk's copy then takes about as long as the kernels of the one before it, so the GPU is not left
// waiting for a big second sub-chunk while a small first one has long finished.
static std::vector<size_t> pipe_cuts(size_t b, size_t e, size_t first, size_t C, bool ramp = false) {
    std::vector<size_t> cut{b};
    if (e <= b) return cut;
    first = std::max<size_t>(64, first / 64 * 64);
    C = std::max<size_t>(64, C / 64 * 64);
    size_t p = b + std::min(e - b, first);
    cut.push_back(p);
    size_t step = first;
    while (p < e) {
        const size_t rem = e - p;
        step = ramp ? std::min(C, 2 * step) : C;
        const size_t m = rem <= step ? rem : rem < 2 * step ? (rem / 2 + 63) / 64 * 64 : step;
        p += m;
        cut.push_back(p);
    }
    return cut;
}

// One shard [b, e) of a large batch, pipelined: sub-chunks (multiples of 64 signatures) go through a ring
// of kRing device input blocks.  Sub-chunk j's records reach block j % kRing on the device's ONE copy
// stream — straight from the caller's arrays when they are pinned (stage_direct), else packed by the
// host threads into pinned staging block j % kRing first — and are verified on slot j % R's stream,
// which waits for that copy (event) and marks the block free when its kernels are done.  The copy
// stream waits (on the GPU) for the verify that last read a block before refilling it, so copies run
// up to kRing sub-chunks ahead of the kernels and never queue behind a running kernel on a compute
// stream.  One copy queue matters: with copies on every slot stream the runtime ran those of one
// stream as blit kernels (`__amd_rocclr_copyBuffer`, ~37 GB/s, on the CUs beside the verify kernels)
// and the C2 host call took 13.8-16 ms for 9.6 ms of kernels (profiles/r03c_timeline_*.txt).  The
// verdicts come back in ONE copy after the last verify.
// Copies a finished pipelined call's verdicts into the caller's arrays (waits for them first).
static int pipe_finish(Device &d, PipeOut &po) {
    if (!po.pending) return CV_OK;
    po.pending = false;
    // host-side join: the call's last launch group on every slot stream, then ONE verdict copy on the
    // device's output stream (which carries nothing else, so it neither waits behind the next call's
    // input copies nor holds a compute stream the next call's kernels run on)
    for (int k = 0; k < kSlots; k++)
        if (po.slot_used[k]) CV_TRY(hipEventSynchronize(po.slot_done[k]));
    if (!d.outs) CV_TRY(hipStreamCreateWithFlags(&d.outs, hipStreamNonBlocking));
    const size_t words = (po.n + 63) / 64;
    CV_TRY(hipMemcpyAsync(po.hout.p, po.dout.p, po.status ? po.o_st + po.n : words * 8, hipMemcpyDeviceToHost, d.outs));
    CV_TRY(hipStreamSynchronize(d.outs));
    std::memcpy(po.bitmap + po.b / 64, po.hout.p, words * 8);
    if (po.status) std::memcpy(po.status + po.b, po.hout.as<uint8_t>() + po.o_st, po.n);
    return CV_OK;
}

// Enqueues the pipelined verify of shard [b, e) on device d with its verdicts going to output slot
// po (which must not be pending); returns without waiting for the GPU.  The join: the device stream
// (slot 0's) waits for the other slot streams' last launch groups, copies the verdicts to po's pinned
// buffer and records po.done.  The ring's in_free / in_ready events stay valid across calls, so the
// next call's copies and kernels queue right behind this one's (cv_ed25519_verify_batch_async).
// async: the sub-chunk plan of cv_ed25519_verify_batch_async (g_async_chunk, no ramp — with a call in
// flight ahead of it the GPU is busy anyway, and bigger launches run closer to the kernels' rate)
static int pipe_enqueue(Device &d, PipeOut &po, size_t b, size_t e, const uint8_t *pk, const uint8_t *sig,
                        const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint64_t *bitmap,
                        uint8_t *status, int threads, bool async = false) {
    const size_t n = e - b;
    const size_t words = (n + 63) / 64;
    const size_t o_st = al16(words * 8), total_out = o_st + al16(n);
    // async sub-chunks: g_async_chunk, up to twice that for big shards (n / 16; same-box sweep:
    // C2 1M best at 262,144, C5 8M at 524,288, profiles/r03l_async_chunk_sweep.log)
    const size_t ach = std::max(g_async_chunk, std::min(2 * g_async_chunk, n / 16 / 64 * 64));
    const std::vector<size_t> cut = async ? pipe_cuts(b, e, ach, ach, false)
                                          : pipe_cuts(b, e, g_pipe_first, g_pipe_chunk, g_pipe_ramp != 0);
    const int nsl = g_pipe_slots;
    hipStream_t ss[kSlots] = {};
    for (int k = 0; k < nsl; k++) {
        CV_TRY(slot_stream(d, k, &ss[k]));
        CV_TRY(slot_events(d.slot[k]));
    }
    if (!d.copy) CV_TRY(hipStreamCreateWithFlags(&d.copy, hipStreamNonBlocking));
    for (int q = 0; q < kRing; q++) {
        if (!d.in_ready[q]) CV_TRY(hipEventCreateWithFlags(&d.in_ready[q], hipEventDisableTiming));
        if (!d.in_free[q]) CV_TRY(hipEventCreateWithFlags(&d.in_free[q], hipEventDisableTiming));
    }
    for (int k = 0; k < nsl; k++)
        if (!po.slot_done[k]) CV_TRY(hipEventCreateWithFlags(&po.slot_done[k], hipEventDisableTiming));
    CV_TRY(po.hout.ensure(total_out));
    CV_TRY(po.dout.ensure(total_out));
    uint8_t *dout = po.dout.as<uint8_t>();
    // error paths: drain every queue, forget the ring's state and every pending output of this device
    auto drain = on_exit([&] {
        (void)hipStreamSynchronize(d.copy);
        for (int k = 0; k < nsl; k++) (void)hipStreamSynchronize(ss[k]);
        for (int q = 0; q < kRing; q++) d.in_used[q] = d.stage_busy[q] = false;
        for (PipeOut &o : d.out)                  // an earlier call still in flight keeps its verdicts
            if (&o != &po) (void)pipe_finish(d, o);
    });
    WorkerPool *pool = &d.workers(threads);
    PipeStats ps;
    bool used[kSlots] = {};
    for (size_t j = 0; j + 1 < cut.size(); j++) {
        const size_t c0 = cut[j], c1 = cut[j + 1], m = c1 - c0;
        const int q = d.ring_next;
        d.ring_next = (d.ring_next + 1) % kRing;
        Slot &sl = d.slot[j % nsl];
        hipStream_t s = ss[j % nsl];
        used[j % nsl] = true;
        double t0 = now_s();
        const Stage st = stage_plan(c0, c1, off, len, pool);
        const bool direct = stage_direct(st, c0, pk, sig, arena, off, len);
        double t1 = now_s();
        ps.plan += t1 - t0;
        if (st.total > d.inblk[q].cap) {             // growing: the old block may still be read
            if (d.in_used[q]) CV_TRY(hipEventSynchronize(d.in_free[q]));
            CV_TRY(d.inblk[q].ensure(st.total));
        }
        if (d.in_used[q]) CV_TRY(hipStreamWaitEvent(d.copy, d.in_free[q], 0));
        uint8_t *dv = d.inblk[q].as<uint8_t>();
        if (direct) {
            t0 = now_s();
            ps.wait += t0 - t1;
            CV_TRY(stage_dma_direct(st, dv, c0, pk, sig, arena, off, len, d.copy));
            ps.direct++;
        } else {
            // staging block q is free once its previous copy has left it
            if (d.stage_busy[q]) {
                CV_TRY(hipEventSynchronize(d.in_ready[q]));
                d.stage_busy[q] = false;
            }
            CV_TRY(d.instage[q].ensure(st.total));
            t0 = now_s();
            ps.wait += t0 - t1;
            uint8_t *h = d.instage[q].as<uint8_t>();
            stage_pack(st, h, c0, pk, sig, arena, off, len, pool, [] {});
            t1 = now_s();
            ps.pack += t1 - t0;
            t0 = t1;
            CV_TRY(hipMemcpyAsync(dv, h, st.total, hipMemcpyHostToDevice, d.copy));
            d.stage_busy[q] = true;
        }
        CV_TRY(hipEventRecord(d.in_ready[q], d.copy));
        CV_TRY(hipStreamWaitEvent(s, d.in_ready[q], 0));
        const size_t w0 = (c0 - b) / 64;
        CV_TRY(launch_verify(d, sl, (uint32_t)m, dv + st.o_pk, dv + st.o_sig, dv + st.o_ar - st.lo,
                             reinterpret_cast<const uint64_t *>(dv + st.o_off),
                             reinterpret_cast<const uint32_t *>(dv + st.o_len),
                             reinterpret_cast<uint64_t *>(dout) + w0, status ? dout + o_st + (c0 - b) : nullptr, s,
                             nullptr, false));
        CV_TRY(hipEventRecord(d.in_free[q], s));
        d.in_used[q] = true;
        ps.enq += now_s() - t0;
        ps.chunks++;
    }
    // completion marks per slot stream (pipe_finish joins on the host); no GPU-side join, which would
    // hold the next call's kernels on that stream until this call had finished
    for (int k = 0; k < kSlots; k++) {
        po.slot_used[k] = k < nsl && used[k];
        if (po.slot_used[k]) CV_TRY(hipEventRecord(po.slot_done[k], ss[k]));
    }
    drain.armed = false;
    po.pending = true;
    po.gen++;
    po.bitmap = bitmap;
    po.status = status;
    po.b = b;
    po.n = n;
    po.o_st = o_st;
    {
        std::lock_guard<std::mutex> g(g_pipe_stats_mu);
        PipeStats &G = g_pipe_stats;
        G.plan += ps.plan;
        G.pack += ps.pack;
        G.wait += ps.wait;
        G.enq += ps.enq;
        G.calls++;
        G.chunks += ps.chunks;
        G.direct += ps.direct;
    }
    return CV_OK;
}

// The device's next free output slot: the older in-flight call is finished first if it still holds it.
static PipeOut &pipe_out(Device &d, int *index = nullptr) {
    PipeOut &po = d.out[d.out_next];
    if (index) *index = d.out_next;
    d.out_next = (d.out_next + 1) % kOuts;
    return po;
}

// One shard [b, e) of a large batch, pipelined (see pipe_enqueue), synchronously: the verdicts are in
// the caller's arrays on return.
static int verify_shard_pipe(Device &d, size_t b, size_t e, const uint8_t *pk, const uint8_t *sig,
                             const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint64_t *bitmap,
                             uint8_t *status, int threads) {
    PipeOut &po = pipe_out(d);
    int rc = pipe_finish(d, po);
    if (rc != CV_OK) return rc;
    rc = pipe_enqueue(d, po, b, e, pk, sig, arena, off, len, bitmap, status, threads);
    if (rc != CV_OK) return rc;
    const double t0 = now_s();
    rc = pipe_finish(d, po);
    {
        std::lock_guard<std::mutex> g(g_pipe_stats_mu);
        g_pipe_stats.sync += now_s() - t0;
    }
    return rc;
}

static int verify_shard(Device &d, size_t b, size_t e, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                        const uint64_t *off, const uint32_t *len, uint64_t *bitmap, uint8_t *status, int threads) {
    const size_t n = e - b;
    if (n == 0) return CV_OK;
    if (n > 0xffffffffull) return CV_E_TOO_LARGE;
    CV_TRY(hipSetDevice(d.ordinal));
    if (n > g_pipe_min) return verify_shard_pipe(d, b, e, pk, sig, arena, off, len, bitmap, status, threads);
    return verify_shard_small(d, b, e, pk, sig, arena, off, len, bitmap, status, threads);
}

// Shards [0, n) over the context's devices (contiguous ranges, multiples of 64) and runs fn per shard
// (fn(device, b, e, packing threads)).
template <class F> static int for_each_shard(cv_ctx *ctx, size_t n, F fn) {
    const size_t ndev = ctx->devs.size();
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int threads = (int)std::max<size_t>(1, std::min<size_t>((size_t)g_pack_threads, hw / ndev));
    size_t per = (n + ndev - 1) / ndev;
    per = (per + 63) / 64 * 64;
    if (ndev == 1 || n <= 64) return fn(ctx->devs[0], 0, n, threads);
    std::vector<int> rc(ndev, CV_OK);
    std::vector<std::thread> th;
    for (size_t k = 0; k < ndev; k++) {
        const size_t b = std::min(n, k * per), e = std::min(n, b + per);
        if (b >= e) continue;
        th.emplace_back([&, k, b, e] { rc[k] = fn(ctx->devs[k], b, e, threads); });
    }
    for (auto &t : th) t.join();
    for (int r : rc)
        if (r != CV_OK) return r;
    return CV_OK;
}

// ---------------------------------------------------------------- keyed verify (per-key comb tables)
// Makes the keys k (used[k] != 0, or all when used == nullptr) of keys[0..nk) resident in d's key
// pool and fills slot_of_key[k]; keyprep launches on s compute the tables of the new ones (at most
// kKeyprepBatch keys per launch, so the scratch stays bounded).  The caller holds the pool
// (pool_begin).  Failure leaves an empty pool (capacity 0, no resident keys), never a key mapped to
// a slot whose tables were not computed or a capacity without its buffers.
static int key_resolve(Device &d, uint32_t cap, size_t nk, const uint8_t *keys, const uint8_t *used,
                       std::vector<uint32_t> &slot_of_key, hipStream_t s) {
    KeyCache &kc = d.kc;
    auto fail = [&kc](hipError_t e) {
        kc.map.clear();
        kc.cap = 0;
        kc.resets++;
        return hip_rc(e);
    };
    size_t nused = 0;
    for (size_t k = 0; k < nk; k++) nused += used ? (used[k] != 0) : 1;
    const size_t need = std::max<size_t>(cap, nused);
    if (kc.cap < need) {                      // (re)allocate the pool; resident tables are dropped
        if (need > 0xffffffffull / 2) return CV_E_TOO_LARGE;
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) return fail(e);
        kc.map.clear();
        kc.cap = 0;
        kc.ktab.release();
        kc.kok.release();
        if ((e = kc.ktab.ensure(need * kKtabBytes)) != hipSuccess) return fail(e);
        if ((e = kc.kok.ensure(need)) != hipSuccess) return fail(e);
        kc.cap = (uint32_t)need;
    }
    if (kc.map.size() + nused > kc.cap) {     // epoch reset: every key of this call gets a fresh slot
        kc.map.clear();
        kc.resets++;
    }
    std::vector<uint8_t> miss_keys;
    std::vector<uint32_t> miss_slots;
    std::vector<std::array<uint8_t, 32>> miss;     // mapped only once their tables are enqueued
    std::unordered_map<std::array<uint8_t, 32>, uint32_t, KeyHash> fresh;   // this call's new keys
    std::array<uint8_t, 32> key;
    slot_of_key.assign(nk, 0);
    uint32_t next = (uint32_t)kc.map.size();
    for (size_t k = 0; k < nk; k++) {
        if (used && !used[k]) continue;
        std::memcpy(key.data(), keys + 32 * k, 32);
        auto it = kc.map.find(key);
        if (it != kc.map.end()) {
            slot_of_key[k] = it->second;
            kc.hits++;
            continue;
        }
        auto f = fresh.find(key);
        if (f != fresh.end()) {                   // a key repeated inside this call's key list
            slot_of_key[k] = f->second;
            continue;
        }
        const uint32_t slot = next++;
        fresh.emplace(key, slot);
        slot_of_key[k] = slot;
        miss_keys.insert(miss_keys.end(), key.begin(), key.end());
        miss_slots.push_back(slot);
        kc.misses++;
    }
    const size_t m = miss_slots.size();
    for (size_t k0 = 0; k0 < m; k0 += kKeyprepBatch) {
        const size_t mk = std::min(kKeyprepBatch, m - k0);
        hipError_t e = kc.keys.ensure(mk * 32);
        if (e == hipSuccess) e = kc.slots.ensure(mk * 4);
        if (e == hipSuccess) e = kc.scratch.ensure(mk * kKtabBytes);
        // the previous batch's keyprep may still read keys / slots / scratch: order the copies after it
        // (same stream), and the host vectors stay alive until the synchronize below
        if (e == hipSuccess) e = hipMemcpyAsync(kc.keys.p, miss_keys.data() + 32 * k0, mk * 32, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(kc.slots.p, miss_slots.data() + k0, mk * 4, hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = cvk_keyprep((uint32_t)mk, kc.keys.as<uint8_t>(), kc.slots.as<uint32_t>(), kc.scratch.as<uint32_t>(),
                            kc.ktab.as<uint32_t>(), kc.kok.as<uint8_t>(), s);
        if (e == hipSuccess && k0 + mk < m) e = hipStreamSynchronize(s);   // buffers are reused by the next batch
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(s);
            return fail(e);
        }
    }
    if (m) {
        // the pageable copies above read miss_keys / miss_slots asynchronously: keep them alive
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) return fail(e);
    }
    for (auto &kv : fresh) kc.map.emplace(kv.first, kv.second);
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
    Slot &sl = pick_slot(d, s);
    CV_TRY(ensure_verify_ws(sl, n));
    CV_TRY(ws_begin(d, sl, s));
    CV_TRY(pool_begin(d.kc, s));
    auto drain = on_exit([s] { (void)hipStreamSynchronize(s); });   // error paths: no copy outlives the call
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
    CV_TRY(cvk_verify_keyed((uint32_t)n, d.pk.as<uint8_t>(), kc.key_index.as<uint32_t>(), kc.slot_of_key.as<uint32_t>(),
                            kc.ktab.as<uint32_t>(), kc.kok.as<uint8_t>(), d.sig.as<uint8_t>(),
                            d.arena.as<uint8_t>() - lo, d.off.as<uint64_t>(), d.len.as<uint32_t>(),
                            d.bitmap.as<uint64_t>(), status ? d.status.as<uint8_t>() : nullptr, sl.ws_hs.as<uint32_t>(),
                            sl.ws_R.as<uint32_t>(), sl.ws_ok.as<uint8_t>(), sl.ws_cap, s, nullptr));
    CV_TRY(ws_end(sl, s));
    CV_TRY(pool_end(kc, s));
    CV_TRY(hipMemcpyAsync(bitmap + b / 64, d.bitmap.p, words * 8, hipMemcpyDeviceToHost, s));
    if (status) CV_TRY(hipMemcpyAsync(status + b, d.status.p, n, hipMemcpyDeviceToHost, s));
    CV_TRY(hipStreamSynchronize(s));
    drain.armed = false;
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
        return for_each_shard(ctx, n, [&](Device &d, size_t b, size_t e, int) {
            return verify_shard_keyed(ctx->key_cap, d, b, e, nk, keys.data(), key_index.data(), sig, msg_arena, msg_off,
                                      msg_len, verdict_bitmap, status);
        });
    }
    return for_each_shard(ctx, n, [&](Device &d, size_t b, size_t e, int threads) {
        return verify_shard(d, b, e, pk, sig, msg_arena, msg_off, msg_len, verdict_bitmap, status, threads);
    });
}

int cv_ed25519_verify_batch_async(cv_ctx *ctx, size_t n, const uint8_t *pk, const uint8_t *sig,
                                  const uint8_t *msg_arena, const uint64_t *msg_off, const uint32_t *msg_len,
                                  uint64_t *verdict_bitmap, uint8_t *status, uint64_t *ticket) {
    if (!ctx || !ticket) return CV_E_ARGS;
    *ticket = 0;
    if (n == 0) return CV_OK;
    if (!pk || !sig || !msg_off || !msg_len || !verdict_bitmap) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    std::vector<std::array<uint64_t, 3>> parts(ctx->devs.size(), {UINT64_MAX, 0, 0});
    const int rc = for_each_shard(ctx, n, [&](Device &d, size_t b, size_t e, int threads) {
        if (e - b > 0xffffffffull) return CV_E_TOO_LARGE;
        CV_TRY(hipSetDevice(d.ordinal));
        int k = 0;
        PipeOut &po = pipe_out(d, &k);
        int r = pipe_finish(d, po);               // the slot's previous call (its verdicts land first)
        if (r == CV_OK)
            r = pipe_enqueue(d, po, b, e, pk, sig, msg_arena, msg_off, msg_len, verdict_bitmap, status, threads, true);
        if (r == CV_OK) parts[(size_t)(&d - ctx->devs.data())] = {(uint64_t)(&d - ctx->devs.data()), (uint64_t)k, po.gen};
        return r;
    });
    if (rc != CV_OK) {
        // a shard failed: the shards that did enqueue are waited for and dropped here — nothing may
        // read the caller's arrays or write its bitmap after an error return
        for (const auto &p : parts) {
            if (p[0] == UINT64_MAX) continue;
            Device &d = ctx->devs[p[0]];
            PipeOut &po = d.out[p[1]];
            (void)hipSetDevice(d.ordinal);
            for (int k = 0; k < kSlots; k++)
                if (po.slot_used[k]) (void)hipEventSynchronize(po.slot_done[k]);
            if (d.copy) (void)hipStreamSynchronize(d.copy);
            po.pending = false;
        }
        return rc;
    }
    std::vector<std::array<uint64_t, 3>> live;
    for (const auto &p : parts)
        if (p[0] != UINT64_MAX) live.push_back(p);
    *ticket = ++ctx->next_ticket;
    ctx->tickets.emplace(*ticket, std::move(live));
    return CV_OK;
}

int cv_wait(cv_ctx *ctx, uint64_t ticket) {
    if (!ctx) return CV_E_ARGS;
    if (ticket == 0) return CV_OK;
    std::lock_guard<std::mutex> g(ctx->mu);
    auto it = ctx->tickets.find(ticket);
    if (it == ctx->tickets.end()) return CV_E_ARGS;
    int rc = CV_OK;
    for (const auto &p : it->second) {
        Device &d = ctx->devs[p[0]];
        PipeOut &po = d.out[p[1]];
        if (po.gen != p[2] || !po.pending) continue;   // already copied (its slot was reused)
        if (hipSetDevice(d.ordinal) != hipSuccess) {
            rc = CV_E_HIP;
            continue;
        }
        const int r = pipe_finish(d, po);
        if (r != CV_OK) rc = r;
    }
    ctx->tickets.erase(it);
    return rc;
}

int cv_ed25519_verify_batch_keyed(cv_ctx *ctx, size_t n, size_t nkeys, const uint8_t *keys, const uint32_t *key_index,
                                  const uint8_t *sig, const uint8_t *msg_arena, const uint64_t *msg_off,
                                  const uint32_t *msg_len, uint64_t *verdict_bitmap, uint8_t *status) {
    if (!ctx) return CV_E_ARGS;
    if (n == 0) return CV_OK;
    if (!keys || !key_index || !sig || !msg_off || !msg_len || !verdict_bitmap || nkeys == 0) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    return for_each_shard(ctx, n, [&](Device &d, size_t b, size_t e, int) {
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
    return for_each_shard(ctx, n, [&](Device &d, size_t b, size_t e, int) {
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
    CV_TRY(launch_verify(*d, pick_slot(*d, s), (uint32_t)n, static_cast<const uint8_t *>(d_pk),
                         static_cast<const uint8_t *>(d_sig), static_cast<const uint8_t *>(d_arena),
                         static_cast<const uint64_t *>(d_off), static_cast<const uint32_t *>(d_len),
                         static_cast<uint64_t *>(d_bitmap), static_cast<uint8_t *>(d_status), s, nullptr, true));
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
    Slot &sl = pick_slot(*d, s);
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    hipError_t e = hipSuccess;
    for (int k = 0; k < 4 && e == hipSuccess; k++) e = hipEventCreate(&ev[k]);
    // one workspace chunk at a time (chunk starts are multiples of 64: whole bitmap words)
    for (size_t c0 = 0; c0 < n && e == hipSuccess; c0 += kVerifyChunk) {
        const size_t m = std::min<size_t>(kVerifyChunk, n - c0);
        e = launch_verify(*d, sl, (uint32_t)m, static_cast<const uint8_t *>(d_pk) + c0 * 32,
                          static_cast<const uint8_t *>(d_sig) + c0 * 64, static_cast<const uint8_t *>(d_arena),
                          static_cast<const uint64_t *>(d_off) + c0, static_cast<const uint32_t *>(d_len) + c0,
                          static_cast<uint64_t *>(d_bitmap) + c0 / 64, nullptr, s, ev, false);
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
    Slot &sl = pick_slot(*d, s);
    if (e == hipSuccess) e = ensure_verify_ws(sl, n);
    if (e == hipSuccess && phase_ms) e = hipEventRecord(ev[0], s);
    if (e == hipSuccess) e = ws_begin(*d, sl, s);
    if (e == hipSuccess) e = pool_begin(d->kc, s);
    std::vector<uint32_t> sok;
    int rc = e == hipSuccess ? key_resolve(*d, ctx->key_cap, nkeys, hkeys.data(), nullptr, sok, s) : hip_rc(e);
    KeyCache &kc = d->kc;
    if (rc == CV_OK) rc = hip_rc(kc.slot_of_key.ensure(nkeys * 4));
    // slot_of_key goes up through the pool's pinned staging, which the previous keyed call's upload may
    // still be reading: that call's pool event (after its verify) has passed once its upload has
    if (rc == CV_OK && kc.pin_busy) rc = hip_rc(hipEventSynchronize(kc.pin_ev));
    if (rc == CV_OK) rc = hip_rc(kc.pin.ensure(nkeys * 4));
    if (rc == CV_OK) {
        std::memcpy(kc.pin.p, sok.data(), nkeys * 4);
        rc = hip_rc(hipMemcpyAsync(kc.slot_of_key.p, kc.pin.p, nkeys * 4, hipMemcpyHostToDevice, s));
    }
    if (rc == CV_OK && !kc.pin_ev) rc = hip_rc(hipEventCreateWithFlags(&kc.pin_ev, hipEventDisableTiming));
    if (rc == CV_OK) rc = hip_rc(hipEventRecord(kc.pin_ev, s));
    kc.pin_busy = rc == CV_OK;
    if (rc == CV_OK)
        rc = hip_rc(cvk_verify_keyed((uint32_t)n, static_cast<const uint8_t *>(d_keys),
                                     static_cast<const uint32_t *>(d_key_index), kc.slot_of_key.as<uint32_t>(),
                                     kc.ktab.as<uint32_t>(), kc.kok.as<uint8_t>(), static_cast<const uint8_t *>(d_sig),
                                     static_cast<const uint8_t *>(d_arena), static_cast<const uint64_t *>(d_off),
                                     static_cast<const uint32_t *>(d_len), static_cast<uint64_t *>(d_bitmap),
                                     static_cast<uint8_t *>(d_status), sl.ws_hs.as<uint32_t>(), sl.ws_R.as<uint32_t>(),
                                     sl.ws_ok.as<uint8_t>(), sl.ws_cap, s, phase_ms ? ev + 1 : nullptr));
    if (sl.ev) {
        const hipError_t e2 = ws_end(sl, s);
        if (rc == CV_OK) rc = hip_rc(e2);
    }
    if (d->kc.ev) {
        const hipError_t e2 = pool_end(d->kc, s);
        if (rc == CV_OK) rc = hip_rc(e2);
    }
    if (rc != CV_OK) (void)hipStreamSynchronize(s);   // error paths: nothing queued outlives the call
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
// scoped device scratch and events of the calibration / diagnostic calls (freed on every return path)
struct ScopedMem {
    void *p = nullptr;
    ~ScopedMem() {
        if (p) (void)hipFree(p);
    }
};
struct ScopedEvents {
    hipEvent_t e[2] = {nullptr, nullptr};
    hipError_t create() {
        hipError_t r = hipSuccess;
        for (hipEvent_t &x : e)
            if (r == hipSuccess) r = hipEventCreate(&x);
        return r;
    }
    ~ScopedEvents() {
        for (hipEvent_t x : e)
            if (x) (void)hipEventDestroy(x);
    }
};

int cv_calibrate(cv_ctx *ctx, int device, double *mad_per_s, double *femul_per_s) {
    if (!ctx) return CV_E_ARGS;
    Device *d = find_dev(ctx, device);
    if (!d) return CV_E_ARGS;
    CV_TRY(hipSetDevice(d->ordinal));
    hipDeviceProp_t prop;
    CV_TRY(hipGetDeviceProperties(&prop, d->ordinal));
    const uint32_t blocks = (uint32_t)prop.multiProcessorCount * 8;   // 8 waves per SIMD worth of work
    ScopedMem scratch;
    ScopedEvents ev;
    CV_TRY(hipMalloc(&scratch.p, 64));
    CV_TRY(ev.create());
    double rates[2] = {0, 0};
    for (int which = 0; which < 2; which++) {
        const uint32_t iters = which == 0 ? 20000 : 2000;
        CV_TRY(cvk_calibrate(iters / 10, which, blocks, scratch.p, d->stream));   // warm-up
        CV_TRY(hipEventRecord(ev.e[0], d->stream));
        CV_TRY(cvk_calibrate(iters, which, blocks, scratch.p, d->stream));
        CV_TRY(hipEventRecord(ev.e[1], d->stream));
        CV_TRY(hipEventSynchronize(ev.e[1]));
        float ms = 0;
        CV_TRY(hipEventElapsedTime(&ms, ev.e[0], ev.e[1]));
        const double per_thread = which == 0 ? 128.0 * iters : 4.0 * iters;
        rates[which] = per_thread * blocks * 256.0 / (ms * 1e-3);
    }
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
    ScopedMem buf;
    ScopedEvents ev;
    CV_TRY(hipMalloc(&buf.p, 64));
    CV_TRY(ev.create());
    uint64_t *clkbuf = static_cast<uint64_t *>(buf.p);
    CV_TRY(cvk_mad_clock(iters / 10, blocks, clkbuf, d->stream));
    CV_TRY(hipEventRecord(ev.e[0], d->stream));
    CV_TRY(cvk_mad_clock(iters, blocks, clkbuf, d->stream));
    CV_TRY(hipEventRecord(ev.e[1], d->stream));
    CV_TRY(hipEventSynchronize(ev.e[1]));
    float ms = 0.f;
    uint64_t clk[2] = {0, 0};
    CV_TRY(hipEventElapsedTime(&ms, ev.e[0], ev.e[1]));
    CV_TRY(hipMemcpy(clk, clkbuf, 16, hipMemcpyDeviceToHost));
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
// their sum, out[6] = waves measured, out[7] = the SHA-512 part of the hash phase.  The workspace is
// the device stream's verify workspace slot.
int cv_diag_prep_phases(cv_ctx *ctx, int device, size_t n, const void *d_pk, const void *d_sig, const void *d_arena,
                        const void *d_off, const void *d_len, double *out) {
    if (!ctx || !out || n == 0) return CV_E_ARGS;
    if (n > kVerifyChunk) return CV_E_TOO_LARGE;
    Device *d = find_dev(ctx, device);
    if (!d || !d_pk || !d_sig || !d_arena || !d_off || !d_len) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    CV_TRY(hipSetDevice(d->ordinal));
    Slot &sl = pick_slot(*d, d->stream);
    CV_TRY(ensure_verify_ws(sl, n));
    const size_t waves = (n + 63) / 64;
    ScopedMem st;
    CV_TRY(hipMalloc(&st.p, waves * 64));
    CV_TRY(ws_begin(*d, sl, d->stream));
    hipError_t e = cvk_prep_probe((uint32_t)n, static_cast<const uint8_t *>(d_pk), static_cast<const uint8_t *>(d_sig),
                                  static_cast<const uint8_t *>(d_arena), static_cast<const uint64_t *>(d_off),
                                  static_cast<const uint32_t *>(d_len), sl.ws_dig.as<uint32_t>(), sl.ws_tab.as<uint32_t>(),
                                  sl.ws_cap, static_cast<uint64_t *>(st.p), d->stream);
    const hipError_t e2 = ws_end(sl, d->stream);
    if (e == hipSuccess) e = e2;
    std::vector<uint64_t> h(waves * 8);
    const hipError_t e3 = hipStreamSynchronize(d->stream);   // also on error: st is freed on return
    if (e == hipSuccess) e = e3;
    if (e == hipSuccess) e = hipMemcpy(h.data(), st.p, waves * 64, hipMemcpyDeviceToHost);
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
