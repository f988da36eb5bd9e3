// cv_api.cpp — the C-ABI (include/cordaverify.h): contexts and their options, per-device executors (one lock,
// one persistent worker thread and a load count per device; batches routed whole to one device or cut over
// several), verify workspace slots, the host-buffer pipeline (copy stream + input ring, direct DMA from pinned
// buffers) for plain, keyed and Merkle batches with synchronous and asynchronous forms, and the
// device-resident entry points used by bench.py.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <chrono>
#include <cmath>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
#include <unordered_map>
#include <vector>

// The library is built with hidden host symbols (corda_amd/build.py: -fvisibility=hidden); only the
// entry points the header declares are exported.
#pragma GCC visibility push(default)
#include "../../include/cordaverify.h"
#pragma GCC visibility pop
#include "cv_launch.h"

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    // slack: allocate 1.25x the request (buffers that grow with the batch); exact sizes for buffers whose
    // caller already sized them (the input ring's blocks)
    hipError_t ensure(size_t bytes, bool slack = true) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(slack ? bytes + bytes / 4 : bytes, 4096);
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
    DevBuf ktab, kok, keys, slots, scratch;
    uint32_t cap = 0;
    std::unordered_map<std::array<uint8_t, 32>, uint32_t, KeyHash> map;
    uint64_t hits = 0, misses = 0, resets = 0;
    // the last stream that used the pool and an event after that use (pool_end: what an epoch reset waits
    // for), and the stream of the last table WRITE (keyprep) with an event after it (key_resolve): a reader on
    // another stream waits only for that (pool_begin) — readers do not wait for readers
    hipStream_t last = nullptr;
    hipEvent_t ev = nullptr;
    hipStream_t wlast = nullptr;
    hipEvent_t wev = nullptr;
    // the device-API keyed call's slot_of_key: device copy, pinned staging, event after its upload
    DevBuf slot_of_key;
    PinBuf pin;
    hipEvent_t pin_ev = nullptr;
    bool pin_busy = false;
};

// One verify workspace (per signature: hs 64 B, 2 tables 2 x 1440 B, R record 128 B, ok 1 B, half-size
// digits 292 B) with what orders its use across streams, its drain-overlap helper, and the Merkle leaf
// digests of the sub-chunks that run on it.  A device has kSlots of them: device-API calls on different
// streams take different slots and run concurrently; the host-buffer pipeline deals its sub-chunks
// round-robin over two slots.
struct Slot {
    DevBuf ws_hs, ws_tab, ws_R, ws_ok, ws_dig, mdig;
    uint32_t ws_cap = 0;
    hipStream_t last = nullptr;   // the stream of the last launch group on this workspace
    hipEvent_t ev = nullptr;      // recorded after that group
    uint64_t stamp = 0;           // last use (least-recently-used choice)
    CvkSplit split;               // drain-overlap helper stream + events (created on first need)
    hipStream_t stream = nullptr; // the slot's own stream (slot 0: the device stream)
    PinBuf pin_in;                // small-path staging of one batch: pk | sig | off | len | arena
    DevBuf packed;                // its device copy
    PinBuf pin_head;              // mid-size batches (verify_shard_mid): pk | sig, staged before the range scan
    DevBuf head;                  // its device copy
};
constexpr int kSlots = 4;
constexpr int kPipeSlots = 4;   // most compute slots a pipelined call deals its sub-chunks over (PipeFrame::ns)
// input blocks of the host pipeline on the device: copies run up to kRing sub-chunks ahead of the kernels, so
// a call's copies are all queued early and a Merkle call submitted behind a verify call copies its leaves
// while that verify's kernels run (round 4: with 6 blocks the verify's copies were paced by its kernels and
// the Merkle copies queued behind them, host C3 0.67x of the device rate)
constexpr int kRing = 16;
constexpr int kStage = 6;       // pinned host staging blocks (pageable inputs are packed into them)
constexpr int kOuts = 4;        // pipelined host calls in flight per device (async verify + Merkle calls)
constexpr size_t kFailKeep = 1024;   // failed asynchronous calls remembered per output (PipeOut::failed)
constexpr int kTlVals = 14;          // CV_STATS_TIMELINE values per timed call (PipeOut::tl_sum)

// The output of one pipelined host call on one device: its results on the device (dout), the pinned
// copy they come back through, and what pipe_finish copies where.  pending: enqueued, results not yet in
// the caller's arrays; gen counts the calls that used this output.  mu serialises finishing it (cv_wait
// runs without the device lock) against reusing it (under the device lock; order: device -> output).
struct PipeOut {
    std::mutex mu;
    DevBuf dout;
    PinBuf hout;
    // after this call's last launch group on each slot stream, and (Merkle calls) on the copy stream
    hipEvent_t slot_done[kPipeSlots + 1] = {};
    bool slot_used[kPipeSlots + 1] = {};
    bool pending = false;
    uint64_t gen = 0;
    struct Seg {
        void *dst;
        size_t off, len;
    };
    Seg seg[4] = {};
    int nseg = 0;
    // keyed calls: the call's distinct keys and their pool slots on the device (kdev: keys | slot_of_key,
    // uploaded through kstage), the auto path's key_index (pinned, DMAed per sub-chunk)
    DevBuf kdev;
    PinBuf kstage, kidx;
    PinBuf tstage;   // transaction calls: the shard's signature boundaries when the caller's are pageable
    hipEvent_t copied = nullptr;   // after the call's result copies on the output stream (pipe_copy_back)
    // CV_OPT_TIMELINE (synchronous calls): timing events — [0] the first input DMA's start, then per sub-chunk j
    // [1 + 3j] its DMA's end (copy stream), [2 + 3j] its launch group's start, [3 + 3j] its end (slot stream);
    // summarised by pipe_copy_back into tl_sum (the result copies timed on the host there)
    std::vector<hipEvent_t> tl;
    int tl_n = 0;
    size_t tl_first = 0;
    bool tl_ready = false;
    // ramp, last DMA end, span, busy, idle, tail, result copy (ms); first sub-chunk; Merkle-group busy, verify-group
    // busy, last Merkle DMA end (ms); launch groups; host: call entry -> first input DMA enqueued, GPU work joined ->
    // results in the caller's arrays (ms)
    double tl_sum[kTlVals] = {};
    double tl_pre_ms = 0, tl_join_s = 0;
    std::vector<uint8_t> tl_merkle;   // per launch group: 1 = a Merkle group (cv_verify_transactions), 0 = verify
    hipEvent_t tl_ev(size_t k) {
        while (tl.size() <= k) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            tl.push_back(e);
        }
        return tl[k];
    }
    // asynchronous calls on this output whose finish failed: (gen, error), kept after the output is reused so a
    // cv_wait on such a call still returns its error.  Only ticketed calls are recorded (a synchronous call returns
    // its error itself), and a ticket whose call has finished leaves the live map, with its result, at the next
    // ticket_add once 64 are live; so fewer than 64 + kOuts x devices recorded failures can still be needed, and
    // the list keeps kFailKeep (a fixed 64 could evict a live ticket's failure behind failing
    // synchronous calls, and cv_wait then returned CV_OK).
    bool ticketed = false;
    std::deque<std::pair<uint64_t, int>> failed;
    int result_of(uint64_t g) const {
        for (const auto &f : failed)
            if (f.first == g) return f.second;
        return CV_OK;
    }
};

// A fixed set of host threads for index-parallel jobs (the host-buffer path's packing, range scans and key
// dedupe): run(ntasks, fn) calls fn(i) for every i in [0, ntasks) on the helpers and the calling thread and
// returns when all are done.  One per device, used under the device lock.
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
    // The caller works through the tasks too and returns once every task is done and every helper that
    // joined has left: helpers still asleep are not waited for (their wake-up, 10-30 us, used to be on
    // every call's critical path), and one that wakes after the run finds no job and sleeps again.
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
            done_.store(0);
            gen_++;
        }
        cv_.notify_all();
        drain(fn, ntasks);
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return active_ == 0 && done_.load() == ntasks; });
        job_ = nullptr;
    }

  private:
    void drain(const std::function<void(size_t)> &fn, size_t ntasks) {
        for (size_t i; (i = next_.fetch_add(1)) < ntasks;) {
            fn(i);
            done_.fetch_add(1);
        }
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
                if (!job_) continue;   // that run is over
                job = job_;
                ntasks = ntasks_;
                active_++;
            }
            drain(*job, ntasks);
            {
                std::lock_guard<std::mutex> g(mu_);
                if (--active_ == 0) done_cv_.notify_one();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t)> *job_ = nullptr;
    size_t ntasks_ = 0, active_ = 0;
    std::atomic<size_t> next_{0}, done_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// One persistent thread per device that runs the shards other threads hand it (dispatch), in order.
class DeviceWorker {
  public:
    DeviceWorker() : th_([this] { loop(); }) {}
    ~DeviceWorker() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_one();
        th_.join();
    }
    void post(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(std::move(f));
        }
        cv_.notify_one();
    }

  private:
    void loop() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;   // stop requested and nothing left
                f = std::move(q_.front());
                q_.pop_front();
            }
            f();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    bool stop_ = false;
    std::thread th_;
};

struct Device {
    int ordinal = 0;
    // mu: held for the whole of a synchronous shard and while an asynchronous one is enqueued; load: the
    // shards in progress or queued on this device (routing); worker: runs shards handed over by dispatch
    std::mutex mu;
    std::atomic<int> load{0};
    std::unique_ptr<DeviceWorker> worker;
    std::mutex worker_mu;   // creation of the worker
    hipStream_t stream = nullptr;
    DevBuf pk, sig, arena, off, len, bitmap, status, seed, tx_begin, digest, ids;
    PinBuf pin_out;                      // small-path verify outputs: bitmap | status
    // zero-copy notary path (verify_shard_small_zc): fine-grained pinned host memory the kernels read
    // (packed records) and store into (verdict nibbles | status) over PCIe
    PinBuf zc_in, zc_out;
    DevBuf pmt;                          // partial Merkle trees: inputs, outputs and workspace, packed
    Slot slot[kSlots];
    uint64_t clock = 0;
    KeyCache kc;
    std::unique_ptr<WorkerPool> pool;    // host packing threads (created on the first large host batch)
    // The host pipeline's input ring: sub-chunk j's records go into device block j % kRing by the ONE copy
    // stream (so every H2D copy runs on one DMA queue, never as a blit kernel beside the verify kernels),
    // packed first into the next pinned staging block when the caller's arrays are pageable.  in_ready[q]:
    // after block q's copies (copy stream); in_free[q]: after the kernels that read it (its slot stream);
    // stage_ev[k]: after the copy out of staging block k.
    hipStream_t copy = nullptr;
    hipStream_t outs = nullptr;          // the pipeline's result copies (pipe_finish)
    PipeOut out[kOuts];
    int out_next = 0;
    DevBuf inblk[kRing];
    hipEvent_t in_ready[kRing] = {}, in_free[kRing] = {};
    bool in_used[kRing] = {};
    int ring_next = 0;
    size_t ring_max = 0;                 // the largest ring block (blocks grow to it)
    PinBuf instage[kStage];
    hipEvent_t stage_ev[kStage] = {};
    bool stage_busy[kStage] = {};
    int stage_next = 0;
    // transaction calls: after each Merkle launch group (the signature groups wait for it), + one join event
    std::vector<hipEvent_t> mev;
    // transaction calls with CV_OPT_TXS_MERKLE_STREAM = 2: the stream their Merkle groups run on (created on first
    // use) and those groups' leaf-digest buffer (the groups run one after another on it)
    hipStream_t mstream = nullptr;
    DevBuf mdigest;
    WorkerPool &workers(int threads) {
        if (!pool || pool->threads() != threads) {
            pool.reset();
            pool.reset(new WorkerPool(threads - 1));
        }
        return *pool;
    }
    void post(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> g(worker_mu);
            if (!worker) worker.reset(new DeviceWorker());
        }
        worker->post(std::move(f));
    }
};

// key-table pool capacity per device (keys); 66 KB of tables per key (1.1 GB at the default; the pool
// grows to a call's distinct keys when they exceed it)
constexpr uint32_t kDefaultKeyCap = 1u << 14;
constexpr size_t kKtabBytes = 16512 * 4;  // CV_KTAB_WORDS: 4 comb rows x 129 affine entries x 128 B
constexpr size_t kTabBytes = 9 * 40 * 4;  // CV_TAB_WORDS: k*P, k = 0..8, cached form (cv_verify.h)
// new keys' tables are computed in launches of at most this many keys (bounded keyprep scratch: 270 MB)
constexpr size_t kKeyprepBatch = 4096;

// Verify workspace capacity: batches above it run in chunks of this many signatures (~13.4 GB of
// workspace at 2^22; same-box A/B at 8M signatures: 2^21 73.2, 2^22 72.4, 2^23 72.4 ms -- fewer
// chunk tails to drain; whole-round chunks of 1,966,080 were slower, 73.4 ms).
constexpr uint32_t kVerifyChunk = 1u << 22;

// ---------------------------------------------------------------- options (cv_set_option)
struct OptDesc {
    int64_t def, lo, hi;
};
static const OptDesc kOpt[CV_OPT_COUNT] = {
    {0, 0, 0},                          // (unused: options start at 1)
    {4096, 0, 1 << 20},                 // CV_OPT_TRI_MAX
    {32768, 0, 1 << 22},                // CV_OPT_QUAD_MAX
    {1, 0, 2},                          // CV_OPT_DRAIN_SPLIT
    {10, 5, 50},                        // CV_OPT_DRAIN_SPLIT_PCT
    {131072, 64, (int64_t)1 << 40},     // CV_OPT_PIPE_MIN
    {32768, 64, 1 << 24},               // CV_OPT_PIPE_FIRST
    {262144, 64, 1 << 24},              // CV_OPT_PIPE_CHUNK
    {196608, 64, 1 << 24},              // CV_OPT_ASYNC_CHUNK (one round of resident waves on MI355X)
    {8, 1, 64},                         // CV_OPT_HOST_THREADS
    {3, 0, 3},                          // CV_OPT_SMALL_ZERO_COPY
    {16384, 1, (int64_t)1 << 40},       // CV_OPT_SMALL_DIRECT_MIN
    {1, 0, 1},                          // CV_OPT_AUTO_KEYED
    {4096, 64, (int64_t)1 << 40},       // CV_OPT_SHARD_MIN
    {262144, 64, (int64_t)1 << 40},     // CV_OPT_SPREAD_MIN
    {262144, 1, 1 << 24},               // CV_OPT_MERKLE_CHUNK
    {32768, 1, (int64_t)1 << 40},       // CV_OPT_PREP_OVERLAP_MIN
    {0, 0, 1},                          // CV_OPT_TIMELINE
    {16, 1, 1024},                      // CV_OPT_PIPE_SPLIT
    {0, 0, 1},                          // CV_OPT_PIPE_OVERLAP_FIRST
    {1, 1, 16},                         // CV_OPT_MID_PIECES
    {2, 2, 4},                          // CV_OPT_PIPE_SLOTS
    {2, 0, 2},                          // CV_OPT_TXS_MERKLE_STREAM
};

// A snapshot of a context's options, taken once per call.
struct Opts {
    CvkPlan plan;
    size_t pipe_min, pipe_first, pipe_chunk, async_chunk, small_direct_min, shard_min, spread_min, merkle_chunk;
    size_t prep_overlap_min;
    size_t pipe_split, mid_pieces, pipe_slots;
    int txs_merkle_stream;
    int threads, small_zc, auto_keyed, timeline, pipe_overlap_first;
};

// host-side time of the pipelined path (cv_diag_stats CV_STATS_PIPE), of the zero-copy small path
// (CV_STATS_SMALL) and the routing counters (CV_STATS_ROUTE)
struct Stats {
    double pipe[5] = {};   // plan, pack, wait, enqueue, sync (seconds)
    uint64_t pipe_calls = 0, pipe_chunks = 0, pipe_direct = 0;
    double small[5] = {};  // plan + setup, pack, launch, sync, assemble
    uint64_t small_calls = 0;
    uint64_t calls = 0, routed_whole = 0, split_calls = 0, shards = 0, keyed_calls = 0, keyed_chunks = 0,
             merkle_calls = 0, merkle_chunks = 0;
    double tl[kTlVals + 1] = {};   // CV_STATS_TIMELINE sums (PipeOut::tl_sum) + calls
};

static inline double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

hipError_t slot_events(Slot &sl) {
    hipError_t e = hipSuccess;
    if (!sl.ev && (e = hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming)) != hipSuccess) return e;
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
    if (e == hipSuccess) e = hipEventCreateWithFlags(&x.done2, hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&x.s2, hipStreamNonBlocking);
    if (e != hipSuccess) {
        for (hipEvent_t v : {x.start, x.done2})
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
// waits for it instead of racing on it.  Callers hold the device lock around ws_begin .. ws_end.
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
    if (!kc.wev && (e = hipEventCreateWithFlags(&kc.wev, hipEventDisableTiming)) != hipSuccess) return e;
    if (kc.wlast && kc.wlast != s) e = hipStreamWaitEvent(s, kc.wev, 0);
    return e;
}
hipError_t pool_end(KeyCache &kc, hipStream_t s) {
    kc.last = s;
    return hipEventRecord(kc.ev, s);
}

// One verify launch group on slot sl, stream s.  split: the drain-overlap sub-chunks may be used.
hipError_t launch_verify(Device &d, const CvkPlan &plan, Slot &sl, uint32_t n, const uint8_t *pk, const uint8_t *sig,
                         const uint8_t *arena, const uint64_t *off, const uint32_t *len, uint64_t *bitmap,
                         uint8_t *status, hipStream_t s, hipEvent_t *ev, bool split,
                         const CvkPrepOverlap *po = nullptr) {
    hipError_t e = ensure_verify_ws(sl, n);
    const hipStream_t prev = sl.last;
    if (e == hipSuccess) e = ws_begin(d, sl, s);
    // the helper stream writes the workspace too: it waits for the slot's previous user as s does
    if (e == hipSuccess && po && prev && prev != s) e = hipStreamWaitEvent(po->aux, sl.ev, 0);
    if (e != hipSuccess) return e;
    if (split && plan.split && n >= 131072) (void)slot_split(d, sl);   // without a helper the chunk runs whole
    e = cvk_verify(&plan, n, pk, sig, arena, off, len, bitmap, status, sl.ws_tab.as<uint32_t>(), sl.ws_ok.as<uint8_t>(),
                   sl.ws_dig.as<uint32_t>(), sl.ws_cap, s, ev, split && sl.split.s2 ? &sl.split : nullptr, po);
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
    std::vector<std::unique_ptr<Device>> devs;
    std::atomic<int64_t> opt[CV_OPT_COUNT];
    std::atomic<uint32_t> key_cap{kDefaultKeyCap};
    std::atomic<uint32_t> rr{0};            // routing: where the search for the least loaded device starts
    // asynchronous calls: ticket -> (device index, output index, that output's gen) per shard
    std::mutex tk_mu;
    uint64_t next_ticket = 0;
    std::unordered_map<uint64_t, std::vector<std::array<uint64_t, 3>>> tickets;
    std::map<uint64_t, int> tickets_done;   // finished tickets pruned from `tickets`, with their result
    std::mutex st_mu;
    Stats stats;
    cv_ctx() {
        for (int k = 0; k < CV_OPT_COUNT; k++) opt[k].store(kOpt[k].def);
    }
    Opts opts() const {
        Opts o;
        o.plan.tri_max = (uint32_t)opt[CV_OPT_TRI_MAX].load();
        o.plan.quad_max = (uint32_t)opt[CV_OPT_QUAD_MAX].load();
        o.plan.split = (int)opt[CV_OPT_DRAIN_SPLIT].load();
        o.plan.split_pct = (int)opt[CV_OPT_DRAIN_SPLIT_PCT].load();
        o.pipe_min = (size_t)opt[CV_OPT_PIPE_MIN].load();
        o.pipe_first = (size_t)opt[CV_OPT_PIPE_FIRST].load() / 64 * 64;
        o.pipe_chunk = (size_t)opt[CV_OPT_PIPE_CHUNK].load() / 64 * 64;
        o.async_chunk = (size_t)opt[CV_OPT_ASYNC_CHUNK].load() / 64 * 64;
        o.threads = (int)opt[CV_OPT_HOST_THREADS].load();
        o.small_zc = (int)opt[CV_OPT_SMALL_ZERO_COPY].load();
        o.small_direct_min = (size_t)opt[CV_OPT_SMALL_DIRECT_MIN].load();
        o.auto_keyed = (int)opt[CV_OPT_AUTO_KEYED].load();
        o.shard_min = (size_t)opt[CV_OPT_SHARD_MIN].load();
        o.spread_min = (size_t)opt[CV_OPT_SPREAD_MIN].load();
        o.merkle_chunk = (size_t)opt[CV_OPT_MERKLE_CHUNK].load();
        o.prep_overlap_min = (size_t)opt[CV_OPT_PREP_OVERLAP_MIN].load();
        o.timeline = (int)opt[CV_OPT_TIMELINE].load();
        o.pipe_split = (size_t)opt[CV_OPT_PIPE_SPLIT].load();
        o.pipe_overlap_first = (int)opt[CV_OPT_PIPE_OVERLAP_FIRST].load();
        o.mid_pieces = (size_t)opt[CV_OPT_MID_PIECES].load();
        o.pipe_slots = (size_t)opt[CV_OPT_PIPE_SLOTS].load();
        o.txs_merkle_stream = (int)opt[CV_OPT_TXS_MERKLE_STREAM].load();
        return o;
    }
};

static void span_slice(size_t i0, size_t i1, const uint64_t *off, const uint32_t *len, uint64_t *out);

extern "C" {

const char *cv_version(void) { return "cordaverify-mi355x 0.3 (gfx950)"; }

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

// max(off[i] + len[i]) over n records (0 for n = 0): the arena bytes a batch reaches (the shims' bounds
// check); slices of 2^20 records on up to 8 threads.
uint64_t cv_msg_extent(size_t n, const uint64_t *off, const uint32_t *len) {
    if (!n || !off || !len) return 0;
    // slices of 2^18 records through span_slice (the AVX2 min / max where the CPU has it; a wrapping record
    // saturates to UINT64_MAX), on up to 8 threads
    constexpr size_t kSlice = 1u << 18;
    const size_t ns = (n + kSlice - 1) / kSlice;
    std::vector<uint64_t> part(ns, 0);
    auto scan = [&](size_t k) {
        uint64_t r[3];
        span_slice(k * kSlice, std::min(n, (k + 1) * kSlice), off, len, r);
        part[k] = r[1];
    };
    const size_t nt = std::min<size_t>((ns + 3) / 4, 8);
    if (nt <= 1) {
        for (size_t k = 0; k < ns; k++) scan(k);
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

int cv_set_option(cv_ctx *ctx, int option, int64_t value) {
    if (!ctx || option <= 0 || option >= CV_OPT_COUNT) return CV_E_ARGS;
    if (value < kOpt[option].lo || value > kOpt[option].hi) return CV_E_ARGS;
    ctx->opt[option].store(value);
    return CV_OK;
}

int cv_get_option(cv_ctx *ctx, int option, int64_t *value) {
    if (!ctx || !value || option <= 0 || option >= CV_OPT_COUNT) return CV_E_ARGS;
    *value = ctx->opt[option].load();
    return CV_OK;
}

int cv_diag_stats(cv_ctx *ctx, int which, double *out, size_t nout, int reset) {
    if (!ctx || (nout && !out)) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->st_mu);
    Stats &s = ctx->stats;
    double v[kTlVals + 1] = {};
    size_t nv = 0;
    if (which == CV_STATS_PIPE) {
        for (int k = 0; k < 5; k++) v[k] = s.pipe[k];
        v[5] = (double)s.pipe_calls;
        v[6] = (double)s.pipe_chunks;
        v[7] = (double)s.pipe_direct;
        nv = 8;
    } else if (which == CV_STATS_SMALL) {
        for (int k = 0; k < 5; k++) v[k] = s.small[k];
        v[5] = (double)s.small_calls;
        nv = 6;
    } else if (which == CV_STATS_ROUTE) {
        const uint64_t r[8] = {s.calls, s.routed_whole, s.split_calls, s.shards, s.keyed_calls, s.keyed_chunks,
                               s.merkle_calls, s.merkle_chunks};
        for (int k = 0; k < 8; k++) v[k] = (double)r[k];
        nv = 8;
    } else if (which == CV_STATS_TIMELINE) {
        for (int k = 0; k <= kTlVals; k++) v[k] = s.tl[k];
        nv = kTlVals + 1;
    } else {
        return CV_E_ARGS;
    }
    for (size_t k = 0; k < nout && k < nv; k++) out[k] = v[k];
    if (reset) {
        if (which == CV_STATS_PIPE) {
            std::fill(s.pipe, s.pipe + 5, 0.0);
            s.pipe_calls = s.pipe_chunks = s.pipe_direct = 0;
        } else if (which == CV_STATS_SMALL) {
            std::fill(s.small, s.small + 5, 0.0);
            s.small_calls = 0;
        } else if (which == CV_STATS_TIMELINE) {
            std::fill(s.tl, s.tl + kTlVals + 1, 0.0);
        } else {
            s.calls = s.routed_whole = s.split_calls = s.shards = s.keyed_calls = s.keyed_chunks = s.merkle_calls =
                s.merkle_chunks = 0;
        }
    }
    return (int)nv;
}

int cv_open(uint32_t device_mask, cv_ctx **out) { return cv_open_ex(device_mask, 1, out); }

// slots_per_device > 1: each GPU of the mask appears that many times in THIS context — independent Device slots
// (own lock, worker, streams, buffers, workspace, key pool) on one GPU — so the multi-device host path
// (routing, shards, per-device dedupe and key pools) runs and is tested on a one-GPU box.
int cv_open_ex(uint32_t device_mask, int slots_per_device, cv_ctx **out) {
    if (!out || slots_per_device < 1 || slots_per_device > 16) return CV_E_ARGS;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return CV_E_NO_DEVICE;
    cv_ctx *ctx = new (std::nothrow) cv_ctx();
    if (!ctx) return CV_E_OOM;
    const int virt = slots_per_device;
    for (int d = 0; d < count && d < 32; d++) {
        if (device_mask && !(device_mask & (1u << d))) continue;
        for (int v = 0; v < virt; v++) {
            ctx->devs.emplace_back(new Device());
            Device &dd = *ctx->devs.back();
            dd.ordinal = d;
            // The host pipeline's concurrently busy streams — slot 0 (the device stream), slot 1, the copy
            // stream and the result-copy stream — are created back to back here, before any helper stream,
            // so the runtime spreads them over distinct hardware queues (GPU_MAX_HW_QUEUES = 4 by default).
            // Created lazily, after the device API's split helpers or a caller's own streams, the copy
            // stream could share a queue with a compute stream and its copies wait behind that stream's
            // kernels (C5 host path 86-90 -> 75 ms, profiles/r03p_c5host_eager_streams_ab.log).
            // The copy and result-copy streams are created at the highest stream priority: the runtime keeps a
            // separate hardware-queue pool per priority, so they get queues of their own whatever the
            // process created before (with 4 normal-priority queues already shared by a caller's streams, the
            // synchronous C2 call slowed 10.4 -> 11.8 ms, gpurun_out/r05k).
            hipStream_t s1 = nullptr;
            int prio_lo = 0, prio_hi = 0;
            if (hipSetDevice(d) != hipSuccess || hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess ||
                hipStreamCreateWithFlags(&dd.stream, hipStreamNonBlocking) != hipSuccess ||
                slot_stream(dd, 1, &s1) != hipSuccess ||
                hipStreamCreateWithPriority(&dd.copy, hipStreamNonBlocking, prio_hi) != hipSuccess ||
                hipStreamCreateWithPriority(&dd.outs, hipStreamNonBlocking, prio_hi) != hipSuccess) {
                cv_close(ctx);
                return CV_E_HIP;
            }
            // Per-device basepoint rows (16.8 MB, built once per process): eager, so the first
            // verify is not charged for them and no later call synchronises to build them.
            if (v == 0 && cvk_prepare(dd.stream) != hipSuccess) {
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
    for (auto &dp : ctx->devs) {
        Device &d = *dp;
        d.worker.reset();   // joins the worker (its queue is empty: every call returned before close)
        (void)hipSetDevice(d.ordinal);
        (void)hipDeviceSynchronize();
        for (DevBuf *b : {&d.pk, &d.sig, &d.arena, &d.off, &d.len, &d.bitmap, &d.status, &d.seed, &d.tx_begin,
                          &d.digest, &d.mdigest, &d.ids, &d.pmt, &d.kc.ktab, &d.kc.kok, &d.kc.keys, &d.kc.slots,
                          &d.kc.slot_of_key, &d.kc.scratch})
            b->release();
        d.pin_out.release();
        d.zc_in.release();
        d.zc_out.release();
        for (int k = 0; k < kSlots; k++) {
            Slot &sl = d.slot[k];
            for (DevBuf *b : {&sl.ws_hs, &sl.ws_tab, &sl.ws_R, &sl.ws_ok, &sl.ws_dig, &sl.mdig, &sl.packed, &sl.head})
                b->release();
            sl.pin_in.release();
            sl.pin_head.release();
            for (hipEvent_t v : {sl.ev, sl.split.start, sl.split.done2})
                if (v) (void)hipEventDestroy(v);
            if (sl.split.s2) (void)hipStreamDestroy(sl.split.s2);
            if (k > 0 && sl.stream) (void)hipStreamDestroy(sl.stream);
        }
        for (PipeOut &o : d.out) {
            o.dout.release();
            o.hout.release();
            o.kdev.release();
            o.kstage.release();
            o.kidx.release();
            o.tstage.release();
            for (hipEvent_t v : o.slot_done)
                if (v) (void)hipEventDestroy(v);
            if (o.copied) (void)hipEventDestroy(o.copied);
            for (hipEvent_t v : o.tl)
                if (v) (void)hipEventDestroy(v);
            o.tl.clear();
        }
        if (d.outs) (void)hipStreamDestroy(d.outs);
        for (int q = 0; q < kRing; q++) {
            d.inblk[q].release();
            for (hipEvent_t v : {d.in_ready[q], d.in_free[q]})
                if (v) (void)hipEventDestroy(v);
        }
        for (int k = 0; k < kStage; k++) {
            d.instage[k].release();
            if (d.stage_ev[k]) (void)hipEventDestroy(d.stage_ev[k]);
        }
        for (hipEvent_t v : d.mev) (void)hipEventDestroy(v);
        d.mev.clear();
        if (d.copy) (void)hipStreamDestroy(d.copy);
        if (d.mstream) (void)hipStreamDestroy(d.mstream);
        d.kc.pin.release();
        for (hipEvent_t v : {d.kc.ev, d.kc.pin_ev, d.kc.wev})
            if (v) (void)hipEventDestroy(v);
        if (d.stream) (void)hipStreamDestroy(d.stream);
        d.pool.reset();
    }
    delete ctx;
}

int cv_device_count(const cv_ctx *ctx) { return ctx ? (int)ctx->devs.size() : 0; }

int cv_host_alloc(cv_ctx *ctx, size_t bytes, void **out) {
    if (!ctx || !out || bytes == 0) return CV_E_ARGS;
    *out = nullptr;
    CV_TRY(hipSetDevice(ctx->devs[0]->ordinal));
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
    for (auto &d : ctx->devs)
        if (d->ordinal == device) return d.get();
    return nullptr;
}

}  // extern "C"

// ---------------------------------------------------------------- routing (dispatch)
// Runs fn(device, b, e, packing threads) over shards of [0, n) and returns the first error.  The shard
// plan ("Routing and threading"):
//   - one device, or n <= shard_min: the whole batch on ONE device — the least loaded (shards in progress
//     or queued on it), ties broken by a rotating start, so concurrent notary batches land on different
//     GPUs instead of each being cut eight ways (a shard below the tri-chain size costs the kernel
//     chain's floor, ~0.22 ms, whatever its size);
//   - n >= spread_min: contiguous shards over ALL devices (a throughput batch);
//   - between: over the devices idle at submission, at most ceil(n / shard_min) of them, at least one
//     (the least loaded) — a lone caller's mid-size batch spreads, a loaded node's does not.
// Shard starts are multiples of `align` (64 for verify: whole bitmap words).  The caller's thread runs
// the first shard; the others go to their devices' workers.  A shard runs under its device's lock;
// nothing holds a lock while waiting for another, so concurrent calls cannot deadlock.
template <class F>
static int dispatch(cv_ctx *ctx, const Opts &o, size_t n, size_t align, F fn) {
    const size_t ndev = ctx->devs.size();
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int threads = (int)std::max<size_t>(1, std::min<size_t>((size_t)o.threads, std::max<size_t>(1, hw / ndev)));
    std::vector<size_t> pick;
    const uint32_t start = ctx->rr.fetch_add(1);
    if (ndev == 1) {
        pick.push_back(0);
    } else if (n >= o.spread_min) {
        for (size_t k = 0; k < ndev; k++) pick.push_back(k);
    } else {
        const size_t kmax = n <= o.shard_min ? 1 : (n + o.shard_min - 1) / o.shard_min;
        for (size_t j = 0; j < ndev && pick.size() < kmax; j++) {
            const size_t k = (start + j) % ndev;
            if (ctx->devs[k]->load.load() == 0) pick.push_back(k);
        }
        if (pick.empty()) {
            size_t best = start % ndev;
            for (size_t j = 0; j < ndev; j++) {
                const size_t k = (start + j) % ndev;
                if (ctx->devs[k]->load.load() < ctx->devs[best]->load.load()) best = k;
            }
            pick.push_back(best);
        }
    }
    const size_t ns = pick.size();
    size_t per = (n + ns - 1) / ns;
    per = (per + align - 1) / align * align;
    struct ShardPart {
        size_t dev, b, e;
    };
    std::vector<ShardPart> parts;
    for (size_t j = 0; j < ns; j++) {
        const size_t b = std::min(n, j * per), e = std::min(n, b + per);
        if (b < e || j == 0) parts.push_back({pick[j], b, e});
    }
    {
        std::lock_guard<std::mutex> g(ctx->st_mu);
        ctx->stats.calls++;
        ctx->stats.shards += parts.size();
        if (parts.size() == 1) ctx->stats.routed_whole++;
        else ctx->stats.split_calls++;
    }
    for (const ShardPart &p : parts) ctx->devs[p.dev]->load.fetch_add(1);
    std::vector<int> rc(parts.size(), CV_OK);
    auto run = [&](size_t j) {
        Device &d = *ctx->devs[parts[j].dev];
        {
            std::lock_guard<std::mutex> g(d.mu);
            rc[j] = fn(d, parts[j].b, parts[j].e, threads);
        }
        d.load.fetch_sub(1);
    };
    if (parts.size() == 1) {
        run(0);
        return rc[0];
    }
    std::mutex m;
    std::condition_variable cv;
    size_t left = parts.size() - 1;
    for (size_t j = 1; j < parts.size(); j++)
        ctx->devs[parts[j].dev]->post([&, j] {
            run(j);
            std::lock_guard<std::mutex> g(m);
            if (--left == 0) cv.notify_one();
        });
    run(0);
    {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return left == 0; });
    }
    for (int r : rc)
        if (r != CV_OK) return r;
    return CV_OK;
}

// ---------------------------------------------------------------- host staging
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

// The byte range [lo, hi) of records [b, e) in an arena (min offset, max end) and their total bytes; the
// scan runs in slices of 64K records over the pool.
struct Span {
    uint64_t lo = UINT64_MAX, hi = 0, bytes = 0;
};
// One slice of arena_span.  The unsigned 64-bit min / max vectorise only with AVX2 (the x86-64 baseline has
// no 64-bit compare): the AVX2 instance runs where the CPU has it (65,536 records: 150 -> 48 us on one core
// of this build host).  Dispatched by a cached cpuid test rather than target_clones, whose load-time resolver
// runs before ThreadSanitizer's runtime is up (tests/sanitize).
template <int> static inline void span_slice_impl(size_t i0, size_t i1, const uint64_t *off, const uint32_t *len,
                                                  uint64_t *out) {
    uint64_t lo = UINT64_MAX, hi = 0, bytes = 0;
    for (size_t i = i0; i < i1; i++) {
        uint64_t end = off[i] + len[i];
        end |= -(uint64_t)(end < off[i]);   // a record whose end wraps saturates: never "in bounds"
        lo = std::min<uint64_t>(lo, off[i]);
        hi = std::max<uint64_t>(hi, end);
        bytes += len[i];
    }
    out[0] = lo;
    out[1] = hi;
    out[2] = bytes;
}
__attribute__((target("avx2"))) static void span_slice_avx2(size_t i0, size_t i1, const uint64_t *off,
                                                            const uint32_t *len, uint64_t *out) {
    span_slice_impl<1>(i0, i1, off, len, out);
}
static void span_slice(size_t i0, size_t i1, const uint64_t *off, const uint32_t *len, uint64_t *out) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2)
        span_slice_avx2(i0, i1, off, len, out);
    else
        span_slice_impl<0>(i0, i1, off, len, out);
}
static Span arena_span(size_t b, size_t e, const uint64_t *off, const uint32_t *len, WorkerPool *pool) {
    // with a pool: slices of 8,192 records (the pipeline's sub-chunks: their scans precede their packing on
    // the call's critical path); without, one thread (AVX2)
    const size_t kSlice = pool ? 8192 : 65536;
    const size_t nslices = (e - b + kSlice - 1) / kSlice;
    std::vector<Span> part(std::max<size_t>(nslices, 1));
    auto scan = [&](size_t k) {
        uint64_t r[3];
        span_slice(b + k * kSlice, std::min(e, b + (k + 1) * kSlice), off, len, r);
        part[k].lo = r[0];
        part[k].hi = r[1];
        part[k].bytes = r[2];
    };
    if (pool && nslices > 1)
        pool->run(nslices, scan);
    else
        for (size_t k = 0; k < nslices; k++) scan(k);
    Span s;
    for (const Span &r : part) {
        s.lo = std::min(s.lo, r.lo);
        s.hi = std::max(s.hi, r.hi);
        s.bytes += r.bytes;
    }
    if (s.hi < s.lo) s.lo = s.hi = 0;
    return s;
}

// Staging layout of signature records [b, e): pk | kidx | sig | off | len | arena, 16-B aligned parts (pk
// absent in keyed staging, kidx present only there).  The arena part is the byte range [lo, hi) the records'
// messages span, with lo rounded down to 16 so the device arena pointer keeps every message's alignment;
// the kernels get arena_dev - lo and the caller's offsets unchanged.  When the messages are scattered (the
// range is more than twice their bytes + 1 MB), they are gathered back to back instead and the offsets
// rewritten ("compact").
struct Stage {
    size_t n = 0, o_pk = 0, o_kidx = 0, o_sig = 0, o_off = 0, o_len = 0, o_ar = 0, total = 0;
    uint64_t lo = 0, hi = 0;
    uint64_t extent = 0;   // max(off + len) over the records, whatever the layout (UINT64_MAX: an end wrapped)
    bool compact = false, keyed = false;
};
static Stage stage_plan(size_t b, size_t e, const uint64_t *off, const uint32_t *len, WorkerPool *pool = nullptr,
                        bool keyed = false) {
    Stage st;
    st.n = e - b;
    st.keyed = keyed;
    const Span sp = arena_span(b, e, off, len, pool);
    const uint64_t lo = sp.lo & ~(uint64_t)15;
    st.compact = sp.hi - lo > 2 * sp.bytes + (1u << 20);
    st.lo = st.compact ? 0 : lo;
    st.hi = st.compact ? sp.bytes : sp.hi;
    st.extent = sp.hi;
    const size_t n = st.n;
    st.o_pk = 0;
    st.o_kidx = keyed ? 0 : al16(n * 32);
    st.o_sig = st.o_kidx + (keyed ? al16(n * 4) : 0);
    st.o_off = st.o_sig + al16(n * 64);
    st.o_len = st.o_off + al16(n * 8);
    st.o_ar = st.o_len + al16(n * 4);
    st.total = st.o_ar + al16(st.hi - st.lo + 16);
    return st;
}
// The records of a stage end inside the caller's arena of arena_bytes (UINT64_MAX: no bound given) and no
// record's off + len wraps.  Checked on the true extent, not on [lo, hi): a compacted stage's hi is the SUM of
// its message lengths, which says nothing about where the scattered records lie.
static bool stage_in_bounds(const Stage &st, uint64_t arena_bytes) {
    return st.extent != UINT64_MAX && st.extent <= arena_bytes;
}
// Packs records [b, e) into h by the plan (keys / key indices + signatures first: `first_part` runs after
// them, so their DMA can start while the rest is packed).
static void stage_pack_tail(const Stage &st, uint8_t *h, size_t b, const uint8_t *arena, const uint64_t *off,
                            const uint32_t *len, WorkerPool *pool);
template <class F>
static void stage_pack(const Stage &st, uint8_t *h, size_t b, const uint8_t *pk, const uint32_t *kidx,
                       const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                       WorkerPool *pool, F first_part) {
    const size_t n = st.n;
    if (st.keyed)
        par_copy({{h + st.o_kidx, kidx + b, n * 4}, {h + st.o_sig, sig + b * 64, n * 64}}, pool);
    else
        par_copy({{h + st.o_pk, pk + b * 32, n * 32}, {h + st.o_sig, sig + b * 64, n * 64}}, pool);
    first_part();
    stage_pack_tail(st, h, b, arena, off, len, pool);
}
// The offsets, lengths and message bytes of a stage (its parts from o_off on).
static void stage_pack_tail(const Stage &st, uint8_t *h, size_t b, const uint8_t *arena, const uint64_t *off,
                            const uint32_t *len, WorkerPool *pool) {
    const size_t n = st.n;
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
static bool stage_direct(const Stage &st, size_t b, const uint8_t *pk, const uint32_t *kidx, const uint8_t *sig,
                         const uint8_t *arena, const uint64_t *off, const uint32_t *len) {
    if (st.compact) return false;
    const size_t n = st.n;
    return (st.keyed ? host_pinned(kidx + b, n * 4) : host_pinned(pk + b * 32, n * 32)) &&
           host_pinned(sig + b * 64, n * 64) && host_pinned(off + b, n * 8) && host_pinned(len + b, n * 4) &&
           (st.hi == st.lo || host_pinned(arena + st.lo, st.hi - st.lo));
}
// The stage's DMAs straight from the caller's pinned arrays into the device block dv (the layout of
// stage_pack).  The 16 bytes after the arena part keep whatever the block held: the kernels read a
// message only through dword windows clamped to its last byte and mask the bytes past it, so those
// bytes never reach a verdict — and a fill there would be a blit KERNEL on the copy queue, which waits
// for a free CU slot behind the running verify waves (it held the C2 copy stream for 2.5 ms,
// profiles/r03d_timeline_pinned.txt).
static hipError_t stage_dma_direct(const Stage &st, uint8_t *dv, size_t b, const uint8_t *pk, const uint32_t *kidx,
                                   const uint8_t *sig, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                                   hipStream_t s) {
    const size_t n = st.n;
    hipError_t e = st.keyed ? hipMemcpyAsync(dv + st.o_kidx, kidx + b, n * 4, hipMemcpyHostToDevice, s)
                            : hipMemcpyAsync(dv + st.o_pk, pk + b * 32, n * 32, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(dv + st.o_sig, sig + b * 64, n * 64, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(dv + st.o_off, off + b, n * 8, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(dv + st.o_len, len + b, n * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && st.hi > st.lo)
        e = hipMemcpyAsync(dv + st.o_ar, arena + st.lo, st.hi - st.lo, hipMemcpyHostToDevice, s);
    return e;
}

// Staging layout of Merkle transactions [t0, t1) with leaves [l0, l1): off | len | tx_begin slice | arena.
// The arena part is the leaves' byte range (or the leaves gathered back to back when scattered, as Stage).
struct MStage {
    size_t t0 = 0, t1 = 0, l0 = 0, l1 = 0, o_off = 0, o_len = 0, o_txb = 0, o_ar = 0, total = 0;
    uint64_t lo = 0, hi = 0;
    uint64_t extent = 0;   // as Stage::extent
    bool compact = false;
};
static MStage mstage_plan(size_t t0, size_t t1, const uint32_t *txb, const uint64_t *off, const uint32_t *len,
                          WorkerPool *pool) {
    MStage st;
    st.t0 = t0;
    st.t1 = t1;
    st.l0 = txb[t0];
    st.l1 = txb[t1];
    const size_t nl = st.l1 - st.l0, nt = t1 - t0;
    const Span sp = nl ? arena_span(st.l0, st.l1, off, len, pool) : Span{0, 0, 0};
    const uint64_t lo = sp.lo & ~(uint64_t)15;
    st.compact = nl && sp.hi - lo > 2 * sp.bytes + (1u << 20);
    st.lo = st.compact ? 0 : (nl ? lo : 0);
    st.hi = st.compact ? sp.bytes : (nl ? sp.hi : 0);
    st.extent = nl ? sp.hi : 0;
    st.o_off = 0;
    st.o_len = al16(nl * 8);
    st.o_txb = st.o_len + al16(nl * 4);
    st.o_ar = st.o_txb + al16((nt + 1) * 4);
    st.total = st.o_ar + al16(st.hi - st.lo + 16);
    return st;
}
static void mstage_pack(const MStage &st, uint8_t *h, const uint32_t *txb, const uint8_t *arena, const uint64_t *off,
                        const uint32_t *len, WorkerPool *pool) {
    const size_t nl = st.l1 - st.l0, nt = st.t1 - st.t0;
    uint64_t *hoff = reinterpret_cast<uint64_t *>(h + st.o_off);
    uint8_t *har = h + st.o_ar;
    if (st.compact) {
        par_copy({{h + st.o_len, len + st.l0, nl * 4}, {h + st.o_txb, txb + st.t0, (nt + 1) * 4}}, nullptr);
        uint64_t pos = 0;
        for (size_t i = 0; i < nl; i++) {
            hoff[i] = pos;
            if (len[st.l0 + i]) std::memcpy(har + pos, arena + off[st.l0 + i], len[st.l0 + i]);
            pos += len[st.l0 + i];
        }
    } else {
        par_copy({{h + st.o_off, off + st.l0, nl * 8}, {h + st.o_len, len + st.l0, nl * 4},
                  {h + st.o_txb, txb + st.t0, (nt + 1) * 4},
                  {har, st.hi > st.lo ? arena + st.lo : nullptr, (size_t)(st.hi - st.lo)}},
                 pool);
    }
    std::memset(har + (st.hi - st.lo), 0, 16);
}
static bool mstage_direct(const MStage &st, const uint32_t *txb, const uint8_t *arena, const uint64_t *off,
                          const uint32_t *len) {
    if (st.compact) return false;
    const size_t nl = st.l1 - st.l0, nt = st.t1 - st.t0;
    return (nl == 0 || (host_pinned(off + st.l0, nl * 8) && host_pinned(len + st.l0, nl * 4))) &&
           host_pinned(txb + st.t0, (nt + 1) * 4) && (st.hi == st.lo || host_pinned(arena + st.lo, st.hi - st.lo));
}
static hipError_t mstage_dma_direct(const MStage &st, uint8_t *dv, const uint32_t *txb, const uint8_t *arena,
                                    const uint64_t *off, const uint32_t *len, hipStream_t s) {
    const size_t nl = st.l1 - st.l0, nt = st.t1 - st.t0;
    hipError_t e = hipSuccess;
    if (nl) e = hipMemcpyAsync(dv + st.o_off, off + st.l0, nl * 8, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && nl) e = hipMemcpyAsync(dv + st.o_len, len + st.l0, nl * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(dv + st.o_txb, txb + st.t0, (nt + 1) * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && st.hi > st.lo)
        e = hipMemcpyAsync(dv + st.o_ar, arena + st.lo, st.hi - st.lo, hipMemcpyHostToDevice, s);
    return e;
}

// ---------------------------------------------------------------- key dedupe
// Host-side key dedupe of the plain entry points: keys = the distinct key bytes in first-seen order,
// key_index[i] = its index.  Returns false when the batch does not repeat keys enough for the keyed path to
// pay (fewer than eight signatures per distinct key: a key's 66 KB of tables cost about 7 plain verifies).
//   - n > 4,096: a gate first samples s = 4 sqrt(n) signatures (512 .. 4,096) at pseudo-random positions (a fixed
//     sequence, so a batch always gets the same decision) and counts repeated keys among them; a batch of c
//     distinct keys shows about s^2 / 2c repeats in a sample of s, so fewer than 4 s^2 / 2n repeats (an
//     estimated ratio below four signatures per key) is taken as distinct-keyed without touching the rest.  A
//     performance guess only: both paths give the same verdicts.
//   - the dedupe proper runs in slices on the pool, each with its own growing open-addressing table (a
//     1,024-key pool stays in cache), giving up once any slice has seen more than n / 8 distinct keys;
//     the slices' key lists are then merged in slice order (first-seen order overall) and the slices'
//     local indices remapped.
// Flat tables on the seeded hash of all 32 key bytes (key_hash32), no per-key allocation.
struct FlatKeys {
    std::vector<uint32_t> first, id;   // bucket -> representative record, distinct-key index (UINT32_MAX = empty)
    size_t mask = 0, count = 0;
    explicit FlatKeys(size_t cap0 = 1024) { reset(cap0); }
    void reset(size_t cap) {
        size_t c = 64;
        while (c < cap) c <<= 1;
        first.assign(c, UINT32_MAX);
        id.assign(c, 0);
        mask = c - 1;
        count = 0;
    }
    // index of the key pk[32 * i] (inserting it as `fresh` when new); *added = whether it was new
    uint32_t find_or_add(const uint8_t *pk, uint32_t i, uint32_t fresh, bool *added) {
        const uint8_t *k = pk + 32 * (size_t)i;
        size_t bkt = (size_t)key_hash32(k) & mask;
        for (;;) {
            const uint32_t f = first[bkt];
            if (f == UINT32_MAX) {
                if (2 * (count + 1) > mask + 1) {   // grow: keep the load at or below 1/2
                    grow(pk);
                    return find_or_add(pk, i, fresh, added);
                }
                first[bkt] = i;
                id[bkt] = fresh;
                count++;
                *added = true;
                return fresh;
            }
            if (std::memcmp(pk + 32 * (size_t)f, k, 32) == 0) {
                *added = false;
                return id[bkt];
            }
            bkt = (bkt + 1) & mask;
        }
    }

  private:
    void grow(const uint8_t *pk) {
        std::vector<uint32_t> f0 = std::move(first), i0 = std::move(id);
        const size_t c = 2 * (mask + 1);
        first.assign(c, UINT32_MAX);
        id.assign(c, 0);
        mask = c - 1;
        for (size_t b = 0; b < f0.size(); b++) {
            if (f0[b] == UINT32_MAX) continue;
            size_t bkt = (size_t)key_hash32(pk + 32 * (size_t)f0[b]) & mask;
            while (first[bkt] != UINT32_MAX) bkt = (bkt + 1) & mask;
            first[bkt] = f0[b];
            id[bkt] = i0[b];
        }
    }
};

// The sample: s = 4 sqrt(n) records (512 .. 4,096): a batch with eight signatures per key then shows about
// 4 s^2 / n = 64 repeats, a distinct-keyed one about s^2 / (2 n) = 8, against a threshold of 2 s^2 / n = 32 —
// Poisson tails far below 10^-6 either way.  Round 4 sampled 4,096 records at every size above 16,384 and deduped
// every batch up to 16,384 in full: 60-100 us of host time on each distinct-keyed notary batch of 16,384-65,536
// signatures (tools/notary_probe.py host phases), for a decision that only picks the faster path.
// LSD radix sort of values below `bound` (passes of 11 bits up to bound's top bit): the gate's 4,096 sample
// positions, which std::sort took ~300 us to order on this container's host (radix: 60 us for three passes) —
// on every large call's path before its first DMA
static void radix_sort_u32(std::vector<uint32_t> &v, uint64_t bound) {
    std::vector<uint32_t> tmp(v.size());
    for (int sh = 0; sh < 32 && (bound - 1) >> sh; sh += 11) {
        uint32_t cnt[2049] = {};
        for (uint32_t x : v) cnt[((x >> sh) & 2047) + 1]++;
        for (int k = 0; k < 2048; k++) cnt[k + 1] += cnt[k];
        for (uint32_t x : v) tmp[cnt[(x >> sh) & 2047]++] = x;
        v.swap(tmp);
    }
}

static bool dedupe_gate(size_t n, const uint8_t *pk) {
    if (n <= 4096) return true;                    // the estimate needs s << n; a full dedupe of <= 4,096 is cheap
    const uint32_t kS = (uint32_t)std::min<double>(4096.0, std::max(512.0, 4.0 * std::sqrt((double)n)));
    FlatKeys t(4 * kS);                            // load <= 1/4: the table never grows while sampling
    uint64_t x = 0x9E3779B97F4A7C15ull;
    uint32_t rep = 0;
    std::vector<uint32_t> pos(kS);
    for (uint32_t j = 0; j < kS; j++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        pos[j] = (uint32_t)((x >> 32) * (uint64_t)n >> 32);
    }
    radix_sort_u32(pos, n);                        // ascending: duplicate positions adjacent
    constexpr uint32_t kAhead = 16;                // the key reads miss the caches: prefetched 16 samples ahead
    for (uint32_t j = 0; j < std::min(kS, kAhead); j++) __builtin_prefetch(pk + 32 * (size_t)pos[j]);
    uint32_t prev = UINT32_MAX;
    for (uint32_t j = 0; j < kS; j++) {
        if (j + kAhead < kS) __builtin_prefetch(pk + 32 * (size_t)pos[j + kAhead]);
        if (pos[j] == prev) continue;               // the same record twice is not a repeated key
        prev = pos[j];
        bool added;
        t.find_or_add(pk, pos[j], (uint32_t)t.count, &added);
        rep += added ? 0 : 1;
    }
    // keyed worth a full dedupe when s^2 / (2 rep) < n / 4, i.e. rep > 2 s^2 / n
    return (double)rep > 2.0 * (double)kS * (double)kS / (double)n;
}

static bool dedupe_keys(size_t n, const uint8_t *pk, std::vector<uint8_t> &keys, std::vector<uint32_t> &key_index,
                        WorkerPool *pool, bool gate = true) {
    if (n < 64 || n > 0xffffffffull) return false;
    if (gate && !dedupe_gate(n, pk)) return false;
    const size_t limit = n / 8;                      // most distinct keys the keyed path takes
    const int nt = pool ? pool->threads() : 1;
    const size_t nsl = (n >= 65536 && nt > 1) ? (size_t)nt * 2 : 1;
    const size_t per = (n + nsl - 1) / nsl;
    key_index.resize(n);
    std::vector<std::vector<uint32_t>> uniq(nsl);   // per slice: the record of each local key, first-seen order
    std::atomic<bool> over{false};
    auto slice = [&](size_t s) {
        const size_t b = s * per, e = std::min(n, b + per);
        FlatKeys t(1024);
        for (size_t i = b; i < e && !over.load(std::memory_order_relaxed); i++) {
            bool added;
            key_index[i] = t.find_or_add(pk, (uint32_t)i, (uint32_t)uniq[s].size(), &added);
            if (added) {
                uniq[s].push_back((uint32_t)i);
                if (uniq[s].size() > limit) over.store(true);
            }
        }
    };
    if (nsl > 1)
        pool->run(nsl, slice);
    else
        slice(0);
    if (over.load()) return false;
    // merge the slices' key lists in slice order; remap[s][local] = global index
    FlatKeys g(4096);
    std::vector<uint32_t> grec;                      // the representative record of each global key
    std::vector<std::vector<uint32_t>> remap(nsl);
    for (size_t s = 0; s < nsl; s++) {
        remap[s].resize(uniq[s].size());
        for (size_t u = 0; u < uniq[s].size(); u++) {
            bool added;
            remap[s][u] = g.find_or_add(pk, uniq[s][u], (uint32_t)grec.size(), &added);
            if (added) {
                grec.push_back(uniq[s][u]);
                if (grec.size() > limit) return false;
            }
        }
    }
    if (nsl > 1 || !remap[0].empty()) {
        auto fix = [&](size_t s) {
            const size_t b = s * per, e = std::min(n, b + per);
            const std::vector<uint32_t> &r = remap[s];
            for (size_t i = b; i < e; i++) key_index[i] = r[key_index[i]];
        };
        if (nsl > 1)
            pool->run(nsl, fix);
        else
            fix(0);
    }
    keys.resize(32 * grec.size());
    for (size_t u = 0; u < grec.size(); u++) std::memcpy(keys.data() + 32 * u, pk + 32 * (size_t)grec[u], 32);
    return true;
}

// ---------------------------------------------------------------- keyed: key pool
// Waits until nothing queued on the device may still read its key pool (before the pool is emptied or
// reallocated: an asynchronous call's sub-chunks may still be reading the slots being reassigned).
static hipError_t pool_quiesce(Device &d) {
    hipError_t e = hipSuccess;
    for (int k = 0; k < kSlots && e == hipSuccess; k++)
        if (d.slot[k].stream) e = hipStreamSynchronize(d.slot[k].stream);
    if (e == hipSuccess && d.kc.last) e = hipEventSynchronize(d.kc.ev);
    return e;
}

// Makes the keys k (used[k] != 0, or all when used == nullptr) of keys[0..nk) resident in d's key
// pool and fills slot_of_key[k]; keyprep launches on s compute the tables of the new ones (at most
// kKeyprepBatch keys per launch, so the scratch stays bounded) and *prepared says whether any ran.  The
// caller holds the device lock and the pool (pool_begin).  Failure leaves an empty pool (capacity 0, no
// resident keys), never a key mapped to a slot whose tables were not computed or a capacity without its
// buffers.
static int key_resolve(Device &d, uint32_t cap, size_t nk, const uint8_t *keys, const uint8_t *used,
                       std::vector<uint32_t> &slot_of_key, hipStream_t s, bool *prepared) {
    KeyCache &kc = d.kc;
    *prepared = false;
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
        hipError_t e = pool_quiesce(d);
        if (e != hipSuccess) return fail(e);
        kc.map.clear();
        kc.cap = 0;
        kc.ktab.release();
        kc.kok.release();
        if ((e = kc.ktab.ensure(need * kKtabBytes)) != hipSuccess) return fail(e);
        if ((e = kc.kok.ensure(need)) != hipSuccess) return fail(e);
        kc.cap = (uint32_t)need;
    }
    // epoch reset: every key of this call gets a fresh slot, after the queued readers of the old ones
    if (kc.map.size() + nused > kc.cap) {
        const hipError_t e = pool_quiesce(d);
        if (e != hipSuccess) return fail(e);
        kc.map.clear();
        kc.resets++;
    }
    std::vector<uint8_t> miss_keys;
    std::vector<uint32_t> miss_slots;
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
        hipError_t e = hipStreamSynchronize(s);
        if (e == hipSuccess) e = hipEventRecord(kc.wev, s);
        if (e != hipSuccess) return fail(e);
        kc.wlast = s;
        *prepared = true;
    }
    for (auto &kv : fresh) kc.map.emplace(kv.first, kv.second);
    return CV_OK;
}

// ---------------------------------------------------------------- verify (host buffers): small paths
// The caller's record arrays of one host-buffer call.  Keyed calls carry keys[nkeys][32] + key_index[n]
// instead of per-record keys.
struct VerifyIn {
    const uint8_t *pk = nullptr, *sig = nullptr, *arena = nullptr;
    const uint64_t *off = nullptr;
    const uint32_t *len = nullptr;
    const uint8_t *keys = nullptr;       // keyed
    const uint32_t *key_index = nullptr; // keyed
    size_t nkeys = 0;
    const uint8_t *used = nullptr;       // keyed: which of the keys the shard uses (nullptr = all)
    bool copy_kidx = false;              // keyed: key_index is the call's own host vector (copied to pinned memory)
    bool auto_keyed = false;             // dedupe pk per shard and take the keyed path
    uint64_t *bitmap = nullptr;
    uint8_t *status = nullptr;
    // cv_ed25519_verify_batch_ex: the arena's size; every staging scan (which finds the byte range its records
    // reach anyway) rejects a shard or sub-chunk whose records reach past it before anything reads the arena
    uint64_t arena_bytes = UINT64_MAX;
    double t_entry = 0;   // host time the call entered the engine (CV_OPT_TIMELINE's host_pre)
};

// Zero-copy form of the small path for tri-chain batches (the notary batches).  The records are packed into
// fine-grained pinned host memory that the fused prep kernel reads over PCIe, and the kernels store the
// status bytes and one verdict byte per wave (4 bits) into pinned host memory: no DMA in, no copy out.
// Measured on the box, notary 4,096 (profiles/r03j_timeline_notary4096.txt), the DMA path paid 19.8 us of
// H2D + 11.6 us from the DMA's completion to the prep's start + 9.6 us for the verdict copy.
static int verify_shard_small_zc(cv_ctx *ctx, Device &d, const Opts &o, const Stage &st, size_t b, const VerifyIn &in,
                                 WorkerPool *pool, double t_plan, bool gather) {
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
    if (!cvk_tri_zc_ok(&o.plan, (uint32_t)n, sl.ws_cap)) return CV_E_HIP;   // (cannot happen: checked by the caller)
    uint8_t *h = d.zc_in.as<uint8_t>();
    if (gather) CV_TRY(sl.packed.ensure(al16(st.total)));
    const uint8_t *dv = gather ? sl.packed.as<uint8_t>() : d.zc_in.dev_as<uint8_t>();
    t[1] = now_s();
    stage_pack(st, h, b, in.pk, nullptr, in.sig, in.arena, in.off, in.len, pool, [] {});
    uint8_t *nib = d.zc_out.as<uint8_t>();
    std::memset(nib + waves, 0, nnib - waves);   // bytes of waves past the batch: no wave stores them
    t[2] = now_s();
    auto drain = on_exit([s] { (void)hipStreamSynchronize(s); });   // error paths: no kernel outlives the call
    CV_TRY(ws_begin(d, sl, s));
    const hipError_t e = cvk_verify_tri_zc(
        &o.plan, (uint32_t)n, dv + st.o_pk, dv + st.o_sig, dv + st.o_ar - st.lo,
        reinterpret_cast<const uint64_t *>(dv + st.o_off), reinterpret_cast<const uint32_t *>(dv + st.o_len),
        d.zc_out.dev_as<uint8_t>(), in.status ? d.zc_out.dev_as<uint8_t>() + al16(nnib) : nullptr,
        sl.ws_tab.as<uint32_t>(), sl.ws_ok.as<uint8_t>(), sl.ws_dig.as<uint32_t>(), sl.ws_cap, s,
        gather ? d.zc_in.dev : nullptr, gather ? sl.packed.p : nullptr, gather ? al16(st.total) : 0);
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
        in.bitmap[b / 64 + w] = x;
    }
    if (in.status) std::memcpy(in.status + b, nib + al16(nnib), n);
    t[5] = now_s();
    {
        std::lock_guard<std::mutex> g(ctx->st_mu);
        for (int k = 0; k < 5; k++) ctx->stats.small[k] += t[k + 1] - t[k];
        ctx->stats.small_calls++;
    }
    return CV_OK;
}

// One shard [b, e) of a batch on one device, small form (notary-sized batches): the zero-copy tri-chain form
// where it applies, else packed into slot 0's pinned staging (or DMAed in place from pinned arrays), moved
// by one DMA (two above 1 MB: the first overlaps packing the second part) into one device block, verified,
// and the bitmap (+ status) come back by one DMA.  b is a multiple of 64, so the shard's bitmap words are
// whole words of the caller's bitmap.
// Mid-size unpipelined batches (from prep_overlap_min): the keys and signatures — all the point kernels read —
// are staged into their own device block and their DMA issued FIRST, before the range scan of the offsets and
// lengths; the scan, the tail's packing (pageable inputs) and its DMA then run beside that DMA, and the point
// decodes start on the slot's helper stream as soon as it lands (cvk_verify, CvkPrepOverlap).
static int verify_shard_mid(cv_ctx *ctx, Device &d, const Opts &o, size_t b, size_t e, const VerifyIn &in,
                            WorkerPool *pool, double t_plan) {
    const size_t n = e - b;
    const size_t words = (n + 63) / 64;
    const size_t o_bm = 0, o_st = al16(words * 8), total_out = o_st + al16(n);
    const size_t h_sig = al16(n * 32), h_total = h_sig + al16(n * 64);
    // pageable inputs go up in about 1 MB pieces of keys + signatures (at most CV_OPT_MID_PIECES)
    const size_t pieces = pool ? std::max<size_t>(1, std::min<size_t>(o.mid_pieces, h_total >> 20)) : 1;
    double t[6];
    t[0] = t_plan;
    Slot &sl = d.slot[0];
    hipStream_t s = nullptr;
    CV_TRY(slot_stream(d, 0, &s));
    CV_TRY(slot_events(sl));
    CV_TRY(slot_split(d, sl));
    CvkPrepOverlap po;
    po.aux = sl.split.s2;
    po.ready = sl.split.start;
    po.done = sl.split.done2;
    CV_TRY(sl.head.ensure(h_total));
    CV_TRY(d.pin_out.ensure(total_out));
    CV_TRY(d.bitmap.ensure(total_out));
    uint8_t *dh = sl.head.as<uint8_t>();
    hipStream_t aux = po.aux;
    auto drain = on_exit([s, aux] {   // error paths: no DMA or helper-stream kernel outlives the call
        (void)hipStreamSynchronize(s);
        (void)hipStreamSynchronize(aux);
    });
    // ---- head: keys | signatures, in place from pinned arrays or packed on the pool
    const bool head_pinned = n >= o.small_direct_min && host_pinned(in.pk + b * 32, n * 32) &&
                             host_pinned(in.sig + b * 64, n * 64);
    if (head_pinned) {
        CV_TRY(hipMemcpyAsync(dh, in.pk + b * 32, n * 32, hipMemcpyHostToDevice, s));
        CV_TRY(hipMemcpyAsync(dh + h_sig, in.sig + b * 64, n * 64, hipMemcpyHostToDevice, s));
    } else {
        // pageable keys and signatures: packed into pinned staging and DMAed in `pieces` record ranges, each range's
        // two DMAs issued as soon as it is packed, so the DMA runs beside the packing of the next range
        CV_TRY(sl.pin_head.ensure(h_total));
        uint8_t *hh = sl.pin_head.as<uint8_t>();
        for (size_t p = 0; p < pieces; p++) {
            const size_t r0 = n * p / pieces, r1 = n * (p + 1) / pieces;
            par_copy({{hh + r0 * 32, in.pk + (b + r0) * 32, (r1 - r0) * 32},
                      {hh + h_sig + r0 * 64, in.sig + (b + r0) * 64, (r1 - r0) * 64}}, pool);
            CV_TRY(hipMemcpyAsync(dh + r0 * 32, hh + r0 * 32, (r1 - r0) * 32, hipMemcpyHostToDevice, s));
            CV_TRY(hipMemcpyAsync(dh + h_sig + r0 * 64, hh + h_sig + r0 * 64, (r1 - r0) * 64, hipMemcpyHostToDevice, s));
        }
    }
    CV_TRY(hipEventRecord(po.ready, s));
    t[1] = now_s();
    // ---- tail: offsets | lengths | message bytes (the Stage layout from o_off on), behind the head's DMA
    const Stage st = stage_plan(b, e, in.off, in.len, head_pinned ? nullptr : pool);
    if (!stage_in_bounds(st, in.arena_bytes)) return CV_E_ARGS;   // (drain: the head's DMA is waited for)
    CV_TRY(sl.packed.ensure(st.total));
    uint8_t *dv = sl.packed.as<uint8_t>();
    if (n >= o.small_direct_min && stage_direct(st, b, in.pk, nullptr, in.sig, in.arena, in.off, in.len)) {
        CV_TRY(hipMemcpyAsync(dv + st.o_off, in.off + b, n * 8, hipMemcpyHostToDevice, s));
        CV_TRY(hipMemcpyAsync(dv + st.o_len, in.len + b, n * 4, hipMemcpyHostToDevice, s));
        if (st.hi > st.lo)
            CV_TRY(hipMemcpyAsync(dv + st.o_ar, in.arena + st.lo, st.hi - st.lo, hipMemcpyHostToDevice, s));
    } else if (pieces > 1 && !st.compact) {
        // pageable tail: offsets and lengths, then the message bytes in `pieces` ranges, each DMAed once packed
        CV_TRY(sl.pin_in.ensure(st.total));
        uint8_t *h = sl.pin_in.as<uint8_t>();
        par_copy({{h + st.o_off, in.off + b, n * 8}, {h + st.o_len, in.len + b, n * 4}}, pool);
        CV_TRY(hipMemcpyAsync(dv + st.o_off, h + st.o_off, st.o_ar - st.o_off, hipMemcpyHostToDevice, s));
        const size_t span = st.hi - st.lo;
        for (size_t p = 0; p < pieces; p++) {
            const size_t a0 = span * p / pieces, a1 = span * (p + 1) / pieces;
            if (a1 > a0) par_copy({{h + st.o_ar + a0, in.arena + st.lo + a0, a1 - a0}}, pool);
            if (p + 1 == pieces) std::memset(h + st.o_ar + span, 0, 16);
            const size_t len = a1 - a0 + (p + 1 == pieces ? 16 : 0);
            if (len) CV_TRY(hipMemcpyAsync(dv + st.o_ar + a0, h + st.o_ar + a0, len, hipMemcpyHostToDevice, s));
        }
    } else {
        CV_TRY(sl.pin_in.ensure(st.total));
        uint8_t *h = sl.pin_in.as<uint8_t>();
        stage_pack_tail(st, h, b, in.arena, in.off, in.len, pool);
        CV_TRY(hipMemcpyAsync(dv + st.o_off, h + st.o_off, st.total - st.o_off, hipMemcpyHostToDevice, s));
    }
    t[2] = now_s();
    uint8_t *dout = d.bitmap.as<uint8_t>();
    CV_TRY(launch_verify(d, o.plan, sl, (uint32_t)n, dh, dh + h_sig, dv + st.o_ar - st.lo,
                         reinterpret_cast<const uint64_t *>(dv + st.o_off), reinterpret_cast<const uint32_t *>(dv + st.o_len),
                         reinterpret_cast<uint64_t *>(dout + o_bm), in.status ? dout + o_st : nullptr, s, nullptr, true, &po));
    CV_TRY(hipMemcpyAsync(d.pin_out.p, dout, in.status ? o_st + n : words * 8, hipMemcpyDeviceToHost, s));
    t[3] = now_s();
    CV_TRY(hipStreamSynchronize(s));
    drain.armed = false;
    t[4] = now_s();
    std::memcpy(in.bitmap + b / 64, d.pin_out.as<uint8_t>() + o_bm, words * 8);
    if (in.status) std::memcpy(in.status + b, d.pin_out.as<uint8_t>() + o_st, n);
    t[5] = now_s();
    {
        std::lock_guard<std::mutex> g(ctx->st_mu);
        for (int k = 0; k < 5; k++) ctx->stats.small[k] += t[k + 1] - t[k];
        ctx->stats.small_calls++;
    }
    return CV_OK;
}

static int verify_shard_small(cv_ctx *ctx, Device &d, const Opts &o, size_t b, size_t e, const VerifyIn &in,
                              int threads) {
    const size_t n = e - b;
    WorkerPool *pool = n >= 16384 ? &d.workers(threads) : nullptr;
    const double t_plan = now_s();
    if (n >= o.prep_overlap_min && (!o.small_zc || !cvk_tri_zc_ok(&o.plan, (uint32_t)n, (uint32_t)n)))
        return verify_shard_mid(ctx, d, o, b, e, in, pool, t_plan);
    // pinned inputs (DMAed in place, nothing to pack): the range scan on this thread — waking the pool's helpers
    // cost ~20 us, more than the scan of a notary batch (16,384 0.409 -> 0.391 ms p50); pageable inputs: on the
    // pool, whose helpers the packing needs next anyway
    const bool in_place = pool && n >= o.small_direct_min && host_pinned(in.pk + b * 32, n * 32);
    const Stage st = stage_plan(b, e, in.off, in.len, in_place ? nullptr : pool);
    if (!stage_in_bounds(st, in.arena_bytes)) return CV_E_ARGS;
    if (o.small_zc && cvk_tri_zc_ok(&o.plan, (uint32_t)n, (uint32_t)n))
        return verify_shard_small_zc(ctx, d, o, st, b, in, pool, t_plan,
                                     o.small_zc == 2 || (o.small_zc == 3 && n >= 2048));
    const size_t words = (n + 63) / 64;
    const size_t o_bm = 0, o_st = al16(words * 8), total_out = o_st + al16(n);
    double t[6];                 // host phases (cv_diag_stats CV_STATS_SMALL, as the zero-copy form)
    t[0] = t_plan;
    Slot &sl = d.slot[0];
    hipStream_t s = nullptr;
    CV_TRY(slot_stream(d, 0, &s));
    CV_TRY(slot_events(sl));
    CV_TRY(sl.pin_in.ensure(st.total));
    CV_TRY(d.pin_out.ensure(total_out));
    CV_TRY(sl.packed.ensure(st.total));
    CV_TRY(d.bitmap.ensure(total_out));
    uint8_t *h = sl.pin_in.as<uint8_t>();
    uint8_t *dv = sl.packed.as<uint8_t>();
    auto drain = on_exit([s] { (void)hipStreamSynchronize(s); });   // error paths: no DMA outlives the call
    t[1] = now_s();
    // Two-stage staging above 1 MB of keys + signatures: they are packed and their DMA is issued
    // first, so it runs while the offsets, lengths and message bytes are packed (notary 65,536:
    // 1.29-1.34 -> 1.21-1.25 ms p50); below, one DMA (a second DMA's ~6 us would cost more than it hides).
    const bool two_stage = st.o_off >= ((size_t)1 << 20);
    // below small_direct_min signatures one packed DMA beats five direct ones even from pinned arrays
    // (notary 4,096: 0.328 ms p50 packed vs 0.342 direct; 65,536: 1.28 vs 1.10, profiles/r03h_bench.json)
    if (n >= o.small_direct_min && stage_direct(st, b, in.pk, nullptr, in.sig, in.arena, in.off, in.len)) {
        CV_TRY(stage_dma_direct(st, dv, b, in.pk, nullptr, in.sig, in.arena, in.off, in.len, s));
    } else {
        hipError_t e1 = hipSuccess;
        stage_pack(st, h, b, in.pk, nullptr, in.sig, in.arena, in.off, in.len, pool, [&] {
            if (two_stage) e1 = hipMemcpyAsync(dv, h, st.o_off, hipMemcpyHostToDevice, s);
        });
        CV_TRY(e1);
        if (two_stage)
            CV_TRY(hipMemcpyAsync(dv + st.o_off, h + st.o_off, st.total - st.o_off, hipMemcpyHostToDevice, s));
        else
            CV_TRY(hipMemcpyAsync(dv, h, st.total, hipMemcpyHostToDevice, s));
    }
    t[2] = now_s();
    uint8_t *dout = d.bitmap.as<uint8_t>();
    CV_TRY(launch_verify(d, o.plan, sl, (uint32_t)n, dv + st.o_pk, dv + st.o_sig, dv + st.o_ar - st.lo,
                         reinterpret_cast<const uint64_t *>(dv + st.o_off), reinterpret_cast<const uint32_t *>(dv + st.o_len),
                         reinterpret_cast<uint64_t *>(dout + o_bm), in.status ? dout + o_st : nullptr, s, nullptr, true));
    CV_TRY(hipMemcpyAsync(d.pin_out.p, dout, in.status ? o_st + n : words * 8, hipMemcpyDeviceToHost, s));
    t[3] = now_s();
    CV_TRY(hipStreamSynchronize(s));
    drain.armed = false;
    t[4] = now_s();
    std::memcpy(in.bitmap + b / 64, d.pin_out.as<uint8_t>() + o_bm, words * 8);
    if (in.status) std::memcpy(in.status + b, d.pin_out.as<uint8_t>() + o_st, n);
    t[5] = now_s();
    {
        std::lock_guard<std::mutex> g(ctx->st_mu);
        for (int k = 0; k < 5; k++) ctx->stats.small[k] += t[k + 1] - t[k];
        ctx->stats.small_calls++;
    }
    return CV_OK;
}

// ---------------------------------------------------------------- the host pipeline
// The pipeline's sub-chunk boundaries of [b, e): [first, C, C, ..., the last two balanced]; every boundary
// but e is b + a multiple of `align`.  With ramp, the sizes after the first double (first, 2 first, ...)
// until they reach C: each sub-chunk's copy then takes about as long as the kernels of the one before it,
// so the GPU is not left waiting for a big second sub-chunk while a small first one has long finished.
// The sub-chunk of an asynchronous pipelined call of n records: 1 or 2 x CV_OPT_ASYNC_CHUNK, the multiple nearest
// n / 16 (so a call has about 16 or fewer launch groups, each a whole number of async chunks).
static size_t async_sub_chunk(const Opts &o, size_t n) {
    const size_t c = std::max<size_t>(64, o.async_chunk / 64 * 64);
    return c * std::min<size_t>(2, std::max<size_t>(1, (n / 16 + c / 2) / c));
}
static std::vector<size_t> pipe_cuts(size_t b, size_t e, size_t first, size_t C, bool ramp = false, size_t align = 64) {
    std::vector<size_t> cut{b};
    if (e <= b) return cut;
    first = std::max<size_t>(align, first / align * align);
    C = std::max<size_t>(align, C / align * align);
    size_t p = b + std::min(e - b, first);
    cut.push_back(p);
    size_t step = first;
    while (p < e) {
        const size_t rem = e - p;
        step = ramp ? std::min(C, 2 * step) : C;
        const size_t m = rem <= step ? rem : rem < 2 * step ? (rem / 2 + align - 1) / align * align : step;
        p += m;
        cut.push_back(p);
    }
    return cut;
}

// Copies a finished pipelined call's results into the caller's arrays (waits for them first).  Results of
// 1 MB and more are copied by the DMA straight into the caller's memory; smaller ones come back through
// the output's pinned buffer.  The caller holds po.mu.
static int pipe_copy_back(Device &d, PipeOut &po) {
    CV_TRY(hipSetDevice(d.ordinal));
    // host-side join: the call's last launch group on every slot stream, then the result copies on the
    // device's output stream (which carries nothing else, so it neither waits behind the next call's input
    // copies nor holds a compute stream the next call's kernels run on)
    for (int k = 0; k <= kPipeSlots; k++)
        if (po.slot_used[k]) CV_TRY(hipEventSynchronize(po.slot_done[k]));
    const bool timeline = po.tl_n > 0 && po.tl.size() >= (size_t)po.tl_n * 3 + 1;
    const double t_copy = now_s();   // (timeline: the result copies' host-side time, from the join on)
    po.tl_join_s = t_copy;
    constexpr size_t kDirect = 1u << 20;
    size_t hb = 0;
    for (int k = 0; k < po.nseg; k++) {
        const PipeOut::Seg &sg = po.seg[k];
        if (sg.len >= kDirect)
            CV_TRY(hipMemcpyAsync(sg.dst, po.dout.as<uint8_t>() + sg.off, sg.len, hipMemcpyDeviceToHost, d.outs));
        else
            hb = std::max(hb, sg.off + sg.len);
    }
    if (hb) CV_TRY(po.hout.ensure(hb));
    for (int k = 0; k < po.nseg; k++) {
        const PipeOut::Seg &sg = po.seg[k];
        if (sg.len && sg.len < kDirect)
            CV_TRY(hipMemcpyAsync(po.hout.as<uint8_t>() + sg.off, po.dout.as<uint8_t>() + sg.off, sg.len,
                                  hipMemcpyDeviceToHost, d.outs));
    }
    // joined by an event after this call's copies, not by hipStreamSynchronize(d.outs): once calls had been
    // joined one at a time (each draining the device), the stream synchronise of this stream kept costing ~1.2
    // ms per call of two later calls in flight (keyed host C2 8.5-8.7 -> 7.3 ms, DESIGN "Host runtime effects")
    if (!po.copied) CV_TRY(hipEventCreateWithFlags(&po.copied, hipEventDisableTiming));
    CV_TRY(hipEventRecord(po.copied, d.outs));
    CV_TRY(hipEventSynchronize(po.copied));
    if (timeline) {
        const double copy_ms = (now_s() - t_copy) * 1e3;
        auto at = [&](size_t k) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, po.tl[0], po.tl[k]);
            return (double)ms;
        };
        const int J = po.tl_n;
        // the union length of a set of [start, end) intervals
        auto union_len = [](std::vector<std::pair<double, double>> iv) {
            if (iv.empty()) return 0.0;
            std::sort(iv.begin(), iv.end());
            double busy = 0, cur0 = iv[0].first, cur1 = iv[0].second;
            for (size_t j = 1; j < iv.size(); j++) {
                if (iv[j].first > cur1) {
                    busy += cur1 - cur0;
                    cur0 = iv[j].first;
                    cur1 = iv[j].second;
                } else {
                    cur1 = std::max(cur1, iv[j].second);
                }
            }
            return busy + cur1 - cur0;
        };
        std::vector<std::pair<double, double>> all, mk, vf;
        double ramp = 1e30, span = 0, dma_end = 0, mdma_end = 0;
        for (int j = 0; j < J; j++) {
            const std::pair<double, double> w{at(2 + 3 * (size_t)j), at(3 + 3 * (size_t)j)};
            const double de = at(1 + 3 * (size_t)j);
            const bool merkle = (size_t)j < po.tl_merkle.size() && po.tl_merkle[j];
            all.push_back(w);
            (merkle ? mk : vf).push_back(w);
            ramp = std::min(ramp, w.first);
            span = std::max(span, w.second);
            dma_end = std::max(dma_end, de);
            if (merkle) mdma_end = std::max(mdma_end, de);
        }
        const double busy = union_len(all);
        const double v[kTlVals] = {ramp, dma_end, span, busy, span - ramp - busy, span - dma_end, copy_ms,
                                   (double)po.tl_first, union_len(mk), union_len(vf), mdma_end, (double)J,
                                   po.tl_pre_ms, 0.0};
        for (int k = 0; k < kTlVals; k++) po.tl_sum[k] = v[k];
        po.tl_ready = true;
        po.tl_n = 0;
    }
    for (int k = 0; k < po.nseg; k++) {
        const PipeOut::Seg &sg = po.seg[k];
        if (sg.len && sg.len < kDirect) std::memcpy(sg.dst, po.hout.as<uint8_t>() + sg.off, sg.len);
    }
    return CV_OK;
}

// Finishes the call pending on po (if any) and returns its result; a failure is also recorded under the call's
// gen, so whoever finishes it — its own cv_wait, a later call reusing the output, an error path's drain — the
// call's waiter gets the error.  The caller holds po.mu.
static int pipe_finish(Device &d, PipeOut &po) {
    if (!po.pending) return CV_OK;
    po.pending = false;
    const bool ticketed = po.ticketed;
    po.ticketed = false;
    const int rc = pipe_copy_back(d, po);
    if (rc != CV_OK) {
        if (ticketed) {
            po.failed.emplace_back(po.gen, rc);
            if (po.failed.size() > kFailKeep) po.failed.pop_front();
        }
    }
    return rc;
}

// The device's next output: the older call still holding it is finished first (its results land in its
// caller's arrays; an error is kept for that call's cv_wait, not handed to the new caller).  Returns it locked.
static PipeOut &pipe_out(Device &d, int *index, std::unique_lock<std::mutex> &lk) {
    PipeOut &po = d.out[d.out_next];
    *index = d.out_next;
    d.out_next = (d.out_next + 1) % kOuts;
    lk = std::unique_lock<std::mutex>(po.mu);
    (void)pipe_finish(d, po);
    return po;
}

// The common frame of a pipelined call on one device: the two compute streams, the ring's events and the
// output's completion events; and the error-path drain.
struct PipeFrame {
    Device &d;
    PipeOut &po;
    int ns = 2;                       // compute slots this call uses (CV_OPT_PIPE_SLOTS for verify calls; set before init)
    hipStream_t ss[kPipeSlots] = {};
    bool used[kPipeSlots + 1] = {};   // + the copy stream (Merkle kernels), always at index kPipeSlots
    double t[5] = {};   // plan, pack, wait, enqueue (seconds)
    uint64_t chunks = 0, direct = 0;
    bool tl = false;    // CV_OPT_TIMELINE: record po.tl's events (synchronous verify calls)
    hipError_t tl_record(size_t k, hipStream_t s) {
        hipEvent_t e = po.tl_ev(k);
        return e ? hipEventRecord(e, s) : hipErrorOutOfMemory;
    }
    int init() {
        for (int k = 0; k < ns; k++) {
            CV_TRY(slot_stream(d, k, &ss[k]));
            CV_TRY(slot_events(d.slot[k]));
        }
        for (int k = 0; k <= kPipeSlots; k++)
            if (!po.slot_done[k]) CV_TRY(hipEventCreateWithFlags(&po.slot_done[k], hipEventDisableTiming));
        for (int q = 0; q < kRing; q++) {
            if (!d.in_ready[q]) CV_TRY(hipEventCreateWithFlags(&d.in_ready[q], hipEventDisableTiming));
            if (!d.in_free[q]) CV_TRY(hipEventCreateWithFlags(&d.in_free[q], hipEventDisableTiming));
        }
        for (int k = 0; k < kStage; k++)
            if (!d.stage_ev[k]) CV_TRY(hipEventCreateWithFlags(&d.stage_ev[k], hipEventDisableTiming));
        // Blocks left below the ring's size by an earlier call grow here, all at once, before this call takes any:
        // a growth frees device memory, which waits for the whole device, and blocks grown one use at a time (a
        // block grows only when a request exceeds it) drained the GPU in call after call — fused C3 calls after
        // separate ones: 18 ms per call of host waits, their DMA done at 77 instead of 59 ms (profiles/r06j)
        for (int q = 0; q < kRing; q++) {
            if (!d.inblk[q].p || d.inblk[q].cap >= d.ring_max) continue;
            if (d.in_used[q]) CV_TRY(hipEventSynchronize(d.in_free[q]));
            CV_TRY(d.inblk[q].ensure(d.ring_max, false));
        }
        return CV_OK;
    }
    // error paths: drain every queue, forget the ring's state and finish every other pending output of
    // this device (an earlier call still in flight keeps its results)
    void drain() {
        (void)hipStreamSynchronize(d.copy);
        if (d.mstream) (void)hipStreamSynchronize(d.mstream);
        for (int k = 0; k < ns; k++) (void)hipStreamSynchronize(ss[k]);
        for (int q = 0; q < kRing; q++) d.in_used[q] = false;
        for (int k = 0; k < kStage; k++) d.stage_busy[k] = false;
        for (PipeOut &o : d.out)
            if (&o != &po) {
                std::lock_guard<std::mutex> g(o.mu);
                (void)pipe_finish(d, o);
            }
    }
    // The next ring block for a stage of `bytes` (waits for a growing block's last reader); the copy
    // stream waits (on the GPU) for the kernels that last read it.
    // A block grows straight to the largest block of the ring (at least 1.25x the request): freeing device
    // memory waits for the whole device, so a ring whose blocks grew one request at a time stalled every
    // call whose sub-chunk sizes differed from the last ones (a synchronous call's ramp, then async calls).
    // hint: the call's largest sub-chunk at this one's bytes per record, so a ramp's first small sub-chunks
    // do not size blocks that its later big ones must grow again.
    int block(int *q_out, size_t bytes, uint8_t **dv, size_t hint = 0) {
        const int q = d.ring_next;
        d.ring_next = (d.ring_next + 1) % kRing;
        if (bytes > d.inblk[q].cap) {
            if (d.in_used[q]) CV_TRY(hipEventSynchronize(d.in_free[q]));
            // one size for every block: ring_max itself, not 1.25x of it — with the buffer's own slack on top,
            // each growth made the next block 1.25x larger again (16 blocks: the last 28x the first; a C3 ring
            // reached ~35 GB)
            const size_t want = std::max(bytes, hint);
            d.ring_max = std::max(d.ring_max, want + want / 4);
            CV_TRY(d.inblk[q].ensure(d.ring_max, false));
        }
        if (d.in_used[q]) CV_TRY(hipStreamWaitEvent(d.copy, d.in_free[q], 0));
        *q_out = q;
        *dv = d.inblk[q].as<uint8_t>();
        return CV_OK;
    }
    // the next pinned staging block, free once its previous copy has left it
    int staging(int *k_out, size_t bytes, uint8_t **h) {
        const int k = d.stage_next;
        d.stage_next = (d.stage_next + 1) % kStage;
        if (d.stage_busy[k]) {
            CV_TRY(hipEventSynchronize(d.stage_ev[k]));
            d.stage_busy[k] = false;
        }
        CV_TRY(d.instage[k].ensure(bytes));
        *h = d.instage[k].as<uint8_t>();
        *k_out = k;
        return CV_OK;
    }
    // the copy out of staging block k was enqueued
    int staged(int k) {
        CV_TRY(hipEventRecord(d.stage_ev[k], d.copy));
        d.stage_busy[k] = true;
        return CV_OK;
    }
    // after sub-chunk j's copies into block q: compute stream j % 2 (or `on`) waits for them
    int copied(int q, int j, bool start_recorded = false, hipStream_t on = nullptr) {
        hipStream_t s = on ? on : ss[j % ns];
        if (tl) CV_TRY(tl_record(1 + 3 * (size_t)j, d.copy));
        CV_TRY(hipEventRecord(d.in_ready[q], d.copy));
        if (s != d.copy) CV_TRY(hipStreamWaitEvent(s, d.in_ready[q], 0));
        if (tl && !start_recorded) CV_TRY(tl_record(2 + 3 * (size_t)j, s));
        return CV_OK;
    }
    // after sub-chunk j's kernels (on compute stream j % 2, or `on`): block q is free once they are done.  A
    // stream other than the compute and copy streams is not joined by complete(): the caller makes a joined
    // stream wait for it.
    int launched(int q, int j, hipStream_t on = nullptr) {
        hipStream_t s = on ? on : ss[j % ns];
        if (tl) CV_TRY(tl_record(3 + 3 * (size_t)j, s));
        CV_TRY(hipEventRecord(d.in_free[q], s));
        d.in_used[q] = true;
        mark_used(s);
        chunks++;
        return CV_OK;
    }
    void mark_used(hipStream_t s) {
        for (int k = 0; k < ns; k++)
            if (ss[k] == s) used[k] = true;
        if (s == d.copy) used[kPipeSlots] = true;
    }
    // completion marks per slot stream (pipe_finish joins on the host; no GPU-side join, which would hold
    // the next call's kernels on that stream until this call had finished)
    int complete() {
        po.tl_n = tl ? (int)chunks : 0;
        for (int k = 0; k <= kPipeSlots; k++) {
            po.slot_used[k] = used[k];
            if (used[k]) CV_TRY(hipEventRecord(po.slot_done[k], k < kPipeSlots ? ss[k] : d.copy));
        }
        po.pending = true;
        po.gen++;
        return CV_OK;
    }
    void account(cv_ctx *ctx) {
        std::lock_guard<std::mutex> g(ctx->st_mu);
        Stats &S = ctx->stats;
        for (int k = 0; k < 4; k++) S.pipe[k] += t[k];
        S.pipe_calls++;
        S.pipe_chunks += chunks;
        S.pipe_direct += direct;
    }
};

// Enqueues the pipelined verify of shard [b, e) on device d into output po (held, not pending); returns
// without waiting for the GPU.  Sub-chunks (multiples of 64 signatures) go through the ring of kRing device
// input blocks: sub-chunk j's records reach block j % kRing on the device's ONE copy stream — straight from
// the caller's arrays when they are pinned (stage_direct), else packed by the host threads into pinned
// staging block j % kRing first — and are verified on slot j % 2's stream, which waits for that copy (event)
// and marks the block free when its kernels are done.  The copy stream waits (on the GPU) for the kernels
// that last read a block before refilling it, so copies run up to kRing sub-chunks ahead of the kernels and
// never queue behind a running kernel on a compute stream.  One copy queue matters: with copies on every
// slot stream the runtime ran those of one stream as blit kernels (`__amd_rocclr_copyBuffer`, ~37 GB/s, on
// the CUs beside the verify kernels) and the C2 host call took 13.8-16 ms for 9.6 ms of kernels
// (profiles/r03c_timeline_*.txt).  Two compute streams: with GPU_MAX_HW_QUEUES = 4 a third shared a
// hardware queue with the copy stream, whose copies then waited behind its Straus kernel (2.4 ms stalls,
// profiles/r03e_timeline_pinned_nofill.txt).
//
// Keyed shards (explicit keys, or the auto path's dedupe of the shard's keys on the host threads) first
// resolve their keys against the device's key pool (new keys' tables computed on slot 0's stream, the
// other stream waits for them), upload the distinct keys and their pool slots once, and stage per
// sub-chunk key indices instead of keys.
//
// async: the sub-chunk plan of the asynchronous entry points (async_chunk, up to twice that for big shards,
// no ramp — with a call in flight ahead of it the GPU is busy anyway, and bigger launches run closer to the
// kernels' rate: C2 1M best at 262,144, C5 8M at 524,288, profiles/r03l_async_chunk_sweep.log).
static int pipe_enqueue(cv_ctx *ctx, Device &d, const Opts &o, PipeOut &po, size_t b, size_t e, const VerifyIn &in,
                        int threads, bool async) {
    const size_t n = e - b;
    const size_t words = (n + 63) / 64;
    const size_t o_st = al16(words * 8), total_out = o_st + al16(n);
    PipeFrame f{d, po};
    f.ns = (int)o.pipe_slots;
    CV_TRY(hipSetDevice(d.ordinal));
    int rc = f.init();
    if (rc != CV_OK) return rc;
    CV_TRY(po.dout.ensure(total_out));
    uint8_t *dout = po.dout.as<uint8_t>();
    auto drain = on_exit([&f] { f.drain(); });
    WorkerPool *pool = &d.workers(threads);
    const bool keyed = in.keys != nullptr;
    // ---- keyed: the shard's distinct keys, resident in the pool, uploaded with their slots
    const uint8_t *keys = in.keys;
    const size_t nkeys = in.nkeys;
    const uint32_t *kidx = in.key_index;       // indexed by the caller's record index
    if (keyed) {
        double t0 = now_s();
        if (in.copy_kidx) {                        // the call's own dedupe output: into pinned memory (DMAed in place)
            CV_TRY(po.kidx.ensure(n * 4));
            std::memcpy(po.kidx.p, kidx + b, n * 4);
            kidx = po.kidx.as<uint32_t>() - b;     // so kidx[i] is record i's key, i in [b, e)
        }
        for (int k = 0; k < f.ns; k++) CV_TRY(pool_begin(d.kc, f.ss[k]));
        std::vector<uint32_t> sok;
        bool prepared = false;
        rc = key_resolve(d, ctx->key_cap.load(), nkeys, keys, in.used, sok, f.ss[0], &prepared);
        if (rc != CV_OK) return rc;
        if (prepared)                              // the other compute stream waits for the new tables
            for (int k = 1; k < f.ns; k++) CV_TRY(pool_begin(d.kc, f.ss[k]));
        const size_t kb = al16(nkeys * 32) + al16(nkeys * 4);
        CV_TRY(po.kstage.ensure(kb));
        CV_TRY(po.kdev.ensure(kb));
        std::memcpy(po.kstage.p, keys, nkeys * 32);
        std::memcpy(po.kstage.as<uint8_t>() + al16(nkeys * 32), sok.data(), nkeys * 4);
        // on the copy stream, ahead of every sub-chunk's records (the sub-chunks' in_ready events cover it)
        CV_TRY(hipMemcpyAsync(po.kdev.p, po.kstage.p, kb, hipMemcpyHostToDevice, d.copy));
        f.t[0] += now_s() - t0;
    }
    const uint8_t *kdev_keys = po.kdev.as<uint8_t>();
    const uint32_t *kdev_slot = keyed ? reinterpret_cast<const uint32_t *>(po.kdev.as<uint8_t>() + al16(nkeys * 32)) : nullptr;
    // asynchronous calls: whole multiples of CV_OPT_ASYNC_CHUNK (default one round of resident hs_straus waves,
    // 3 per SIMD x 1,024 SIMDs x 64 lanes = 196,608), one or two of them by the shard's size (n / 16), so each launch
    // group ends on a full round (profiles/r06d: C2 1M 9.80 ms per call at 196,608 against 9.91 at 262,144; C5 8M
    // 71.2 at 393,216 against 72-74)
    const size_t ach = async_sub_chunk(o, n);
    // synchronous calls: about 16 sub-chunks after the ramp, between 2 x pipe_first and pipe_chunk.  A 1M C2 call
    // (tools/sync_pipe_sweep.py, two rounds on one box): 262,144-record sub-chunks 13.0-13.3 ms, 98,304 12.0,
    // 65,536 11.6, 49,152 12.9, 32,768 13.3; an 8M C5 call is compute-bound and keeps 262,144 (74 ms).
    // (keyed calls keep pipe_chunk: each of their sub-chunks carries more fixed work)
    // (sub-chunks in whole rounds of resident waves after the ramp, 196,608 or 393,216: 10.97-11.9 ms per call
    // against 10.38 — fewer, larger sub-chunks leave a longer tail; profiles/r06t_sync_pipe_round_sweep.log)
    const size_t sch = keyed ? o.pipe_chunk
                             : std::min(o.pipe_chunk, std::max(2 * o.pipe_first, (n / o.pipe_split + 63) / 64 * 64));
    const std::vector<size_t> cut = async ? pipe_cuts(b, e, ach, ach, false) : pipe_cuts(b, e, o.pipe_first, sch, true);
    size_t max_m = 1;
    for (size_t j = 0; j + 1 < cut.size(); j++) max_m = std::max(max_m, cut[j + 1] - cut[j]);
    f.tl = o.timeline && !async;
    po.tl_ready = false;
    po.tl_merkle.clear();
    po.tl_pre_ms = 0;
    po.tl_first = cut.size() > 1 ? cut[1] - cut[0] : 0;
    for (size_t j = 0; j + 1 < cut.size(); j++) {
        const size_t c0 = cut[j], c1 = cut[j + 1], m = c1 - c0;
        Slot &sl = d.slot[j % f.ns];
        hipStream_t s = f.ss[j % f.ns];
        double t0 = now_s();
        const Stage st = stage_plan(c0, c1, in.off, in.len, pool, keyed);
        if (!stage_in_bounds(st, in.arena_bytes)) return CV_E_ARGS;   // before this sub-chunk's copy (drain: the ones before it)
        const bool direct = stage_direct(st, c0, in.pk, kidx, in.sig, in.arena, in.off, in.len);
        double t1 = now_s();
        f.t[0] += t1 - t0;
        int q;
        uint8_t *dv;
        if ((rc = f.block(&q, st.total, &dv, (size_t)((double)st.total / (double)m * (double)max_m))) != CV_OK) return rc;
        if (f.tl && j == 0) CV_TRY(f.tl_record(0, d.copy));
        // Synchronous calls: the first sub-chunk's keys and signatures (all the point decodes read: 96 of its ~400 B
        // per C2 record) are DMAed first and its point blocks start on the slot's helper stream as soon as they
        // land, beside the rest of the DMA and the scalars (CvkPrepOverlap, as the mid-size path): the ramp before
        // the first kernel is the DMA of 3 MB instead of 13 MB.
        CvkPrepOverlap pov;
        const bool overlap0 = !async && !keyed && j == 0 && o.pipe_overlap_first && m <= kVerifyChunk;
        if (overlap0) {
            CV_TRY(slot_split(d, sl));
            pov.aux = sl.split.s2;
            pov.ready = sl.split.start;
            pov.done = sl.split.done2;
        }
        if (direct) {
            t0 = now_s();
            f.t[2] += t0 - t1;
            if (overlap0) {
                CV_TRY(hipMemcpyAsync(dv + st.o_pk, in.pk + c0 * 32, m * 32, hipMemcpyHostToDevice, d.copy));
                CV_TRY(hipMemcpyAsync(dv + st.o_sig, in.sig + c0 * 64, m * 64, hipMemcpyHostToDevice, d.copy));
                CV_TRY(hipEventRecord(pov.ready, d.copy));
                CV_TRY(hipMemcpyAsync(dv + st.o_off, in.off + c0, m * 8, hipMemcpyHostToDevice, d.copy));
                CV_TRY(hipMemcpyAsync(dv + st.o_len, in.len + c0, m * 4, hipMemcpyHostToDevice, d.copy));
                if (st.hi > st.lo)
                    CV_TRY(hipMemcpyAsync(dv + st.o_ar, in.arena + st.lo, st.hi - st.lo, hipMemcpyHostToDevice, d.copy));
            } else {
                CV_TRY(stage_dma_direct(st, dv, c0, in.pk, kidx, in.sig, in.arena, in.off, in.len, d.copy));
            }
            f.direct++;
        } else {
            uint8_t *h;
            int sk;
            if ((rc = f.staging(&sk, st.total, &h)) != CV_OK) return rc;
            t0 = now_s();
            f.t[2] += t0 - t1;
            hipError_t e1 = hipSuccess;
            stage_pack(st, h, c0, in.pk, kidx, in.sig, in.arena, in.off, in.len, pool, [&] {
                if (!overlap0) return;
                e1 = hipMemcpyAsync(dv, h, st.o_off, hipMemcpyHostToDevice, d.copy);
                if (e1 == hipSuccess) e1 = hipEventRecord(pov.ready, d.copy);
            });
            CV_TRY(e1);
            t1 = now_s();
            f.t[1] += t1 - t0;
            t0 = t1;
            const size_t from = overlap0 ? st.o_off : 0;
            CV_TRY(hipMemcpyAsync(dv + from, h + from, st.total - from, hipMemcpyHostToDevice, d.copy));
            if ((rc = f.staged(sk)) != CV_OK) return rc;
        }
        if (f.tl && j == 0 && in.t_entry > 0) po.tl_pre_ms = (now_s() - in.t_entry) * 1e3;
        if (f.tl && overlap0) {   // the timeline's first kernel start: the point blocks on the helper stream
            CV_TRY(hipStreamWaitEvent(pov.aux, pov.ready, 0));
            CV_TRY(f.tl_record(2, pov.aux));
        }
        if ((rc = f.copied(q, (int)j, f.tl && overlap0)) != CV_OK) return rc;
        const size_t w0 = (c0 - b) / 64;
        const uint64_t *doff = reinterpret_cast<const uint64_t *>(dv + st.o_off);
        const uint32_t *dlen = reinterpret_cast<const uint32_t *>(dv + st.o_len);
        uint64_t *dbm = reinterpret_cast<uint64_t *>(dout) + w0;
        uint8_t *dst = in.status ? dout + o_st + (c0 - b) : nullptr;
        if (keyed) {
            CV_TRY(ensure_verify_ws(sl, m));
            CV_TRY(ws_begin(d, sl, s));
            const hipError_t ek = cvk_verify_keyed(&o.plan, (uint32_t)m, kdev_keys, reinterpret_cast<const uint32_t *>(dv + st.o_kidx),
                                                   kdev_slot, d.kc.ktab.as<uint32_t>(), d.kc.kok.as<uint8_t>(),
                                                   dv + st.o_sig, dv + st.o_ar - st.lo, doff, dlen, dbm, dst,
                                                   sl.ws_hs.as<uint32_t>(), sl.ws_R.as<uint32_t>(), sl.ws_ok.as<uint8_t>(),
                                                   sl.ws_cap, s, nullptr);
            const hipError_t e2 = ws_end(sl, s);
            CV_TRY(ek);
            CV_TRY(e2);
        } else {
            CV_TRY(launch_verify(d, o.plan, sl, (uint32_t)m, dv + st.o_pk, dv + st.o_sig, dv + st.o_ar - st.lo, doff, dlen,
                                 dbm, dst, s, nullptr, false, overlap0 ? &pov : nullptr));
        }
        if ((rc = f.launched(q, (int)j)) != CV_OK) return rc;
        f.t[3] += now_s() - t0;
    }
    if (keyed) {
        for (int k = 0; k < f.ns; k++)
            if (f.used[k]) CV_TRY(pool_end(d.kc, f.ss[k]));   // (the pool's last user: either stream)
        std::lock_guard<std::mutex> g(ctx->st_mu);
        ctx->stats.keyed_chunks += f.chunks;
    }
    if ((rc = f.complete()) != CV_OK) return rc;
    drain.armed = false;
    po.nseg = 0;
    po.seg[po.nseg++] = {in.bitmap + b / 64, 0, words * 8};
    if (in.status) po.seg[po.nseg++] = {in.status + b, o_st, n};
    f.account(ctx);
    return CV_OK;
}

// Enqueues the pipelined Merkle ids of transactions [t0, t1) on device d into output po: sub-chunks of about
// merkle_chunk leaves (whole transactions), each staged (direct DMA from pinned arrays, else packed) into a
// ring block by the copy stream and hashed on the copy stream itself behind its copies (leaf kernel + tree
// kernel, leaf digests in the device's digest buffer); the ids and statuses go to po's device buffer and come
// back once.  The leaf bytes dominate (C3: 2 GB per 1M transactions), so the call is bound by the copy.
struct MerkleIn {
    const uint8_t *arena;
    const uint64_t *off;
    const uint32_t *len;
    const uint32_t *txb;   // ntx + 1 absolute leaf indices
    uint8_t *ids, *status;
    uint64_t arena_bytes = UINT64_MAX;   // the caller's arena size (the _bounded / _ex entry points), else unbounded
};
// a Merkle stage's leaves inside the caller's arena (and none wrapping), checked before anything reads them
static bool mstage_in_bounds(const MStage &st, uint64_t arena_bytes) {
    return st.extent != UINT64_MAX && st.extent <= arena_bytes;
}
static int merkle_enqueue(cv_ctx *ctx, Device &d, const Opts &o, PipeOut &po, size_t t0, size_t t1, const MerkleIn &in,
                          int threads) {
    const size_t nt = t1 - t0;
    const size_t o_st = al16(nt * 32), total_out = o_st + al16(nt);
    PipeFrame f{d, po};
    CV_TRY(hipSetDevice(d.ordinal));
    int rc = f.init();
    if (rc != CV_OK) return rc;
    CV_TRY(po.dout.ensure(total_out));
    uint8_t *dout = po.dout.as<uint8_t>();
    auto drain = on_exit([&f] { f.drain(); });
    WorkerPool *pool = &d.workers(threads);
    // sub-chunk cuts: whole transactions, about merkle_chunk leaves each (at least one transaction), and at most
    // ~12 per shard, so one call's copies fit the ring ahead of its kernels
    const size_t nl_all = in.txb[t1] - in.txb[t0];
    const size_t per = std::max<size_t>(o.merkle_chunk, (nl_all + kRing - 5) / (kRing - 4));
    std::vector<size_t> cut{t0};
    while (cut.back() < t1) {
        const size_t c = cut.back();
        const uint64_t want = (uint64_t)in.txb[c] + per;
        size_t nx = (size_t)(std::upper_bound(in.txb + c + 1, in.txb + t1 + 1, (uint32_t)std::min<uint64_t>(want, UINT32_MAX)) - in.txb) - 1;
        nx = std::max(nx, c + 1);
        cut.push_back(std::min(nx, t1));
    }
    // The kernels run on the copy stream itself, behind the call's copies: on a compute stream they would queue
    // behind the verify kernels already there (a C3 node submits the Merkle ids of batch k+1 behind the verify
    // of batch k, which keeps both compute streams busy for ~75 ms: host C3 0.76x of the device rate), on the
    // copy stream they wait only for their leaves and take CU slots between the verify's waves.  The copies of
    // up to kRing - 2 sub-chunks go first, then their kernels (a copy stream stalled behind a kernel that waits
    // for CU slots moves nothing), so a call's copies run back to back.  One leaf-digest buffer serves them all
    // (the kernels run one after another); it grows after the copy stream's queued kernels.
    size_t max_nl = 0;
    for (size_t j = 0; j + 1 < cut.size(); j++) max_nl = std::max<size_t>(max_nl, in.txb[cut[j + 1]] - in.txb[cut[j]]);
    if (max_nl * 32 + 32 > d.digest.cap) {
        CV_TRY(hipStreamSynchronize(d.copy));
        CV_TRY(d.digest.ensure(max_nl * 32 + 32));
    }
    struct Pending {
        MStage st;
        int q;
        uint8_t *dv;
    };
    std::vector<Pending> pend;
    auto flush = [&]() -> int {
        const double ta = now_s();
        for (const Pending &p : pend) {
            const MStage &st = p.st;
            const size_t nl = st.l1 - st.l0;
            CV_TRY(cvk_merkle((uint32_t)(st.t1 - st.t0), (uint32_t)nl, (uint32_t)st.l0, p.dv + st.o_ar - st.lo,
                              reinterpret_cast<const uint64_t *>(p.dv + st.o_off),
                              reinterpret_cast<const uint32_t *>(p.dv + st.o_len),
                              reinterpret_cast<const uint32_t *>(p.dv + st.o_txb), d.digest.as<uint32_t>(),
                              dout + (st.t0 - t0) * 32, dout + o_st + (st.t0 - t0), d.copy));
            CV_TRY(hipEventRecord(d.in_free[p.q], d.copy));
            d.in_used[p.q] = true;
            f.chunks++;
        }
        pend.clear();
        f.used[kPipeSlots] = true;
        f.t[3] += now_s() - ta;
        return CV_OK;
    };
    for (size_t j = 0; j + 1 < cut.size(); j++) {
        const size_t c0 = cut[j], c1 = cut[j + 1];
        double ta = now_s();
        const MStage st = mstage_plan(c0, c1, in.txb, in.off, in.len, pool);
        if (!mstage_in_bounds(st, in.arena_bytes)) return CV_E_ARGS;   // past the arena, or a leaf's off + len wraps
        const bool direct = mstage_direct(st, in.txb, in.arena, in.off, in.len);
        double tb = now_s();
        f.t[0] += tb - ta;
        int q;
        uint8_t *dv;
        if ((rc = f.block(&q, st.total, &dv)) != CV_OK) return rc;
        if (direct) {
            ta = now_s();
            f.t[2] += ta - tb;
            CV_TRY(mstage_dma_direct(st, dv, in.txb, in.arena, in.off, in.len, d.copy));
            f.direct++;
        } else {
            uint8_t *h;
            int sk;
            if ((rc = f.staging(&sk, st.total, &h)) != CV_OK) return rc;
            ta = now_s();
            f.t[2] += ta - tb;
            mstage_pack(st, h, in.txb, in.arena, in.off, in.len, pool);
            tb = now_s();
            f.t[1] += tb - ta;
            ta = tb;
            CV_TRY(hipMemcpyAsync(dv, h, st.total, hipMemcpyHostToDevice, d.copy));
            if ((rc = f.staged(sk)) != CV_OK) return rc;
        }
        f.t[3] += now_s() - ta;
        pend.push_back({st, q, dv});
        if (pend.size() + 2 >= (size_t)kRing && (rc = flush()) != CV_OK) return rc;
    }
    if ((rc = flush()) != CV_OK) return rc;
    if ((rc = f.complete()) != CV_OK) return rc;
    drain.armed = false;
    po.nseg = 0;
    po.seg[po.nseg++] = {in.ids + t0 * 32, 0, nt * 32};
    if (in.status) po.seg[po.nseg++] = {in.status + t0, o_st, nt};
    f.account(ctx);
    {
        std::lock_guard<std::mutex> g(ctx->st_mu);
        ctx->stats.merkle_chunks += cut.size() - 1;
        ctx->stats.pipe_chunks -= f.chunks;   // counted as Merkle sub-chunks only
    }
    return CV_OK;
}

// One shard of a small synchronous Merkle call (a resolve chain's or a notary batch's transactions, staging below
// kMerkleSmall bytes): packed into slot 0's pinned staging (or DMAed in place from pinned arrays), one DMA, the
// two kernels, one result copy and one synchronisation — the pipeline's per-call frame (ring events, output
// join, result stream) costs more than it hides at this size.
constexpr size_t kMerkleSmall = 24u << 20;
static int merkle_shard_small(Device &d, const MStage &st, const MerkleIn &in, WorkerPool *pool) {
    const size_t nt = st.t1 - st.t0, nl = st.l1 - st.l0;
    const size_t o_st = al16(nt * 32), total_out = o_st + al16(nt);
    Slot &sl = d.slot[0];
    hipStream_t s = nullptr;
    CV_TRY(slot_stream(d, 0, &s));
    CV_TRY(slot_events(sl));
    CV_TRY(sl.pin_in.ensure(st.total));
    CV_TRY(sl.packed.ensure(st.total));
    CV_TRY(d.pin_out.ensure(total_out));
    CV_TRY(d.ids.ensure(total_out));
    if (nl * 32 + 32 > sl.mdig.cap) {
        if (sl.last && sl.ev) CV_TRY(hipEventSynchronize(sl.ev));
        CV_TRY(sl.mdig.ensure(nl * 32 + 32));
    }
    uint8_t *dv = sl.packed.as<uint8_t>();
    auto drain = on_exit([s] { (void)hipStreamSynchronize(s); });   // error paths: no DMA outlives the call
    if (st.total >= (1u << 20) && mstage_direct(st, in.txb, in.arena, in.off, in.len)) {
        CV_TRY(mstage_dma_direct(st, dv, in.txb, in.arena, in.off, in.len, s));
    } else if (!st.compact && st.hi - st.lo >= (4u << 20)) {
        // a contiguous leaf range of 4 MB and more: the records first, then the leaf bytes in 2 MB pieces, each
        // piece's DMA issued as soon as it is packed (the copies overlap the packing)
        uint8_t *h = sl.pin_in.as<uint8_t>();
        const size_t nl = st.l1 - st.l0, nt = st.t1 - st.t0;
        par_copy({{h + st.o_off, in.off + st.l0, nl * 8}, {h + st.o_len, in.len + st.l0, nl * 4},
                  {h + st.o_txb, in.txb + st.t0, (nt + 1) * 4}}, nullptr);
        CV_TRY(hipMemcpyAsync(dv, h, st.o_ar, hipMemcpyHostToDevice, s));
        const size_t span = st.hi - st.lo;
        constexpr size_t kPiece = 2u << 20;
        for (size_t p0 = 0; p0 < span; p0 += kPiece) {
            const size_t m = std::min(kPiece, span - p0);
            par_copy({{h + st.o_ar + p0, in.arena + st.lo + p0, m}}, pool);
            CV_TRY(hipMemcpyAsync(dv + st.o_ar + p0, h + st.o_ar + p0, m, hipMemcpyHostToDevice, s));
        }
    } else {
        mstage_pack(st, sl.pin_in.as<uint8_t>(), in.txb, in.arena, in.off, in.len, pool);
        CV_TRY(hipMemcpyAsync(dv, sl.pin_in.p, st.total, hipMemcpyHostToDevice, s));
    }
    uint8_t *dout = d.ids.as<uint8_t>();
    CV_TRY(ws_begin(d, sl, s));
    const hipError_t ek = cvk_merkle((uint32_t)nt, (uint32_t)nl, (uint32_t)st.l0, dv + st.o_ar - st.lo,
                                     reinterpret_cast<const uint64_t *>(dv + st.o_off),
                                     reinterpret_cast<const uint32_t *>(dv + st.o_len),
                                     reinterpret_cast<const uint32_t *>(dv + st.o_txb), sl.mdig.as<uint32_t>(), dout,
                                     dout + o_st, s);
    const hipError_t e2 = ws_end(sl, s);
    CV_TRY(ek);
    CV_TRY(e2);
    CV_TRY(hipMemcpyAsync(d.pin_out.p, dout, in.status ? o_st + nt : nt * 32, hipMemcpyDeviceToHost, s));
    CV_TRY(hipStreamSynchronize(s));
    drain.armed = false;
    std::memcpy(in.ids + st.t0 * 32, d.pin_out.p, nt * 32);
    if (in.status) std::memcpy(in.status + st.t0, d.pin_out.as<uint8_t>() + o_st, nt);
    return CV_OK;
}

// ---------------------------------------------------------------- transactions (verifySignatures)
// The fused form of SignedTransaction.verifySignatures over a batch: each transaction's id (WireTransaction.id)
// and whether every one of its signatures verifies over that id.  The ids are computed into the output's device
// buffer and read there as the signatures' messages: no id round trip through the host and no message upload,
// so a verify never waits for the host to hand it the ids of a Merkle call (the separate calls left the verify
// kernels idle ~6 ms per C3 step, profiles/README.md, round 4).
//
// One shard = transactions [t0, t1) and their signatures [s0, s1) on device d.  Sub-chunks of whole transactions
// (about merkle_chunk leaves, ramped: a quarter, a half, then full) and of signatures (multiples of 64 from s0,
// sized as pipe_enqueue's) share the input ring and the copy stream; the launch groups alternate over the two
// compute streams.  A Merkle group (leaf + tree kernels on the slot's digest workspace) records mev[J]; the
// signature groups whose transactions all lie in sub-chunks 0..J are issued after Merkle group J + 1, each
// waiting for its own copy and for the mev of every Merkle group its transactions lie in (a group may start
// inside an earlier sub-chunk, whose kernels can still be queued on the other stream), then writing its message
// references (cvk_tx_sig_refs: id offsets within the shard) and verifying.  Last, the per-transaction verdicts (cvk_tx_verdicts) on the stream of the
// last group, after the other stream's last group.
// dout: ids | Merkle status | tx_ok | signature status | verdict bitmap | message offsets | lengths | boundaries
struct TxIn {
    MerkleIn m;             // the leaves; m.ids and m.status may be null
    const uint8_t *pk, *sig;
    const uint32_t *tsb;    // ntx + 1 signature boundaries
    uint8_t *sig_status;    // may be null
    uint8_t *tx_ok;
    double t_entry = 0;     // host time the call entered the engine (CV_OPT_TIMELINE's host_pre)
};
static int txs_enqueue(cv_ctx *ctx, Device &d, const Opts &o, PipeOut &po, size_t t0, size_t t1, const TxIn &in,
                       int threads, bool async) {
    const MerkleIn &mi = in.m;
    const size_t nt = t1 - t0, s0 = in.tsb[t0], s1 = in.tsb[t1], ns = s1 - s0;
    const size_t words = (ns + 63) / 64;
    const size_t o_mst = al16(nt * 32), o_ok = o_mst + al16(nt), o_sst = o_ok + al16(nt);
    const size_t o_bm = o_sst + (in.sig_status ? al16(ns) : 0), o_off = o_bm + al16(words * 8);
    const size_t o_len = o_off + al16(ns * 8), o_tsb = o_len + al16(ns * 4), total_out = o_tsb + al16((nt + 1) * 4);
    PipeFrame f{d, po};
    f.ns = (int)o.pipe_slots;
    CV_TRY(hipSetDevice(d.ordinal));
    int rc = f.init();
    if (rc != CV_OK) return rc;
    CV_TRY(po.dout.ensure(total_out));
    uint8_t *dout = po.dout.as<uint8_t>();
    const uint32_t *dtsb = reinterpret_cast<const uint32_t *>(dout + o_tsb);
    uint64_t *doff = reinterpret_cast<uint64_t *>(dout + o_off);
    uint32_t *dlen = reinterpret_cast<uint32_t *>(dout + o_len);
    uint64_t *dbm = reinterpret_cast<uint64_t *>(dout + o_bm);
    auto drain = on_exit([&f] { f.drain(); });
    WorkerPool *pool = &d.workers(threads);
    f.tl = o.timeline && !async;   // (timeline: groups tagged Merkle / verify in po.tl_merkle)
    po.tl_ready = false;
    po.tl_merkle.clear();
    po.tl_pre_ms = 0;
    po.tl_first = 0;
    if (f.tl) CV_TRY(f.tl_record(0, d.copy));
    // the shard's signature boundaries go first on the copy stream, so every group's copy event covers them
    {
        const double ta = now_s();
        const uint32_t *src = in.tsb + t0;
        if (!host_pinned(src, (nt + 1) * 4)) {   // (po was finished by pipe_out: no DMA still reads tstage)
            CV_TRY(po.tstage.ensure((nt + 1) * 4));
            std::memcpy(po.tstage.p, src, (nt + 1) * 4);
            src = po.tstage.as<uint32_t>();
        }
        CV_TRY(hipMemcpyAsync(dout + o_tsb, src, (nt + 1) * 4, hipMemcpyHostToDevice, d.copy));
        f.t[0] += now_s() - ta;
        if (f.tl) po.tl_pre_ms = (now_s() - in.t_entry) * 1e3;
    }
    // Merkle sub-chunks: whole transactions, ramped up to `per` leaves (at least one transaction each)
    const size_t nl_all = mi.txb[t1] - mi.txb[t0];
    // about six full Merkle sub-chunks per shard (C3: 1M leaves, ~360 MB each): twelve were 3-4 % slower per
    // call (85.3-86.3 against 82.5-82.6 ms, profiles/r04o_fused_merkle_chunk.log) — fewer Merkle groups to
    // interleave with the signature groups' kernels
    const size_t per = std::max<size_t>(o.merkle_chunk, (nl_all + 5) / 6);
    std::vector<size_t> mcut{t0};
    for (size_t want = std::max<size_t>(1, per / 4); mcut.back() < t1; want = std::min(per, 2 * want)) {
        const size_t c = mcut.back();
        const uint64_t target = (uint64_t)mi.txb[c] + want;
        size_t nx = (size_t)(std::upper_bound(mi.txb + c + 1, mi.txb + t1 + 1,
                                              (uint32_t)std::min<uint64_t>(target, UINT32_MAX)) - mi.txb) - 1;
        mcut.push_back(std::min(std::max(nx, c + 1), t1));
    }
    const size_t nm = mcut.size() - 1;
    size_t max_nl = 0;
    for (size_t j = 0; j < nm; j++) max_nl = std::max<size_t>(max_nl, mi.txb[mcut[j + 1]] - mi.txb[mcut[j]]);
    // CV_OPT_TXS_MERKLE_STREAM: the Merkle groups on the compute streams (0: each group takes the next slot, its
    // leaf digests in that slot's workspace), or all on one stream (1 the copy stream, behind their leaves; 2 a
    // stream of their own, the default) with one leaf-digest buffer, their groups running one after another there.
    // Async C3 (1M txs x 8 signers) per call, interleaved on three boxes: 0 82.8 / 82.8, 80.0 / 80.3, 82.9 / 81.8 ms;
    // 1 83.4 / 82.8; 2 80.3 / 81.6, 78.6 / 79.3, 80.8 / 80.9 (profiles/r06k_*, r06l_*, r06m_*): off the compute
    // streams the signature groups alternate undisturbed and the Merkle kernels take CU slots between their waves
    hipStream_t mst = nullptr;
    DevBuf *mdig = nullptr;
    if (o.txs_merkle_stream == 1) {
        mst = d.copy;
        mdig = &d.digest;   // (the separate Merkle calls' buffer: they run on the copy stream too)
    } else if (o.txs_merkle_stream == 2) {
        if (!d.mstream) CV_TRY(hipStreamCreateWithFlags(&d.mstream, hipStreamNonBlocking));
        mst = d.mstream;
        mdig = &d.mdigest;
    }
    if (mst) {
        if (max_nl * 32 + 32 > mdig->cap) {
            CV_TRY(hipStreamSynchronize(mst));
            CV_TRY(mdig->ensure(max_nl * 32 + 32));
        }
    } else {
        for (int k = 0; k < f.ns; k++) {   // the two slots' leaf-digest workspaces
            Slot &sl = d.slot[k];
            if (max_nl * 32 + 32 > sl.mdig.cap) {
                if (sl.last && sl.ev) CV_TRY(hipEventSynchronize(sl.ev));
                CV_TRY(hipStreamSynchronize(f.ss[k]));
                CV_TRY(sl.mdig.ensure(max_nl * 32 + 32));
            }
        }
    }
    while (d.mev.size() < nm + 1) {
        hipEvent_t v = nullptr;
        CV_TRY(hipEventCreateWithFlags(&v, hipEventDisableTiming));
        d.mev.push_back(v);
    }
    // signature sub-chunks: as pipe_enqueue's plan for ns records; at least vmin unless the shard ends there
    const size_t vch = async ? async_sub_chunk(o, ns)
                             : std::min(o.pipe_chunk, std::max(2 * o.pipe_first, (ns / 16 + 63) / 64 * 64));
    // (signature groups of whole vch units only, the records past a Merkle sub-chunk's last whole group joining the
    // next sub-chunk's: 1-2 % slower per async C3 call, profiles/r06m_txs_whole_groups_ab.log)
    const size_t vmin = std::min(vch, std::max<size_t>(o.pipe_first, 4096));
    int g = 0;           // launch groups so far (group g runs on compute stream g % 2)
    int vg = 0;          // signature groups so far (with the Merkle groups on their own stream: on stream vg % 2)
    size_t p = s0;       // the next signature to stage
    // the signature groups whose transactions all lie in Merkle sub-chunks 0..jc (to the shard's end if last)
    auto emit_sigs = [&](size_t jc, bool last) -> int {
        const size_t avail = last ? s1 : s0 + (in.tsb[mcut[jc + 1]] - s0) / 64 * 64;
        while (p < avail) {
            const size_t m = std::min(vch, avail - p);
            if (!last && m < vmin) break;
            double ta = now_s();
            const size_t o_sig = al16(m * 32), bytes = o_sig + al16(m * 64);
            int q;
            uint8_t *dv;
            int r = f.block(&q, bytes, &dv, al16(vch * 32) + al16(vch * 64));
            if (r != CV_OK) return r;
            double tb;
            if (host_pinned(in.pk + p * 32, m * 32) && host_pinned(in.sig + p * 64, m * 64)) {
                tb = now_s();
                f.t[2] += tb - ta;
                CV_TRY(hipMemcpyAsync(dv, in.pk + p * 32, m * 32, hipMemcpyHostToDevice, d.copy));
                CV_TRY(hipMemcpyAsync(dv + o_sig, in.sig + p * 64, m * 64, hipMemcpyHostToDevice, d.copy));
                f.direct++;
            } else {
                uint8_t *h;
                int sk;
                if ((r = f.staging(&sk, bytes, &h)) != CV_OK) return r;
                tb = now_s();
                f.t[2] += tb - ta;
                par_copy({{h, in.pk + p * 32, m * 32}, {h + o_sig, in.sig + p * 64, m * 64}}, pool);
                ta = now_s();
                f.t[1] += ta - tb;
                tb = ta;
                CV_TRY(hipMemcpyAsync(dv, h, bytes, hipMemcpyHostToDevice, d.copy));
                if ((r = f.staged(sk)) != CV_OK) return r;
            }
            const int ks = mst ? vg++ % f.ns : g % f.ns;
            Slot &sl = d.slot[ks];
            hipStream_t s = f.ss[ks];
            if ((r = f.copied(q, g, false, s)) != CV_OK) return r;
            // every Merkle group holding one of its transactions: the first one's (the largest t with tsb[t] <= p)
            // through jc — a group on the other stream may not have run yet
            const size_t tf = (size_t)(std::upper_bound(in.tsb + t0, in.tsb + t1 + 1, (uint32_t)p) - in.tsb) - 1;
            const size_t jf = (size_t)(std::upper_bound(mcut.begin(), mcut.end(), tf) - mcut.begin()) - 1;
            for (size_t j = jf; j <= jc; j++) CV_TRY(hipStreamWaitEvent(s, d.mev[j], 0));
            const size_t c0 = p - s0;
            CV_TRY(cvk_tx_sig_refs((uint32_t)m, (uint32_t)c0, (uint32_t)nt, (uint32_t)s0, dtsb, doff, dlen, s));
            CV_TRY(launch_verify(d, o.plan, sl, (uint32_t)m, dv, dv + o_sig, dout, doff + c0, dlen + c0, dbm + c0 / 64,
                                 in.sig_status ? dout + o_sst + c0 : nullptr, s, nullptr, false));
            if (f.tl) po.tl_merkle.push_back(0);
            if ((r = f.launched(q, g++, s)) != CV_OK) return r;
            f.t[3] += now_s() - tb;
            p += m;
        }
        return CV_OK;
    };
    // On the compute streams, Merkle group J goes one step ahead of the signature groups of sub-chunk J - 1, so on
    // its stream it queues behind older signature groups only and has usually run by the time the groups that read
    // its ids start.  On a stream of its own it waits for nothing but its leaves, so the signature groups of
    // sub-chunk J follow it directly: the call's first signature group no longer waits for a second Merkle group's
    // copy (the loop's fill)
#ifdef CV_TXS_LAG   // (A/B builds only)
    const size_t lag = CV_TXS_LAG;
#else
    const size_t lag = mst ? 0 : 1;
#endif
    for (size_t J = 0; J < nm; J++) {
        double ta = now_s();
        const MStage st = mstage_plan(mcut[J], mcut[J + 1], mi.txb, mi.off, mi.len, pool);
        if (!mstage_in_bounds(st, mi.arena_bytes)) return CV_E_ARGS;   // past the arena, or a leaf's off + len wraps
        const bool direct = mstage_direct(st, mi.txb, mi.arena, mi.off, mi.len);
        double tb = now_s();
        f.t[0] += tb - ta;
        int q;
        uint8_t *dv;
        if ((rc = f.block(&q, st.total, &dv, (size_t)((double)st.total / (double)std::max<size_t>(1, st.l1 - st.l0) *
                                                      (double)max_nl))) != CV_OK)
            return rc;
        if (direct) {
            ta = now_s();
            f.t[2] += ta - tb;
            CV_TRY(mstage_dma_direct(st, dv, mi.txb, mi.arena, mi.off, mi.len, d.copy));
            f.direct++;
        } else {
            uint8_t *h;
            int sk;
            if ((rc = f.staging(&sk, st.total, &h)) != CV_OK) return rc;
            ta = now_s();
            f.t[2] += ta - tb;
            mstage_pack(st, h, mi.txb, mi.arena, mi.off, mi.len, pool);
            tb = now_s();
            f.t[1] += tb - ta;
            ta = tb;
            CV_TRY(hipMemcpyAsync(dv, h, st.total, hipMemcpyHostToDevice, d.copy));
            if ((rc = f.staged(sk)) != CV_OK) return rc;
        }
        hipStream_t s = mst ? mst : f.ss[g % f.ns];
        if ((rc = f.copied(q, g, false, s)) != CV_OK) return rc;
        {
            Slot *sl = mst ? nullptr : &d.slot[g % f.ns];
            if (sl) CV_TRY(ws_begin(d, *sl, s));
            const hipError_t ek = cvk_merkle((uint32_t)(st.t1 - st.t0), (uint32_t)(st.l1 - st.l0), (uint32_t)st.l0,
                                             dv + st.o_ar - st.lo, reinterpret_cast<const uint64_t *>(dv + st.o_off),
                                             reinterpret_cast<const uint32_t *>(dv + st.o_len),
                                             reinterpret_cast<const uint32_t *>(dv + st.o_txb),
                                             sl ? sl->mdig.as<uint32_t>() : mdig->as<uint32_t>(),
                                             dout + (st.t0 - t0) * 32, dout + o_mst + (st.t0 - t0), s);
            const hipError_t e2 = sl ? ws_end(*sl, s) : hipSuccess;
            CV_TRY(ek);
            CV_TRY(e2);
            if (sl) CV_TRY(hipEventRecord(d.mev[J], s));
        }
        if (f.tl) po.tl_merkle.push_back(1);
        if ((rc = f.launched(q, g++, s)) != CV_OK) return rc;
        // (own stream: after launched()'s events, so a stream that waits for mev[J] also covers them)
        if (mst) CV_TRY(hipEventRecord(d.mev[J], s));
        f.t[3] += now_s() - ta;
        if (J >= lag && (rc = emit_sigs(J - lag, false)) != CV_OK) return rc;
    }
    if ((rc = emit_sigs(nm - 1, true)) != CV_OK) return rc;
    // ---- per-transaction verdicts, behind both streams' last groups
    {
        const int kl = mst ? (vg + f.ns - 1) % f.ns : (g - 1) % f.ns;
        hipStream_t s = f.ss[kl];
        for (int k = 0; k < f.ns; k++)
            if (k != kl && f.used[k]) {
                CV_TRY(hipEventRecord(d.mev[nm], f.ss[k]));
                CV_TRY(hipStreamWaitEvent(s, d.mev[nm], 0));
            }
        // Merkle groups on a stream of their own: the last one (every transaction's status and id) first; the
        // call's join on this stream then covers that stream's part of the call as well
        if (mst && nm) CV_TRY(hipStreamWaitEvent(s, d.mev[nm - 1], 0));
        CV_TRY(cvk_tx_verdicts((uint32_t)nt, (uint32_t)s0, dtsb, dout + o_mst, dbm, dout + o_ok, s));
        f.mark_used(s);
    }
    if ((rc = f.complete()) != CV_OK) return rc;
    drain.armed = false;
    po.nseg = 0;
    po.seg[po.nseg++] = {in.tx_ok + t0, o_ok, nt};
    if (mi.ids) po.seg[po.nseg++] = {mi.ids + t0 * 32, 0, nt * 32};
    if (mi.status) po.seg[po.nseg++] = {mi.status + t0, o_mst, nt};
    if (in.sig_status && ns) po.seg[po.nseg++] = {in.sig_status + s0, o_sst, ns};
    f.account(ctx);
    {
        std::lock_guard<std::mutex> g2(ctx->st_mu);
        ctx->stats.merkle_chunks += nm;
    }
    return CV_OK;
}

// A finished synchronous call's GPU timeline (CV_OPT_TIMELINE) into the context's sums.  The caller holds st_mu.
static void timeline_account(cv_ctx *ctx, PipeOut &po) {
    if (!po.tl_ready) return;
    po.tl_sum[kTlVals - 1] = (now_s() - po.tl_join_s) * 1e3;   // GPU work joined -> the call's results are back
    for (int k = 0; k < kTlVals; k++) ctx->stats.tl[k] += po.tl_sum[k];
    ctx->stats.tl[kTlVals] += 1;
    po.tl_ready = false;
}

// A pipelined call's part on one device, for its ticket: (device index, output index, gen).
using Part = std::array<uint64_t, 3>;

// One shard of a verify call on device d.  Synchronous calls: small plain shards take the one-DMA (or
// zero-copy) path, the rest the pipeline and wait for it; asynchronous calls always take the pipeline and
// record their output in *part.
static size_t dev_index(cv_ctx *ctx, const Device &d) {
    for (size_t k = 0; k < ctx->devs.size(); k++)
        if (ctx->devs[k].get() == &d) return k;
    return 0;
}

// One shard of a verify call on device d.  Synchronous calls: small plain shards take the one-DMA (or
// zero-copy) path, the rest the pipeline and wait for it; asynchronous calls always take the pipeline and
// record their output in *part.  Auto-keyed shards dedupe their own keys first (on the device's host
// threads) and fall back to the plain path when they repeat fewer than eight times per key.
static int verify_shard(cv_ctx *ctx, Device &d, const Opts &o, size_t b, size_t e, const VerifyIn &in0, int threads,
                        bool async, Part *part) {
    const size_t n = e - b;
    if (n == 0) return CV_OK;
    if (n > 0xffffffffull) return CV_E_TOO_LARGE;
    CV_TRY(hipSetDevice(d.ordinal));
    VerifyIn in = in0;
    std::vector<uint8_t> dkeys, used;
    std::vector<uint32_t> didx;
    if (in.auto_keyed) {
        const double t0 = now_s();
        in.auto_keyed = false;
        if (dedupe_keys(n, in.pk + b * 32, dkeys, didx, &d.workers(threads), false)) {
            in.keys = dkeys.data();
            in.nkeys = dkeys.size() / 32;
            in.key_index = didx.data() - b;        // indexed by the caller's record index
            in.copy_kidx = true;
        }
        std::lock_guard<std::mutex> g(ctx->st_mu);
        ctx->stats.pipe[0] += now_s() - t0;
    } else if (in.keys) {
        used.assign(in.nkeys, 0);
        for (size_t i = b; i < e; i++) {
            if (in.key_index[i] >= in.nkeys) return CV_E_ARGS;
            used[in.key_index[i]] = 1;
        }
        in.used = used.data();
    }
    const bool keyed = in.keys != nullptr;
    if (!async && !keyed && n <= o.pipe_min) return verify_shard_small(ctx, d, o, b, e, in, threads);
    int k = 0;
    std::unique_lock<std::mutex> lk;
    const double tw = now_s();
    PipeOut &po = pipe_out(d, &k, lk);   // (finishes that output's previous call if still pending)
    {
        std::lock_guard<std::mutex> g(ctx->st_mu);
        ctx->stats.pipe[2] += now_s() - tw;
    }
    int rc = pipe_enqueue(ctx, d, o, po, b, e, in, threads, async);
    if (rc != CV_OK) return rc;
    if (keyed) {
        std::lock_guard<std::mutex> g(ctx->st_mu);
        ctx->stats.keyed_calls++;
    }
    if (async) {
        *part = {(uint64_t)dev_index(ctx, d), (uint64_t)k, po.gen};
        po.ticketed = true;
        return CV_OK;
    }
    const double t0 = now_s();
    rc = pipe_finish(d, po);
    std::lock_guard<std::mutex> g(ctx->st_mu);
    ctx->stats.pipe[4] += now_s() - t0;
    timeline_account(ctx, po);
    return rc;
}

// A ticket for the parts of an asynchronous call.  Once 64 tickets are outstanding, those whose every part is
// done (its output finished, or reused by a later call) move to the finished list with their result, so a
// caller that drops tickets does not grow the live map and a late cv_wait still gets the call's status; the
// finished list keeps the last kTicketsDone results.
constexpr size_t kTicketsDone = 4096;
static uint64_t ticket_add(cv_ctx *ctx, std::vector<Part> parts) {
    std::lock_guard<std::mutex> g(ctx->tk_mu);
    if (ctx->tickets.size() >= 64) {
        for (auto it = ctx->tickets.begin(); it != ctx->tickets.end();) {
            bool live = false;
            int rc = CV_OK;
            for (const Part &p : it->second) {
                PipeOut &po = ctx->devs[p[0]]->out[p[1]];
                std::lock_guard<std::mutex> pg(po.mu);
                live = live || (po.gen == p[2] && po.pending);
                const int r = po.result_of(p[2]);
                if (r != CV_OK) rc = r;
            }
            if (live) {
                ++it;
                continue;
            }
            ctx->tickets_done.emplace(it->first, rc);
            it = ctx->tickets.erase(it);
        }
        while (ctx->tickets_done.size() > kTicketsDone) ctx->tickets_done.erase(ctx->tickets_done.begin());
    }
    const uint64_t t = ++ctx->next_ticket;
    ctx->tickets.emplace(t, std::move(parts));
    return t;
}

// Waits for parts (each output's lock only — no device lock, so other threads keep submitting) and returns
// the first error of any part, also of parts an earlier call's reuse of their output already finished.
static int parts_wait(cv_ctx *ctx, const std::vector<Part> &parts) {
    int rc = CV_OK;
    for (const Part &p : parts) {
        Device &d = *ctx->devs[p[0]];
        PipeOut &po = d.out[p[1]];
        std::lock_guard<std::mutex> g(po.mu);
        const int r = (po.gen == p[2] && po.pending) ? pipe_finish(d, po) : po.result_of(p[2]);
        if (r != CV_OK && rc == CV_OK) rc = r;
    }
    return rc;
}

// The keyed decision of the plain entry points: batches the tri-chain latency form takes (n <= tri_max)
// stay on the plain path whatever their keys — there the per-signature chain is the latency, and the tri
// chain beats the keyed comb chain (notary batch of 4,096 with 64 signers 0.47 vs 0.34 ms distinct).
static bool want_keyed(const Opts &o, size_t n, const uint8_t *pk) {
    if (!o.auto_keyed || n <= o.plan.tri_max) return false;
    return dedupe_gate(n, pk);
}

extern "C" {

// Diagnostic: the host-side key dedupe of cv_ed25519_verify_batch on its own (no device needed).
int cv_diag_dedupe_keys(size_t n, const uint8_t *pk, uint32_t *key_index, size_t *nkeys) {
    if (!pk || !key_index || !nkeys) return CV_E_ARGS;
    std::vector<uint8_t> keys;
    std::vector<uint32_t> idx;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    std::unique_ptr<WorkerPool> pool(n >= 65536 ? new WorkerPool((int)std::min(7u, hw - 1)) : nullptr);
    if (!dedupe_keys(n, pk, keys, idx, pool.get())) {
        *nkeys = 0;
        return 0;
    }
    std::memcpy(key_index, idx.data(), n * sizeof(uint32_t));
    *nkeys = keys.size() / 32;
    return 1;
}

static int verify_call(cv_ctx *ctx, size_t n, VerifyIn in, uint64_t *ticket) {
    in.t_entry = now_s();
    const Opts o = ctx->opts();
    const bool async = ticket != nullptr;
    if (!in.keys && want_keyed(o, n, in.pk)) in.auto_keyed = true;
    std::vector<Part> parts(ctx->devs.size(), Part{UINT64_MAX, 0, 0});
    const int rc = dispatch(ctx, o, n, 64, [&](Device &d, size_t b, size_t e, int threads) {
        Part p{UINT64_MAX, 0, 0};
        const int r = verify_shard(ctx, d, o, b, e, in, threads, async, &p);
        if (r == CV_OK && async && p[0] != UINT64_MAX) parts[dev_index(ctx, d)] = p;
        return r;
    });
    std::vector<Part> live;
    for (const Part &p : parts)
        if (p[0] != UINT64_MAX) live.push_back(p);
    if (rc != CV_OK) {
        // a shard failed: the shards that did enqueue are waited for here — nothing may read the caller's
        // arrays or write its bitmap after an error return
        (void)parts_wait(ctx, live);
        return rc;
    }
    if (async) *ticket = live.empty() ? 0 : ticket_add(ctx, std::move(live));
    return CV_OK;
}

int cv_ed25519_verify_batch(cv_ctx *ctx, size_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg_arena,
                            const uint64_t *msg_off, const uint32_t *msg_len, uint64_t *verdict_bitmap,
                            uint8_t *status) {
    if (!ctx) return CV_E_ARGS;
    if (n == 0) return CV_OK;
    if (!pk || !sig || !msg_off || !msg_len || !verdict_bitmap) return CV_E_ARGS;
    VerifyIn in;
    in.pk = pk;
    in.sig = sig;
    in.arena = msg_arena;
    in.off = msg_off;
    in.len = msg_len;
    in.bitmap = verdict_bitmap;
    in.status = status;
    return verify_call(ctx, n, in, nullptr);
}

int cv_ed25519_verify_batch_async(cv_ctx *ctx, size_t n, const uint8_t *pk, const uint8_t *sig,
                                  const uint8_t *msg_arena, const uint64_t *msg_off, const uint32_t *msg_len,
                                  uint64_t *verdict_bitmap, uint8_t *status, uint64_t *ticket) {
    if (!ctx || !ticket) return CV_E_ARGS;
    *ticket = 0;
    if (n == 0) return CV_OK;
    if (!pk || !sig || !msg_off || !msg_len || !verdict_bitmap) return CV_E_ARGS;
    VerifyIn in;
    in.pk = pk;
    in.sig = sig;
    in.arena = msg_arena;
    in.off = msg_off;
    in.len = msg_len;
    in.bitmap = verdict_bitmap;
    in.status = status;
    return verify_call(ctx, n, in, ticket);
}

int cv_ed25519_verify_batch_ex(cv_ctx *ctx, size_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg_arena,
                               uint64_t arena_bytes, const uint64_t *msg_off, const uint32_t *msg_len,
                               uint64_t *verdict_bitmap, uint8_t *status, uint64_t *ticket) {
    if (!ctx) return CV_E_ARGS;
    if (ticket) *ticket = 0;
    if (n == 0) return CV_OK;
    if (!pk || !sig || !msg_off || !msg_len || !verdict_bitmap) return CV_E_ARGS;
    VerifyIn in;
    in.pk = pk;
    in.sig = sig;
    in.arena = msg_arena;
    in.off = msg_off;
    in.len = msg_len;
    in.bitmap = verdict_bitmap;
    in.status = status;
    in.arena_bytes = arena_bytes;
    return verify_call(ctx, n, in, ticket);
}

int cv_wait(cv_ctx *ctx, uint64_t ticket) {
    if (!ctx) return CV_E_ARGS;
    if (ticket == 0) return CV_OK;
    std::vector<Part> parts;
    {
        std::lock_guard<std::mutex> g(ctx->tk_mu);
        auto it = ctx->tickets.find(ticket);
        if (it == ctx->tickets.end()) {
            auto dn = ctx->tickets_done.find(ticket);
            if (dn == ctx->tickets_done.end()) return CV_E_ARGS;
            const int rc = dn->second;
            ctx->tickets_done.erase(dn);
            return rc;
        }
        parts = std::move(it->second);
        ctx->tickets.erase(it);
    }
    return parts_wait(ctx, parts);
}

int cv_ed25519_verify_batch_keyed(cv_ctx *ctx, size_t n, size_t nkeys, const uint8_t *keys, const uint32_t *key_index,
                                  const uint8_t *sig, const uint8_t *msg_arena, const uint64_t *msg_off,
                                  const uint32_t *msg_len, uint64_t *verdict_bitmap, uint8_t *status) {
    if (!ctx) return CV_E_ARGS;
    if (n == 0) return CV_OK;
    if (!keys || !key_index || !sig || !msg_off || !msg_len || !verdict_bitmap || nkeys == 0) return CV_E_ARGS;
    if (nkeys > 0xffffffffull) return CV_E_TOO_LARGE;
    VerifyIn in;
    in.sig = sig;
    in.arena = msg_arena;
    in.off = msg_off;
    in.len = msg_len;
    in.keys = keys;
    in.key_index = key_index;
    in.nkeys = nkeys;
    in.bitmap = verdict_bitmap;
    in.status = status;
    return verify_call(ctx, n, in, nullptr);
}

int cv_key_cache_reserve(cv_ctx *ctx, size_t max_keys) {
    if (!ctx || max_keys == 0 || max_keys > 0x7fffffffull) return CV_E_ARGS;
    ctx->key_cap.store((uint32_t)max_keys);
    return CV_OK;
}

int cv_key_cache_stats(cv_ctx *ctx, int device, uint64_t *out4) {
    if (!ctx || !out4) return CV_E_ARGS;
    Device *d = find_dev(ctx, device);
    if (!d) return CV_E_ARGS;
    out4[0] = out4[1] = out4[2] = out4[3] = 0;
    for (auto &dp : ctx->devs) {            // every (virtual) device of that ordinal
        if (dp->ordinal != device) continue;
        std::lock_guard<std::mutex> g(dp->mu);
        out4[0] += dp->kc.map.size();
        out4[1] += dp->kc.cap;
        out4[2] += dp->kc.hits;
        out4[3] += dp->kc.misses;
    }
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
    auto drain = on_exit([s] { (void)hipStreamSynchronize(s); });   // the pageable copies read the caller's arrays
    CV_TRY(hipMemcpyAsync(d.seed.p, seed + b * 32, n * 32, hipMemcpyHostToDevice, s));
    if (hi > lo) CV_TRY(hipMemcpyAsync(d.arena.p, arena + lo, hi - lo, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(d.off.p, off + b, n * 8, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(d.len.p, len + b, n * 4, hipMemcpyHostToDevice, s));
    CV_TRY(cvk_sign((uint32_t)n, d.seed.as<uint8_t>(), d.arena.as<uint8_t>() - lo, d.off.as<uint64_t>(),
                    d.len.as<uint32_t>(), d.pk.as<uint8_t>(), d.sig.as<uint8_t>(), s));
    CV_TRY(hipMemcpyAsync(pk + b * 32, d.pk.p, n * 32, hipMemcpyDeviceToHost, s));
    CV_TRY(hipMemcpyAsync(sig + b * 64, d.sig.p, n * 64, hipMemcpyDeviceToHost, s));
    CV_TRY(hipStreamSynchronize(s));
    drain.armed = false;
    return CV_OK;
}

int cv_ed25519_sign_batch(cv_ctx *ctx, size_t n, const uint8_t *seed, const uint8_t *msg_arena,
                          const uint64_t *msg_off, const uint32_t *msg_len, uint8_t *pk_out, uint8_t *sig_out) {
    if (!ctx) return CV_E_ARGS;
    if (n == 0) return CV_OK;
    if (!seed || !msg_off || !msg_len || !pk_out || !sig_out) return CV_E_ARGS;
    const Opts o = ctx->opts();
    return dispatch(ctx, o, n, 64, [&](Device &d, size_t b, size_t e, int) {
        return sign_shard(d, b, e, seed, msg_arena, msg_off, msg_len, pk_out, sig_out);
    });
}

// ---------------------------------------------------------------- Merkle (host buffers)
static int merkle_call(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                       const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, uint8_t *ids, uint8_t *tx_status,
                       uint64_t *ticket, uint64_t arena_bytes = UINT64_MAX) {
    if (!ctx) return CV_E_ARGS;
    if (ticket) *ticket = 0;
    if (ntx == 0) return CV_OK;
    if (!tx_leaf_begin || !ids) return CV_E_ARGS;
    const size_t nleaves = tx_leaf_begin[ntx];
    if (tx_leaf_begin[0] != 0) return CV_E_ARGS;
    for (size_t t = 0; t < ntx; t++)
        if (tx_leaf_begin[t + 1] < tx_leaf_begin[t]) return CV_E_ARGS;
    if (nleaves && (!leaf_off || !leaf_len)) return CV_E_ARGS;
    if (ntx > 0xfffffffeull || nleaves > 0xffffffffull) return CV_E_TOO_LARGE;
    Opts o = ctx->opts();
    // shards of whole transactions: the leaf work per transaction (Σ blocks) decides, so a batch is cut by
    // leaves — transaction counts scaled so each device gets ~1/k of the leaves (C3: uniform)
    o.shard_min = std::max<size_t>(1, o.shard_min / 8);          // ~4,096 signatures' worth of transactions
    o.spread_min = std::max<size_t>(1, o.spread_min / 8);
    MerkleIn in{leaf_arena, leaf_off, leaf_len, tx_leaf_begin, ids, tx_status, arena_bytes};
    {
        std::lock_guard<std::mutex> g(ctx->st_mu);
        ctx->stats.merkle_calls++;
    }
    std::vector<Part> parts(ctx->devs.size(), Part{UINT64_MAX, 0, 0});
    const int rc = dispatch(ctx, o, ntx, 1, [&](Device &d, size_t t0, size_t t1, int threads) {
        if (t1 <= t0) return CV_OK;
        CV_TRY(hipSetDevice(d.ordinal));
        // small synchronous shards: one DMA, no pipeline frame.  Their records alone (12 B per leaf, 4 per
        // transaction) bound the staging from below, so a shard past kMerkleSmall by them skips the range scan
        // of its leaves (C3's 6M leaves: several ms on the synchronous call's critical path)
        const size_t nlv = (size_t)tx_leaf_begin[t1] - tx_leaf_begin[t0];
        if (!ticket && nlv * 12 + (t1 - t0) * 4 <= kMerkleSmall) {
            WorkerPool *pool = &d.workers(threads);
            const MStage st = mstage_plan(t0, t1, tx_leaf_begin, leaf_off, leaf_len, pool);
            if (!mstage_in_bounds(st, in.arena_bytes)) return CV_E_ARGS;   // past the arena, or off + len wraps
            if (st.total <= kMerkleSmall) return merkle_shard_small(d, st, in, pool);
        }
        int k = 0, r = CV_OK;
        std::unique_lock<std::mutex> lk;
        PipeOut &po = pipe_out(d, &k, lk);
        r = merkle_enqueue(ctx, d, o, po, t0, t1, in, threads);
        if (r != CV_OK) return r;
        if (ticket) {
            parts[dev_index(ctx, d)] = {(uint64_t)dev_index(ctx, d), (uint64_t)k, po.gen};
            po.ticketed = true;
            return CV_OK;
        }
        return pipe_finish(d, po);
    });
    std::vector<Part> live;
    for (const Part &p : parts)
        if (p[0] != UINT64_MAX) live.push_back(p);
    if (rc != CV_OK) {
        (void)parts_wait(ctx, live);
        return rc;
    }
    if (ticket) *ticket = live.empty() ? 0 : ticket_add(ctx, std::move(live));
    return CV_OK;
}

int cv_merkle_tx_ids_ex(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                        const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, uint8_t *ids, uint8_t *tx_status) {
    return merkle_call(ctx, ntx, leaf_arena, leaf_off, leaf_len, tx_leaf_begin, ids, tx_status, nullptr);
}

int cv_merkle_tx_ids_async(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                           const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, uint8_t *ids, uint8_t *tx_status,
                           uint64_t *ticket) {
    if (!ticket) return CV_E_ARGS;
    return merkle_call(ctx, ntx, leaf_arena, leaf_off, leaf_len, tx_leaf_begin, ids, tx_status, ticket);
}

int cv_merkle_tx_ids(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                     const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, uint8_t *ids) {
    return merkle_call(ctx, ntx, leaf_arena, leaf_off, leaf_len, tx_leaf_begin, ids, nullptr, nullptr);
}

int cv_merkle_tx_ids_bounded(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, uint64_t leaf_arena_bytes,
                             const uint64_t *leaf_off, const uint32_t *leaf_len, const uint32_t *tx_leaf_begin,
                             uint8_t *ids, uint8_t *tx_status, uint64_t *ticket) {
    return merkle_call(ctx, ntx, leaf_arena, leaf_off, leaf_len, tx_leaf_begin, ids, tx_status, ticket,
                       leaf_arena_bytes);
}

// One shard of a small synchronous transaction call (a notary's or a resolve chain's batch: staging up to
// kMerkleSmall bytes): leaves, keys, signatures and boundaries packed into slot 0's pinned staging (one DMA),
// then on one stream the Merkle kernels, the message references, the verify (a tri-chain or quad batch at
// notary sizes) and the per-transaction verdicts, and one result copy — the pipeline's per-call frame costs more
// than it hides at this size (fused 0.41 / 0.47 ms against 0.34 / 0.44 for the separate calls at 32 / 512
// transactions x 8 signers through the frame, profiles/r04m_txsmall.log).
static int txs_shard_small(Device &d, const Opts &o, const MStage &st, const TxIn &in, WorkerPool *pool) {
    const MerkleIn &mi = in.m;
    const size_t t0 = st.t0, nt = st.t1 - st.t0, nl = st.l1 - st.l0;
    const size_t s0 = in.tsb[t0], ns = in.tsb[st.t1] - s0, words = (ns + 63) / 64;
    // staging: the Merkle stage | pk | sig | boundaries
    const size_t o_pk = al16(st.total), o_sig = o_pk + al16(ns * 32), o_tsb = o_sig + al16(ns * 64);
    const size_t total = o_tsb + al16((nt + 1) * 4);
    // device results: ids | Merkle status | tx_ok | signature status (copied back as one block) | bitmap | off | len
    const size_t o_mst = al16(nt * 32), o_ok = o_mst + al16(nt), o_sst = o_ok + al16(nt);
    const size_t back = o_sst + (in.sig_status ? ns : 0), o_bm = al16(o_sst + ns), o_off = o_bm + al16(words * 8);
    const size_t o_len = o_off + al16(ns * 8), total_out = o_len + al16(ns * 4);
    Slot &sl = d.slot[0];
    hipStream_t s = nullptr;
    CV_TRY(slot_stream(d, 0, &s));
    CV_TRY(slot_events(sl));
    CV_TRY(sl.pin_in.ensure(total));
    CV_TRY(sl.packed.ensure(total));
    CV_TRY(d.pin_out.ensure(al16(back)));
    CV_TRY(d.ids.ensure(total_out));
    if (nl * 32 + 32 > sl.mdig.cap) {
        if (sl.last && sl.ev) CV_TRY(hipEventSynchronize(sl.ev));
        CV_TRY(sl.mdig.ensure(nl * 32 + 32));
    }
    uint8_t *h = sl.pin_in.as<uint8_t>(), *dv = sl.packed.as<uint8_t>(), *dout = d.ids.as<uint8_t>();
    auto drain = on_exit([s] { (void)hipStreamSynchronize(s); });   // error paths: no DMA outlives the call
    mstage_pack(st, h, mi.txb, mi.arena, mi.off, mi.len, pool);
    par_copy({{h + o_pk, in.pk + s0 * 32, ns * 32}, {h + o_sig, in.sig + s0 * 64, ns * 64},
              {h + o_tsb, in.tsb + t0, (nt + 1) * 4}}, pool);
    CV_TRY(hipMemcpyAsync(dv, h, total, hipMemcpyHostToDevice, s));
    const uint32_t *dtsb = reinterpret_cast<const uint32_t *>(dv + o_tsb);
    uint64_t *doff = reinterpret_cast<uint64_t *>(dout + o_off);
    uint32_t *dlen = reinterpret_cast<uint32_t *>(dout + o_len);
    uint64_t *dbm = reinterpret_cast<uint64_t *>(dout + o_bm);
    CV_TRY(ws_begin(d, sl, s));
    const hipError_t ek = cvk_merkle((uint32_t)nt, (uint32_t)nl, (uint32_t)st.l0, dv + st.o_ar - st.lo,
                                     reinterpret_cast<const uint64_t *>(dv + st.o_off),
                                     reinterpret_cast<const uint32_t *>(dv + st.o_len),
                                     reinterpret_cast<const uint32_t *>(dv + st.o_txb), sl.mdig.as<uint32_t>(), dout,
                                     dout + o_mst, s);
    const hipError_t e2 = ws_end(sl, s);
    CV_TRY(ek);
    CV_TRY(e2);
    if (ns) {
        CV_TRY(cvk_tx_sig_refs((uint32_t)ns, 0, (uint32_t)nt, (uint32_t)s0, dtsb, doff, dlen, s));
        CV_TRY(launch_verify(d, o.plan, sl, (uint32_t)ns, dv + o_pk, dv + o_sig, dout, doff, dlen, dbm,
                             in.sig_status ? dout + o_sst : nullptr, s, nullptr, false));
    }
    CV_TRY(cvk_tx_verdicts((uint32_t)nt, (uint32_t)s0, dtsb, dout + o_mst, dbm, dout + o_ok, s));
    CV_TRY(hipMemcpyAsync(d.pin_out.p, dout, back, hipMemcpyDeviceToHost, s));
    CV_TRY(hipStreamSynchronize(s));
    drain.armed = false;
    const uint8_t *r = d.pin_out.as<uint8_t>();
    std::memcpy(in.tx_ok + t0, r + o_ok, nt);
    if (mi.ids) std::memcpy(mi.ids + t0 * 32, r, nt * 32);
    if (mi.status) std::memcpy(mi.status + t0, r + o_mst, nt);
    if (in.sig_status && ns) std::memcpy(in.sig_status + s0, r + o_sst, ns);
    return CV_OK;
}

static int txs_call(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                    const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, const uint8_t *pk, const uint8_t *sig,
                    const uint32_t *tx_sig_begin, uint8_t *ids, uint8_t *tx_status, uint8_t *sig_status, uint8_t *tx_ok,
                    uint64_t *ticket, uint64_t arena_bytes = UINT64_MAX) {
    if (!ctx) return CV_E_ARGS;
    if (ticket) *ticket = 0;
    if (ntx == 0) return CV_OK;
    if (!tx_leaf_begin || !tx_sig_begin || !tx_ok) return CV_E_ARGS;
    if (tx_leaf_begin[0] != 0 || tx_sig_begin[0] != 0) return CV_E_ARGS;
    for (size_t t = 0; t < ntx; t++)
        if (tx_leaf_begin[t + 1] < tx_leaf_begin[t] || tx_sig_begin[t + 1] < tx_sig_begin[t]) return CV_E_ARGS;
    const size_t nleaves = tx_leaf_begin[ntx], nsig = tx_sig_begin[ntx];
    if (nleaves && (!leaf_off || !leaf_len)) return CV_E_ARGS;
    if (nsig && (!pk || !sig)) return CV_E_ARGS;
    if (ntx > 0xfffffffeull) return CV_E_TOO_LARGE;
    Opts o = ctx->opts();
    // shards of whole transactions, scaled as merkle_call's (~4,096 signatures' worth at C3's 8 per transaction)
    o.shard_min = std::max<size_t>(1, o.shard_min / 8);
    o.spread_min = std::max<size_t>(1, o.spread_min / 8);
    TxIn in{{leaf_arena, leaf_off, leaf_len, tx_leaf_begin, ids, tx_status, arena_bytes}, pk, sig, tx_sig_begin, sig_status,
            tx_ok, now_s()};
    {
        std::lock_guard<std::mutex> g(ctx->st_mu);
        ctx->stats.merkle_calls++;
    }
    std::vector<Part> parts(ctx->devs.size(), Part{UINT64_MAX, 0, 0});
    const int rc = dispatch(ctx, o, ntx, 1, [&](Device &d, size_t t0, size_t t1, int threads) {
        if (t1 <= t0) return CV_OK;
        CV_TRY(hipSetDevice(d.ordinal));
        // small synchronous shards: one DMA, one stream (the records alone bound the staging from below: a shard
        // past kMerkleSmall by them skips the range scan of its leaves, as merkle_call)
        const size_t nlv = (size_t)tx_leaf_begin[t1] - tx_leaf_begin[t0];
        const size_t ns = tx_sig_begin[t1] - tx_sig_begin[t0];
        if (!ticket && nlv * 12 + (t1 - t0) * 4 + ns * 96 <= kMerkleSmall) {
            WorkerPool *pool = &d.workers(threads);
            const MStage st = mstage_plan(t0, t1, tx_leaf_begin, leaf_off, leaf_len, pool);
            if (!mstage_in_bounds(st, in.m.arena_bytes)) return CV_E_ARGS;   // past the arena, or off + len wraps
            if (st.total + ns * 96 <= kMerkleSmall) return txs_shard_small(d, o, st, in, pool);
        }
        int k = 0, r = CV_OK;
        std::unique_lock<std::mutex> lk;
        PipeOut &po = pipe_out(d, &k, lk);
        r = txs_enqueue(ctx, d, o, po, t0, t1, in, threads, ticket != nullptr);
        if (r != CV_OK) return r;
        if (ticket) {
            parts[dev_index(ctx, d)] = {(uint64_t)dev_index(ctx, d), (uint64_t)k, po.gen};
            po.ticketed = true;
            return CV_OK;
        }
        const double ts = now_s();
        r = pipe_finish(d, po);
        std::lock_guard<std::mutex> g(ctx->st_mu);
        ctx->stats.pipe[4] += now_s() - ts;
        timeline_account(ctx, po);
        return r;
    });
    std::vector<Part> live;
    for (const Part &p : parts)
        if (p[0] != UINT64_MAX) live.push_back(p);
    if (rc != CV_OK) {
        (void)parts_wait(ctx, live);
        return rc;
    }
    if (ticket) *ticket = live.empty() ? 0 : ticket_add(ctx, std::move(live));
    return CV_OK;
}

int cv_verify_transactions(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                           const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, const uint8_t *pk, const uint8_t *sig,
                           const uint32_t *tx_sig_begin, uint8_t *ids, uint8_t *tx_status, uint8_t *sig_status,
                           uint8_t *tx_ok) {
    return txs_call(ctx, ntx, leaf_arena, leaf_off, leaf_len, tx_leaf_begin, pk, sig, tx_sig_begin, ids, tx_status,
                    sig_status, tx_ok, nullptr);
}

int cv_verify_transactions_async(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, const uint64_t *leaf_off,
                                 const uint32_t *leaf_len, const uint32_t *tx_leaf_begin, const uint8_t *pk,
                                 const uint8_t *sig, const uint32_t *tx_sig_begin, uint8_t *ids, uint8_t *tx_status,
                                 uint8_t *sig_status, uint8_t *tx_ok, uint64_t *ticket) {
    if (!ticket) return CV_E_ARGS;
    return txs_call(ctx, ntx, leaf_arena, leaf_off, leaf_len, tx_leaf_begin, pk, sig, tx_sig_begin, ids, tx_status,
                    sig_status, tx_ok, ticket);
}

int cv_verify_transactions_ex(cv_ctx *ctx, size_t ntx, const uint8_t *leaf_arena, uint64_t leaf_arena_bytes,
                              const uint64_t *leaf_off, const uint32_t *leaf_len, const uint32_t *tx_leaf_begin,
                              const uint8_t *pk, const uint8_t *sig, const uint32_t *tx_sig_begin, uint8_t *ids,
                              uint8_t *tx_status, uint8_t *sig_status, uint8_t *tx_ok, uint64_t *ticket) {
    return txs_call(ctx, ntx, leaf_arena, leaf_off, leaf_len, tx_leaf_begin, pk, sig, tx_sig_begin, ids, tx_status,
                    sig_status, tx_ok, ticket, leaf_arena_bytes);
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
    Opts o = ctx->opts();
    o.shard_min = o.spread_min = SIZE_MAX;   // one device, the least loaded (tear-off batches are small)
    return dispatch(ctx, o, ntrees, 1, [&](Device &d, size_t, size_t, int) {
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
        auto drain = on_exit([s] { (void)hipStreamSynchronize(s); });
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
        drain.armed = false;
        return CV_OK;
    });
}

int cv_tx_verdicts(size_t ntx, const uint64_t *bitmap, const uint32_t *tx_sig_begin, uint8_t *tx_ok) {
    if (ntx == 0) return CV_OK;
    if (!bitmap || !tx_sig_begin || !tx_ok) return CV_E_ARGS;
    // one masked word test per bitmap word the transaction's range touches
    for (size_t t = 0; t < ntx; t++) {
        const uint32_t b = tx_sig_begin[t], e = tx_sig_begin[t + 1];
        if (e < b) return CV_E_ARGS;
        bool ok = e > b;
        for (uint32_t w = b >> 6; ok && e > b && w <= (e - 1) >> 6; w++) {
            const uint32_t lo = w == (b >> 6) ? (b & 63) : 0, hi = w == ((e - 1) >> 6) ? ((e - 1) & 63) : 63;
            const uint64_t mask = (hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & ~((1ull << lo) - 1);
            ok = (bitmap[w] & mask) == mask;
        }
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
    const Opts o = ctx->opts();
    std::lock_guard<std::mutex> g(d->mu);              // enqueue only; ordered on the workspace (ws_begin)
    CV_TRY(hipSetDevice(d->ordinal));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : d->stream;
    CV_TRY(launch_verify(*d, o.plan, pick_slot(*d, s), (uint32_t)n, static_cast<const uint8_t *>(d_pk),
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
    const Opts o = ctx->opts();
    std::lock_guard<std::mutex> g(d->mu);
    CV_TRY(hipSetDevice(d->ordinal));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : d->stream;
    Slot &sl = pick_slot(*d, s);
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    hipError_t e = hipSuccess;
    for (int k = 0; k < 4 && e == hipSuccess; k++) e = hipEventCreate(&ev[k]);
    // one workspace chunk at a time (chunk starts are multiples of 64: whole bitmap words)
    for (size_t c0 = 0; c0 < n && e == hipSuccess; c0 += kVerifyChunk) {
        const size_t m = std::min<size_t>(kVerifyChunk, n - c0);
        e = launch_verify(*d, o.plan, sl, (uint32_t)m, static_cast<const uint8_t *>(d_pk) + c0 * 32,
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
    const Opts o = ctx->opts();
    std::lock_guard<std::mutex> g(d->mu);
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
    // device-API keyed calls also wait for the pool's previous user on another stream (their streams are the
    // caller's: an epoch reset can only wait for the last of them, so they stay a chain)
    if (e == hipSuccess && d->kc.last && d->kc.last != s) e = hipStreamWaitEvent(s, d->kc.ev, 0);
    std::vector<uint32_t> sok;
    bool prepared = false;
    int rc = e == hipSuccess ? key_resolve(*d, ctx->key_cap.load(), nkeys, hkeys.data(), nullptr, sok, s, &prepared) : hip_rc(e);
    KeyCache &kc = d->kc;
    // a slot_of_key that grows is freed: the previous keyed call still queued on the pool reads it
    if (rc == CV_OK && nkeys * 4 > kc.slot_of_key.cap) rc = hip_rc(pool_quiesce(*d));
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
        rc = hip_rc(cvk_verify_keyed(&o.plan, (uint32_t)n, static_cast<const uint8_t *>(d_keys),
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
    std::lock_guard<std::mutex> g(d->mu);
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
    std::lock_guard<std::mutex> g(d->mu);
    CV_TRY(hipSetDevice(d->ordinal));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : d->stream;
    CV_TRY(cvk_merkle((uint32_t)ntx, (uint32_t)nleaves, 0, static_cast<const uint8_t *>(d_arena),
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
// scoped device scratch and events of the calibration calls (freed on every return path)
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
    std::lock_guard<std::mutex> g(d->mu);
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
    std::lock_guard<std::mutex> g(d->mu);
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

}  // extern "C"
