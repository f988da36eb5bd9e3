// cv_api.cpp — the C-ABI (include/cordaverify.h): contexts, per-device workspaces, host-buffer
// batches sharded over the context's GPUs (one host thread + one HIP stream per device), and the
// device-resident entry points used by bench.py.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/cordaverify.h"

extern "C" {
hipError_t cvk_verify(uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena, const uint64_t *off,
                      const uint32_t *len, uint64_t *bitmap, uint8_t *status, uint32_t *ws_hs, uint32_t *ws_tab,
                      uint32_t *ws_R, uint8_t *ws_ok, uint32_t ws_cap, hipStream_t stream, hipEvent_t *ev);
hipError_t cvk_sign(uint32_t n, const uint8_t *seed, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                    uint8_t *pk, uint8_t *sig, hipStream_t stream);
hipError_t cvk_merkle(uint32_t ntx, uint32_t nleaves, const uint8_t *arena, const uint64_t *leaf_off,
                      const uint32_t *leaf_len, const uint32_t *tx_begin, uint32_t *leaf_digest, uint8_t *ids,
                      uint8_t *status, hipStream_t stream);
hipError_t cvk_calibrate(uint32_t iters, int which, uint32_t blocks, void *scratch, hipStream_t stream);
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

struct Device {
    int ordinal = 0;
    hipStream_t stream = nullptr;
    DevBuf pk, sig, arena, off, len, bitmap, status, seed, tx_begin, digest, ids;
    DevBuf ws_hs, ws_tab, ws_R, ws_ok;   // verify workspace (hs 64 B + tab 1280 B + R 128 B + ok 1 B per signature)
    uint32_t ws_cap = 0;
};

// Verify workspace capacity: batches above it run in chunks of this many signatures.
constexpr uint32_t kVerifyChunk = 1u << 21;

hipError_t ensure_verify_ws(Device &d, size_t n) {
    uint32_t want = (uint32_t)std::min<size_t>(kVerifyChunk, (n + 511) / 512 * 512);
    if (want <= d.ws_cap) return hipSuccess;
    hipError_t e;
    if ((e = d.ws_hs.ensure((size_t)want * 64)) != hipSuccess) return e;
    if ((e = d.ws_tab.ensure((size_t)want * 1280)) != hipSuccess) return e;
    if ((e = d.ws_R.ensure((size_t)want * 128)) != hipSuccess) return e;
    if ((e = d.ws_ok.ensure((size_t)want)) != hipSuccess) return e;
    d.ws_cap = want;
    return hipSuccess;
}

hipError_t launch_verify(Device &d, uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                         const uint64_t *off, const uint32_t *len, uint64_t *bitmap, uint8_t *status, hipStream_t s,
                         hipEvent_t *ev = nullptr) {
    hipError_t e = ensure_verify_ws(d, n);
    if (e != hipSuccess) return e;
    return cvk_verify(n, pk, sig, arena, off, len, bitmap, status, d.ws_hs.as<uint32_t>(), d.ws_tab.as<uint32_t>(),
                      d.ws_R.as<uint32_t>(), d.ws_ok.as<uint8_t>(), d.ws_cap, s, ev);
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

int cv_open(uint32_t device_mask, cv_ctx **out) {
    if (!out) return CV_E_ARGS;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return CV_E_NO_DEVICE;
    cv_ctx *ctx = new (std::nothrow) cv_ctx();
    if (!ctx) return CV_E_OOM;
    for (int d = 0; d < count && d < 32; d++) {
        if (device_mask && !(device_mask & (1u << d))) continue;
        Device dev;
        dev.ordinal = d;
        if (hipSetDevice(d) != hipSuccess || hipStreamCreateWithFlags(&dev.stream, hipStreamNonBlocking) != hipSuccess) {
            cv_close(ctx);
            return CV_E_HIP;
        }
        ctx->devs.push_back(dev);
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
                          &d.digest, &d.ids, &d.ws_hs, &d.ws_tab, &d.ws_R, &d.ws_ok})
            b->release();
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
// are whole words of the caller's bitmap.
static int verify_shard(Device &d, size_t b, size_t e, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                        const uint64_t *off, const uint32_t *len, uint64_t *bitmap, uint8_t *status) {
    const size_t n = e - b;
    if (n == 0) return CV_OK;
    if (n > 0xffffffffull) return CV_E_TOO_LARGE;
    CV_TRY(hipSetDevice(d.ordinal));
    // arena sub-range used by this shard; offsets are rebased by passing (d_arena - lo)
    uint64_t lo = UINT64_MAX, hi = 0;
    for (size_t i = b; i < e; i++) {
        lo = std::min<uint64_t>(lo, off[i]);
        hi = std::max<uint64_t>(hi, off[i] + len[i]);
    }
    if (hi < lo) hi = lo;
    const size_t words = (n + 63) / 64;
    CV_TRY(d.pk.ensure(n * 32));
    CV_TRY(d.sig.ensure(n * 64));
    CV_TRY(d.arena.ensure(hi - lo + 16));
    CV_TRY(d.off.ensure(n * 8));
    CV_TRY(d.len.ensure(n * 4));
    CV_TRY(d.bitmap.ensure(words * 8));
    CV_TRY(d.status.ensure(n));
    hipStream_t s = d.stream;
    CV_TRY(hipMemcpyAsync(d.pk.p, pk + b * 32, n * 32, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(d.sig.p, sig + b * 64, n * 64, hipMemcpyHostToDevice, s));
    if (hi > lo) CV_TRY(hipMemcpyAsync(d.arena.p, arena + lo, hi - lo, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(d.off.p, off + b, n * 8, hipMemcpyHostToDevice, s));
    CV_TRY(hipMemcpyAsync(d.len.p, len + b, n * 4, hipMemcpyHostToDevice, s));
    CV_TRY(launch_verify(d, (uint32_t)n, d.pk.as<uint8_t>(), d.sig.as<uint8_t>(), d.arena.as<uint8_t>() - lo,
                         d.off.as<uint64_t>(), d.len.as<uint32_t>(), d.bitmap.as<uint64_t>(),
                         status ? d.status.as<uint8_t>() : nullptr, s));
    CV_TRY(hipMemcpyAsync(bitmap + b / 64, d.bitmap.p, words * 8, hipMemcpyDeviceToHost, s));
    if (status) CV_TRY(hipMemcpyAsync(status + b, d.status.p, n, hipMemcpyDeviceToHost, s));
    CV_TRY(hipStreamSynchronize(s));
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

extern "C" {

int cv_ed25519_verify_batch(cv_ctx *ctx, size_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *msg_arena,
                            const uint64_t *msg_off, const uint32_t *msg_len, uint64_t *verdict_bitmap,
                            uint8_t *status) {
    if (!ctx) return CV_E_ARGS;
    if (n == 0) return CV_OK;
    if (!pk || !sig || !msg_off || !msg_len || !verdict_bitmap) return CV_E_ARGS;
    std::lock_guard<std::mutex> g(ctx->mu);
    return for_each_shard(ctx, n, [&](Device &d, size_t b, size_t e) {
        return verify_shard(d, b, e, pk, sig, msg_arena, msg_off, msg_len, verdict_bitmap, status);
    });
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

}  // extern "C"
