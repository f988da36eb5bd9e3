// lat_parts.hip — where the notary-batch (tri form) kernel chain spends its time: the fused latency prep
// split into its roles and their parts (SHA-512 + mod L + effective S | lattice + digits | point decode |
// decode + tables), and the tri-chain Straus kernel, each timed alone with HIP events (median of reps) on
// honest signatures over 32-byte messages, as a notary batch has them.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-sched-strategy=max-ilp \
//         -I corda_amd/csrc tools/microbench/lat_parts.hip -o lat_parts && ./lat_parts [n ...]
#include "../../corda_amd/csrc/cv_k_lat.hip"
#include "../../corda_amd/csrc/cv_k_misc.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            std::exit(1);                                                                        \
        }                                                                                        \
    } while (0)

__global__ __launch_bounds__(64, 1) void k_empty(uint32_t n, uint32_t *out) {
    if (blockIdx.x * 64 + threadIdx.x == n) out[0] = 1;
}

// SHA-512(R || Abyte || M) mod L and the effective S
__global__ __launch_bounds__(64, 1) void k_hash(uint32_t n, const uint8_t *pk, const uint8_t *sig, const uint8_t *arena,
                                                const uint64_t *off, const uint32_t *len, uint32_t *hs_out) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    uint32_t aw[8], rw[8], sw[8], hs[CV_HS_WORDS];
    load_words8(aw, pk + (size_t)i * 32);
    load_words8(rw, sig + (size_t)i * 64);
    load_words8(sw, sig + (size_t)i * 64 + 32);
    cv_keyed_hs(aw, rw, sw, arena + off[i], len[i], hs);
    store_words(hs_out + (size_t)i * CV_HS_WORDS, hs, CV_HS_WORDS / 4);
}

// the lattice reduction and the tri form's digit words, from stored h || s
__global__ __launch_bounds__(64, 1) void k_lattice(uint32_t n, uint32_t cap, const uint32_t *hs_in, uint32_t *dig) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    uint32_t hs[CV_HS_WORDS];
#pragma unroll
    for (int q = 0; q < CV_HS_WORDS; q++) hs[q] = hs_in[(size_t)i * CV_HS_WORDS + q];
    cv_hs_scalars<true, false>(hs, dig + i, cap);
}

// the whole scalars role of the fused prep
__global__ __launch_bounds__(64, 1) void k_scalars(uint32_t n, uint32_t cap, const uint8_t *pk, const uint8_t *sig,
                                                   const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                                                   uint32_t *dig) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i < n) cv_scalars_lane<true, false>(i, cap, pk, sig, arena, off, len, dig);
}

// one point decode per lane (lane pairs: A, R), no table
__global__ __launch_bounds__(64, 1) void k_decode(uint32_t n, const uint8_t *pk, const uint8_t *sig, uint32_t *out) {
    const uint32_t g = blockIdx.x * 64 + threadIdx.x;
    const uint32_t i = g >> 1;
    if (i >= n) return;
    const bool is_r = (g & 1u) != 0;
    uint32_t w[8];
    load_words8(w, is_r ? sig + (size_t)i * 64 : pk + (size_t)i * 32);
    ge_p3 P;
    const bool ok = ge_decode_0_1_0<false>(P, w);
    uint32_t t[10];
    fe_store(t, P.X);
    out[g] = t[0] ^ t[9] ^ (ok ? 1u : 0u);
}

// the whole points role (four lanes per signature, as the tri form's prep)
__global__ __launch_bounds__(64, 1) void k_points(uint32_t n, const uint8_t *pk, const uint8_t *sig, uint32_t *tab,
                                                  uint32_t *tabR, uint8_t *ok, uint8_t *status) {
    cv_points_quad_lane<false>(blockIdx.x * 64 + threadIdx.x, n, pk, sig, tab, tabR, ok, status);
}

// one lane per signature, the prep's parts back to back with s_memrealtime stamps (100 MHz): SHA-512 + mod L
// + effective S | lattice (sc_halfsize) | window digit words | decode of A | its odd-multiple table
__global__ __launch_bounds__(64, 1) void k_clk(uint32_t n, uint32_t cap, const uint8_t *pk, const uint8_t *sig,
                                               const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                                               uint32_t *dig, uint32_t *tab, uint64_t *stamps) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    uint64_t t[6];
    uint32_t aw[8], rw[8], sw[8], hs[CV_HS_WORDS];
    load_words8(aw, pk + (size_t)i * 32);
    load_words8(rw, sig + (size_t)i * 64);
    load_words8(sw, sig + (size_t)i * 64 + 32);
    t[0] = __builtin_amdgcn_s_memrealtime();
    cv_keyed_hs(aw, rw, sw, arena + off[i], len[i], hs);
    asm volatile("" ::"v"(hs[0]), "v"(hs[15]));
    t[1] = __builtin_amdgcn_s_memrealtime();
    uint32_t u[8], v[8], w[8];
    bool v_neg;
    int nwin;
    sc_halfsize(u, v, v_neg, nwin, w, hs, hs + 8);
    asm volatile("" ::"v"(u[0]), "v"(v[0]), "v"(w[0]));
    t[2] = __builtin_amdgcn_s_memrealtime();
#pragma unroll 4
    for (int win = 0; win < 64; win++) {
        const int da = -digit16(u, win), dr = v_neg ? -digit16(v, win) : digit16(v, win);
        const int dlo = win < 32 ? digit16(w, win) : 0, dhi = win < 32 ? digit16(w, 32 + win) : 0;
        dig[(size_t)win * cap + i] = ((uint32_t)da & 0x1fu) | (((uint32_t)dr & 0x1fu) << 5) |
                                     (((uint32_t)dlo & 0x1fu) << 10) | (((uint32_t)dhi & 0x1fu) << 15);
    }
    t[3] = __builtin_amdgcn_s_memrealtime();
    ge_p3 P;
    const bool ok = ge_decode_0_1_0<false>(P, aw);
    asm volatile("" ::"v"(P.X.v[0]), "v"(P.T.v[9]));
    t[4] = __builtin_amdgcn_s_memrealtime();
    ge_cached_multiples8_half(tab + (size_t)i * CV_TAB_WORDS, P, ok);
    t[5] = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < 5; k++) stamps[(size_t)i * 5 + k] = t[k + 1] - t[k];
}

template <typename F> static float time_ms(F launch, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int r = 0; r < reps + 3; r++) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 3) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
    std::vector<uint32_t> sizes;
    for (int a = 1; a < argc; a++) sizes.push_back((uint32_t)std::atoi(argv[a]));
    if (sizes.empty()) sizes = {256, 4096};
    const int reps = 40;
    for (uint32_t n : sizes) {
        const uint32_t cap = n;
        std::vector<uint8_t> seed(32 * (size_t)n), msg(32 * (size_t)n + 16, 0);
        std::vector<uint64_t> off(n);
        std::vector<uint32_t> len(n, 32);
        uint64_t x = 0x243F6A8885A308D3ull + n;
        for (auto &c : seed) { x = x * 6364136223846793005ull + 1442695040888963407ull; c = (uint8_t)(x >> 56); }
        for (size_t j = 0; j < 32 * (size_t)n; j++) { x = x * 6364136223846793005ull + 1; msg[j] = (uint8_t)(x >> 56); }
        for (uint32_t i = 0; i < n; i++) off[i] = 32ull * i;
        uint8_t *d_seed, *d_msg, *d_pk, *d_sig, *d_ok, *d_status;
        uint64_t *d_off, *d_bm;
        uint32_t *d_len, *d_hs, *d_dig, *d_tab, *d_tabR, *d_out;
        CK(hipMalloc(&d_seed, seed.size()));
        CK(hipMalloc(&d_msg, msg.size()));
        CK(hipMalloc(&d_pk, 32 * (size_t)n));
        CK(hipMalloc(&d_sig, 64 * (size_t)n));
        CK(hipMalloc(&d_ok, n));
        CK(hipMalloc(&d_status, n));
        CK(hipMalloc(&d_off, 8 * (size_t)n));
        CK(hipMalloc(&d_bm, 8 * (size_t)((n + 63) / 64)));
        CK(hipMalloc(&d_len, 4 * (size_t)n));
        CK(hipMalloc(&d_hs, 4 * (size_t)CV_HS_WORDS * n));
        CK(hipMalloc(&d_dig, 4 * (size_t)CV_HS_DIGWORDS * n));
        CK(hipMalloc(&d_tab, 4 * (size_t)CV_TAB_WORDS * n));
        CK(hipMalloc(&d_tabR, 4 * (size_t)CV_TAB_WORDS * n));
        CK(hipMalloc(&d_out, 8 * (size_t)n));
        CK(hipMemcpy(d_seed, seed.data(), seed.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(d_msg, msg.data(), msg.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(d_off, off.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_len, len.data(), 4 * (size_t)n, hipMemcpyHostToDevice));
        cv_sign_kernel<<<(n + CV_BLOCK - 1) / CV_BLOCK, CV_BLOCK>>>(n, d_seed, d_msg, d_off, d_len, d_pk, d_sig);
        CK(hipDeviceSynchronize());
        const uint32_t g1 = (n + 63) / 64, g2 = (2 * n + 63) / 64, g4 = (4 * n + 63) / 64;
        const float t_empty = time_ms([&] { k_empty<<<g1, 64>>>(n, d_out); }, reps);
        const float t_hash = time_ms([&] { k_hash<<<g1, 64>>>(n, d_pk, d_sig, d_msg, d_off, d_len, d_hs); }, reps);
        const float t_lat = time_ms([&] { k_lattice<<<g1, 64>>>(n, cap, d_hs, d_dig); }, reps);
        const float t_sc = time_ms([&] { k_scalars<<<g1, 64>>>(n, cap, d_pk, d_sig, d_msg, d_off, d_len, d_dig); }, reps);
        const float t_dec = time_ms([&] { k_decode<<<g2, 64>>>(n, d_pk, d_sig, d_out); }, reps);
        const float t_pts = time_ms([&] { k_points<<<g4, 64>>>(n, d_pk, d_sig, d_tab, d_tabR, d_ok, d_status); }, reps);
        const float t_prep = time_ms([&] {
            cv_prep_lat_kernel<true, false><<<g4 + g1, 64>>>(n, cap, g4, 1, d_pk, d_sig, d_msg, d_off, d_len, d_dig,
                                                             d_tab, d_tabR, d_ok, d_status, d_bm);
        }, reps);
        const float t_tri = time_ms([&] {
            cv_hs_straus_tri_kernel<true><<<(16 * n + CV_BLOCK - 1) / CV_BLOCK, CV_BLOCK>>>(n, cap, d_dig, d_tab, d_tabR,
                                                                                         d_ok, d_bm, nullptr);
        }, reps);
        const float t_chain = time_ms([&] {
            cv_prep_lat_kernel<true, false><<<g4 + g1, 64>>>(n, cap, g4, 1, d_pk, d_sig, d_msg, d_off, d_len, d_dig,
                                                             d_tab, d_tabR, d_ok, d_status, d_bm);
            cv_hs_straus_tri_kernel<true><<<(16 * n + CV_BLOCK - 1) / CV_BLOCK, CV_BLOCK>>>(n, cap, d_dig, d_tab, d_tabR,
                                                                                         d_ok, d_bm, nullptr);
        }, reps);
        uint64_t *d_st;
        CK(hipMalloc(&d_st, 8 * 5 * (size_t)n));
        k_clk<<<g1, 64>>>(n, cap, d_pk, d_sig, d_msg, d_off, d_len, d_dig, d_tab, d_st);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> st(5 * (size_t)n);
        CK(hipMemcpy(st.data(), d_st, 8 * st.size(), hipMemcpyDeviceToHost));
        CK(hipFree(d_st));
        double part[5];
        for (int k = 0; k < 5; k++) {
            std::vector<uint64_t> col(n);
            for (uint32_t i = 0; i < n; i++) col[i] = st[5 * (size_t)i + k];
            std::sort(col.begin(), col.end());
            part[k] = col[n / 2] * 0.01;   // 100 MHz ticks -> us
        }
        std::printf("{\"n\": %u, \"lane_us_median\": {\"hash\": %.1f, \"halfsize\": %.1f, \"digits\": %.1f, "
                    "\"decode\": %.1f, \"table_half\": %.1f}}\n", n, part[0], part[1], part[2], part[3], part[4]);
        std::vector<uint64_t> bm((n + 63) / 64);
        CK(hipMemcpy(bm.data(), d_bm, 8 * bm.size(), hipMemcpyDeviceToHost));
        uint32_t acc = 0;
        for (uint32_t i = 0; i < n; i++) acc += (uint32_t)((bm[i / 64] >> (i % 64)) & 1u);
        std::printf("{\"n\": %u, \"accepted\": %u, \"us\": {\"empty\": %.1f, \"hash\": %.1f, \"lattice\": %.1f, "
                    "\"scalars\": %.1f, \"decode\": %.1f, \"points\": %.1f, \"prep\": %.1f, \"tri\": %.1f, \"prep+tri\": %.1f}}\n",
                    n, acc, 1e3 * t_empty, 1e3 * t_hash, 1e3 * t_lat, 1e3 * t_sc, 1e3 * t_dec, 1e3 * t_pts,
                    1e3 * t_prep, 1e3 * t_tri, 1e3 * t_chain);
        for (void *p : {(void *)d_seed, (void *)d_msg, (void *)d_pk, (void *)d_sig, (void *)d_ok, (void *)d_status,
                        (void *)d_off, (void *)d_bm, (void *)d_len, (void *)d_hs, (void *)d_dig, (void *)d_tab,
                        (void *)d_tabR, (void *)d_out})
            CK(hipFree(p));
    }
    return 0;
}
