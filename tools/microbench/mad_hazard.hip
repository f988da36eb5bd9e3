// mad_hazard.hip — is a dependent v_mad_u64_u32 read at distance 1 / 2 / 3 (no s_nop between) exact
// on gfx950, and what does each spacing cost?  LLVM pads some distance-1/2 accumulator reads with
// "s_nop 0"; this checks the hardware result against the host for every spacing, then times them.
//   hipcc --offload-arch=gfx950 -O3 mad_hazard.hip -o mad_hazard && ./mad_hazard
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define NL 10

// D = number of independent accumulators interleaved inside ONE asm block (distance D between a
// chain's dependent mads).  Each chain m accumulates sum_k a[k] * b[(k + m) % NL].
template <int D> __device__ __forceinline__ void chains(uint64_t (&t)[4], const uint32_t (&a)[NL], const uint32_t (&b)[NL]) {
#pragma unroll
    for (int k = 0; k < NL; k++) {
        if constexpr (D == 1) {
            asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(t[0]) : "v"(a[k]), "v"(b[k]) : "vcc");
        } else if constexpr (D == 2) {
            asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_mad_u64_u32 %1, vcc, %2, %4, %1"
                         : "+v"(t[0]), "+v"(t[1]) : "v"(a[k]), "v"(b[k]), "v"(b[(k + 1) % NL]) : "vcc");
        } else if constexpr (D == 3) {
            asm volatile("v_mad_u64_u32 %0, vcc, %3, %4, %0\n\tv_mad_u64_u32 %1, vcc, %3, %5, %1\n\t"
                         "v_mad_u64_u32 %2, vcc, %3, %6, %2"
                         : "+v"(t[0]), "+v"(t[1]), "+v"(t[2])
                         : "v"(a[k]), "v"(b[k]), "v"(b[(k + 1) % NL]), "v"(b[(k + 2) % NL]) : "vcc");
        } else {
            asm volatile("v_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_mad_u64_u32 %1, vcc, %4, %6, %1\n\t"
                         "v_mad_u64_u32 %2, vcc, %4, %7, %2\n\tv_mad_u64_u32 %3, vcc, %4, %8, %3"
                         : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3])
                         : "v"(a[k]), "v"(b[k]), "v"(b[(k + 1) % NL]), "v"(b[(k + 2) % NL]), "v"(b[(k + 3) % NL])
                         : "vcc");
        }
    }
}

// whole chains in ONE asm block: distance-1 dependent mads, 10 in a row (worst case)
__device__ __forceinline__ void chain1_block(uint64_t &t, const uint32_t (&a)[NL], const uint32_t (&b)[NL]) {
    asm volatile(
        "v_mad_u64_u32 %0, vcc, %1, %11, %0\n\tv_mad_u64_u32 %0, vcc, %2, %12, %0\n\t"
        "v_mad_u64_u32 %0, vcc, %3, %13, %0\n\tv_mad_u64_u32 %0, vcc, %4, %14, %0\n\t"
        "v_mad_u64_u32 %0, vcc, %5, %15, %0\n\tv_mad_u64_u32 %0, vcc, %6, %16, %0\n\t"
        "v_mad_u64_u32 %0, vcc, %7, %17, %0\n\tv_mad_u64_u32 %0, vcc, %8, %18, %0\n\t"
        "v_mad_u64_u32 %0, vcc, %9, %19, %0\n\tv_mad_u64_u32 %0, vcc, %10, %20, %0"
        : "+v"(t)
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]), "v"(a[9]),
          "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]), "v"(b[8]), "v"(b[9])
        : "vcc");
}

template <int D>
__global__ void k_check(int n, const uint32_t *A, const uint32_t *B, uint64_t *O) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t a[NL], b[NL];
    for (int k = 0; k < NL; k++) { a[k] = A[i * NL + k]; b[k] = B[i * NL + k]; }
    uint64_t t[4] = {1, 2, 3, 4};
    if constexpr (D == 0) chain1_block(t[0], a, b);
    else chains<D>(t, a, b);
    for (int m = 0; m < 4; m++) O[(size_t)i * 4 + m] = t[m];
}

template <int D>
__global__ void k_time(int iters, uint64_t *out) {
    uint32_t a[NL], b[NL];
    for (int k = 0; k < NL; k++) { a[k] = threadIdx.x * 2654435761u + k; b[k] = blockIdx.x * 40503u + 7 * k; }
    uint64_t t[4] = {1, 2, 3, 4};
    uint64_t u[4] = {5, 6, 7, 8};
    for (int it = 0; it < iters; it++) {
        if constexpr (D == 0) { chain1_block(t[0], a, b); chain1_block(u[0], a, b); }
        else { chains<D>(t, a, b); chains<D>(u, a, b); }
    }
    uint64_t s = t[0] ^ t[1] ^ t[2] ^ t[3] ^ u[0] ^ u[1] ^ u[2] ^ u[3];
    if (s == 0x1234567ull) out[0] = s;
}

int main() {
    const int n = 1 << 20;
    std::vector<uint32_t> A(n * NL), B(n * NL);
    uint64_t x = 88172645463325252ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (uint32_t)x; };
    for (auto &v : A) v = rnd();
    for (auto &v : B) v = rnd();
    uint32_t *dA, *dB;
    uint64_t *dO;
    (void)hipMalloc(&dA, A.size() * 4);
    (void)hipMalloc(&dB, B.size() * 4);
    (void)hipMalloc(&dO, (size_t)n * 32);
    (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    std::vector<uint64_t> O((size_t)n * 4);
    int bad_total = 0;
    for (int D = 0; D <= 4; D++) {
        (void)hipMemset(dO, 0, (size_t)n * 32);
        switch (D) {
            case 0: hipLaunchKernelGGL(k_check<0>, dim3(n / 256), dim3(256), 0, 0, n, dA, dB, dO); break;
            case 1: hipLaunchKernelGGL(k_check<1>, dim3(n / 256), dim3(256), 0, 0, n, dA, dB, dO); break;
            case 2: hipLaunchKernelGGL(k_check<2>, dim3(n / 256), dim3(256), 0, 0, n, dA, dB, dO); break;
            case 3: hipLaunchKernelGGL(k_check<3>, dim3(n / 256), dim3(256), 0, 0, n, dA, dB, dO); break;
            case 4: hipLaunchKernelGGL(k_check<4>, dim3(n / 256), dim3(256), 0, 0, n, dA, dB, dO); break;
        }
        (void)hipMemcpy(O.data(), dO, (size_t)n * 32, hipMemcpyDeviceToHost);
        const int nch = D == 0 ? 1 : D;
        long bad = 0;
        for (int i = 0; i < n; i++) {
            for (int m = 0; m < nch; m++) {
                uint64_t t = (uint64_t)(m + 1);
                for (int k = 0; k < NL; k++) t += (uint64_t)A[i * NL + k] * B[i * NL + (k + m) % NL];
                if (O[(size_t)i * 4 + m] != t) bad++;
            }
        }
        printf("spacing %s: %ld mismatches of %ld\n", D == 0 ? "1 (one asm block)" : (D == 1 ? "1 (asm per mad)" : D == 2 ? "2" : D == 3 ? "3" : "4"),
               bad, (long)n * nch);
        bad_total += bad != 0;
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    for (int wv = 2; wv <= 4; wv++) {
        for (int D = 0; D <= 4; D++) {
            const int blocks = prop.multiProcessorCount * wv, iters = 4000;
            auto launch = [&](int it) {
                switch (D) {
                    case 0: hipLaunchKernelGGL(k_time<0>, dim3(blocks), dim3(256), 0, 0, it, dO); break;
                    case 1: hipLaunchKernelGGL(k_time<1>, dim3(blocks), dim3(256), 0, 0, it, dO); break;
                    case 2: hipLaunchKernelGGL(k_time<2>, dim3(blocks), dim3(256), 0, 0, it, dO); break;
                    case 3: hipLaunchKernelGGL(k_time<3>, dim3(blocks), dim3(256), 0, 0, it, dO); break;
                    case 4: hipLaunchKernelGGL(k_time<4>, dim3(blocks), dim3(256), 0, 0, it, dO); break;
                }
            };
            launch(iters / 8);
            (void)hipEventRecord(e0);
            launch(iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const int nch = D == 0 ? 1 : D;
            const double mads = (double)iters * 2 * NL * nch * blocks * 256;
            printf("waves/SIMD %d spacing-variant %d: %.3f ms, %.2f Tmad/s\n", wv, D, ms, mads / (ms * 1e-3) / 1e12);
        }
    }
    return bad_total;
}
