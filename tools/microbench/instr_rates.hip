// instr_rates.hip — per-instruction VALU issue rates on gfx950 (calibrates the verify kernel's
// cost model: which 32x32->64 multiply form and which carry idioms are cheapest).
//   hipcc --offload-arch=gfx950 -O3 instr_rates.hip -o instr_rates && ./instr_rates
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAINS 8
#define UNROLL 16

#define BENCH(NAME, ASM, CONSTR_OUT, CONSTR_IN)                                                  \
    __global__ void NAME(int iters, unsigned long long *out) {                                   \
        unsigned long long acc[CHAINS];                                                          \
        unsigned a[CHAINS], b[CHAINS];                                                           \
        for (int k = 0; k < CHAINS; k++) {                                                       \
            acc[k] = threadIdx.x + k;                                                            \
            a[k] = threadIdx.x * 2654435761u + k;                                                \
            b[k] = blockIdx.x * 40503u + 7 * k + 1;                                              \
        }                                                                                        \
        for (int it = 0; it < iters; it++) {                                                     \
            _Pragma("unroll") for (int r = 0; r < UNROLL; r++) {                                 \
                _Pragma("unroll") for (int k = 0; k < CHAINS; k++) {                             \
                    asm volatile(ASM : CONSTR_OUT(acc[k]) : CONSTR_IN(a[k]), "v"(b[(k + r) & 7]) : "vcc"); \
                }                                                                                \
            }                                                                                    \
        }                                                                                        \
        unsigned long long s = 0;                                                                \
        for (int k = 0; k < CHAINS; k++) s ^= acc[k];                                            \
        if (s == 0x1234567ull) out[0] = s;                                                       \
    }

#define OUT64 "+v"
#define IN32 "v"
BENCH(k_mad_i64_i32, "v_mad_i64_i32 %0, vcc, %1, %2, %0", OUT64, IN32)
BENCH(k_mad_u64_u32, "v_mad_u64_u32 %0, vcc, %1, %2, %0", OUT64, IN32)
BENCH(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 1, %0", OUT64, IN32)
BENCH(k_ashr_i64, "v_ashrrev_i64 %0, 7, %0", OUT64, IN32)

// 32-bit ops: use acc low word
#define BENCH32(NAME, ASM)                                                                       \
    __global__ void NAME(int iters, unsigned long long *out) {                                   \
        unsigned acc[CHAINS], b[CHAINS];                                                         \
        for (int k = 0; k < CHAINS; k++) { acc[k] = threadIdx.x + k; b[k] = blockIdx.x * 40503u + 7 * k + 1; } \
        for (int it = 0; it < iters; it++) {                                                     \
            _Pragma("unroll") for (int r = 0; r < UNROLL; r++) {                                 \
                _Pragma("unroll") for (int k = 0; k < CHAINS; k++) {                             \
                    asm volatile(ASM : "+v"(acc[k]) : "v"(b[(k + r) & 7]));                      \
                }                                                                                \
            }                                                                                    \
        }                                                                                        \
        unsigned s = 0;                                                                          \
        for (int k = 0; k < CHAINS; k++) s ^= acc[k];                                            \
        if (s == 0x1234567u) out[0] = s;                                                         \
    }
BENCH32(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
BENCH32(k_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
BENCH32(k_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %0")
BENCH32(k_mul_hi_u32_u24, "v_mul_hi_u32_u24 %0, %0, %1")
BENCH32(k_add_u32, "v_add_u32 %0, %0, %1")
BENCH32(k_lshl_add_u32, "v_lshl_add_u32 %0, %0, 4, %1")
BENCH32(k_dot2_u32_u16, "v_dot2_u32_u16 %0, %0, %1, %0")
BENCH32(k_pk_mad_u16, "v_pk_mad_u16 %0, %0, %1, %0")

typedef void (*kfn)(int, unsigned long long *);

int main() {
    struct { const char *name; kfn f; } ks[] = {
        {"v_mad_i64_i32", k_mad_i64_i32}, {"v_mad_u64_u32", k_mad_u64_u32}, {"v_lshl_add_u64", k_lshl_add_u64},
        {"v_ashrrev_i64", k_ashr_i64}, {"v_mul_lo_u32", k_mul_lo_u32},
        {"v_mul_hi_u32", k_mul_hi_u32}, {"v_mad_u32_u24", k_mad_u32_u24}, {"v_mul_hi_u32_u24", k_mul_hi_u32_u24},
        {"v_add_u32", k_add_u32}, {"v_lshl_add_u32", k_lshl_add_u32}, {"v_dot2_u32_u16", k_dot2_u32_u16},
        {"v_pk_mad_u16", k_pk_mad_u16},
    };
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int blocks = cus * 8, threads = 256, iters = 4000;
    unsigned long long *out;
    hipMalloc(&out, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("CUs %d clock(kHz) %d\n", cus, prop.clockRate);
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, iters / 8, out);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, iters, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double ops = (double)iters * UNROLL * CHAINS * blocks * threads;
        double rate = ops / (ms * 1e-3);
        // wave-instructions per SIMD per cycle at the nominal clock
        double per_simd_cycle = rate / 64.0 / (cus * 4.0) / (prop.clockRate * 1e3);
        printf("%-18s %8.2f Tops/s  %.3f wave-instr/SIMD/clk  (%.2f clk per wave-instr)\n", k.name, rate / 1e12,
               per_simd_cycle, 1.0 / per_simd_cycle);
    }
    return 0;
}
