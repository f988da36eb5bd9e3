// instr_mix.hip — issue cost of the field layer's instruction classes on gfx950, alone and mixed
// with v_mad_u64_u32 (the MAC).  Answers: does a 32-bit ALU op / 64-bit shift cost the SIMD the same
// issue time as a MAC, and does it hide behind one?  (profiles/README.md, round 2; superseded by issue_cost.hip.)
//   hipcc --offload-arch=gfx950 -O3 instr_mix.hip -o instr_mix && ./instr_mix
// Each kernel: 8 independent chains x 16 unrolled slots per iteration; WAVES waves per SIMD.
// Reported: cycles per SLOT per SIMD (a slot = one MAC plus the ops the variant adds), with the clock
// read from s_memrealtime-calibrated s_memtime inside the kernel (shader clock, not the nominal).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHAINS 8
#define UNROLL 16

__device__ __forceinline__ unsigned long long memtime() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
    return t;
}
__device__ __forceinline__ unsigned long long memrealtime() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
    return t;
}

// BODY(k, r) uses: unsigned long long acc[k]; unsigned x[k], y[k], b[]
#define KERNEL(NAME, BODY)                                                                        \
    __global__ void NAME(int iters, unsigned long long *out, unsigned long long *clk) {          \
        unsigned long long acc[CHAINS];                                                           \
        unsigned x[CHAINS], y[CHAINS], b[CHAINS];                                                 \
        for (int k = 0; k < CHAINS; k++) {                                                        \
            acc[k] = threadIdx.x + k;                                                             \
            x[k] = threadIdx.x * 2654435761u + k;                                                 \
            y[k] = threadIdx.x * 40503u + 3 * k;                                                  \
            b[k] = blockIdx.x * 40503u + 7 * k + 1;                                               \
        }                                                                                         \
        unsigned long long t0 = memtime(), r0 = memrealtime();                                    \
        for (int it = 0; it < iters; it++) {                                                      \
            _Pragma("unroll") for (int r = 0; r < UNROLL; r++) {                                  \
                _Pragma("unroll") for (int k = 0; k < CHAINS; k++) { BODY }                       \
            }                                                                                     \
        }                                                                                         \
        unsigned long long t1 = memtime(), r1 = memrealtime();                                    \
        unsigned long long s = 0;                                                                 \
        for (int k = 0; k < CHAINS; k++) s ^= acc[k] ^ x[k] ^ y[k];                               \
        if (s == 0x1234567ull) out[0] = s;                                                        \
        if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }          \
    }

#define MAD asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k]) : "v"(x[k]), "v"(b[(k + r) & 7]) : "vcc");
#define AND32 asm volatile("v_and_b32 %0, %0, %1" : "+v"(y[k]) : "v"(b[(k + r) & 7]));
#define ADD32 asm volatile("v_add_u32 %0, %0, %1" : "+v"(y[k]) : "v"(b[(k + r) & 7]));
#define SHR32 asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(y[k]));
#define MUL24 asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(y[k]) : "v"(b[(k + r) & 7]));
#define MULLO asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(y[k]) : "v"(b[(k + r) & 7]));
#define ADD3 asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(y[k]) : "v"(b[(k + r) & 7]));
#define BFE asm volatile("v_bfe_u32 %0, %0, 3, 26" : "+v"(y[k]));
#define ALIGNB asm volatile("v_alignbit_b32 %0, %0, %1, 26" : "+v"(y[k]) : "v"(b[(k + r) & 7]));
#define ANDOR asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(y[k]) : "v"(b[(k + r) & 7]));
#define CNDM asm volatile("v_cmp_gt_u32 vcc, %1, %0\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(y[k]) : "v"(b[(k + r) & 7]) : "vcc");
#define SHR64 asm volatile("v_lshrrev_b64 %0, 26, %0" : "+v"(acc[k]));
#define LSHLADD64 asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(acc[k]));
#define ADDCO asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, 0, %2, vcc" : "+v"(y[k]) : "v"(b[(k + r) & 7]), "v"(x[k]) : "vcc");
#define MOVB asm volatile("v_mov_b32 %0, %1" : "=v"(y[k]) : "v"(b[(k + r) & 7]));
#define FMA64 asm volatile("v_fma_f64 %0, %1, %1, %0" : "+v"(acc[k]) : "v"((double)0.0) );
#define PKMOV asm volatile("v_pk_mov_b32 %0, %0, %1 op_sel:[0,1]" : "+v"(acc[k]) : "v"(acc[(k+1)&7]));
#define MULHI asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(y[k]) : "v"(b[(k + r) & 7]));
#define DPP asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(y[k]) : "v"(x[k]));


#define ANDLIT asm volatile("v_and_b32 %0, 0x3ffffff, %0" : "+v"(y[k]));
#define ANDSGPR asm volatile("v_and_b32 %0, %1, %0" : "+v"(y[k]) : "s"(0x3ffffffu));
#define NOP asm volatile("s_nop 0");
#define MAD2CH asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k & 1]) : "v"(x[k]), "v"(b[(k + r) & 7]) : "vcc");
#define MAD3CH asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k % 3]) : "v"(x[k]), "v"(b[(k + r) & 7]) : "vcc");
#define MAD1CH asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[0]) : "v"(x[k]), "v"(b[(k + r) & 7]) : "vcc");
#define MULLO2 asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(y[k]) : "v"(b[(k + r) & 7]));
#define SHL1 asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(y[k]));
#define SUBREV asm volatile("v_subrev_u32 %0, %1, %0" : "+v"(y[k]) : "v"(b[(k + r) & 7]));
#define ADDLIT asm volatile("v_add_u32 %0, 0x7ffffda, %0" : "+v"(y[k]));
KERNEL(k_mad, MAD)
KERNEL(k_and, AND32)
KERNEL(k_add, ADD32)
KERNEL(k_shr, SHR32)
KERNEL(k_mul24, MUL24)
KERNEL(k_mullo, MULLO)
KERNEL(k_mulhi, MULHI)
KERNEL(k_add3, ADD3)
KERNEL(k_bfe, BFE)
KERNEL(k_alignbit, ALIGNB)
KERNEL(k_andor, ANDOR)
KERNEL(k_shr64, SHR64)
KERNEL(k_lshladd64, LSHLADD64)
KERNEL(k_addco_pair, ADDCO)
KERNEL(k_mov, MOVB)
KERNEL(k_dpp, DPP)
KERNEL(k_pkmov, PKMOV)
KERNEL(k_mad_and, MAD AND32)
KERNEL(k_mad_2and, MAD AND32 ADD32)
KERNEL(k_mad_shr64, MAD SHR64)
KERNEL(k_mad_mul24, MAD MUL24)
KERNEL(k_mad_lshladd64, MAD LSHLADD64)
KERNEL(k_mad_mov, MAD MOVB)
KERNEL(k_2mad_and, MAD MAD AND32)
KERNEL(k_mad_bfe, MAD BFE)

KERNEL(k_andlit, ANDLIT)
KERNEL(k_andsgpr, ANDSGPR)
KERNEL(k_addlit, ADDLIT)
KERNEL(k_mad_andlit, MAD ANDLIT)
KERNEL(k_mad_andsgpr, MAD ANDSGPR)
KERNEL(k_mad_nop, MAD NOP)
KERNEL(k_mad1ch, MAD1CH)
KERNEL(k_mad2ch, MAD2CH)
KERNEL(k_mad3ch, MAD3CH)
KERNEL(k_mad_mullo, MAD MULLO2)
KERNEL(k_mad_shl, MAD SHL1)
KERNEL(k_mad_andlit_shr64, MAD ANDLIT SHR64)
KERNEL(k_3mad_andlit_shr64_mullo, MAD MAD MAD ANDLIT SHR64 MULLO2)

typedef void (*kfn)(int, unsigned long long *, unsigned long long *);

int main(int argc, char **argv) {
    struct { const char *name; kfn f; double ops_per_slot; } ks[] = {
        {"v_mad_u64_u32", k_mad, 1}, {"v_and_b32 lit", k_andlit, 1}, {"v_and_b32 sgpr", k_andsgpr, 1}, {"v_add_u32 lit", k_addlit, 1},
        {"mad+and lit", k_mad_andlit, 2}, {"mad+and sgpr", k_mad_andsgpr, 2}, {"mad+s_nop", k_mad_nop, 2},
        {"mad 1 chain", k_mad1ch, 1}, {"mad 2 chains", k_mad2ch, 1}, {"mad 3 chains", k_mad3ch, 1},
        {"mad+mul_lo", k_mad_mullo, 2}, {"mad+shl32", k_mad_shl, 2}, {"mad+andlit+shr64", k_mad_andlit_shr64, 3},
        {"3mad+andlit+shr64+mullo", k_3mad_andlit_shr64_mullo, 6},
 {"v_and_b32", k_and, 1}, {"v_add_u32", k_add, 1},
        {"v_lshrrev_b32", k_shr, 1}, {"v_mul_u32_u24", k_mul24, 1}, {"v_mul_lo_u32", k_mullo, 1},
        {"v_mul_hi_u32", k_mulhi, 1}, {"v_add3_u32", k_add3, 1}, {"v_bfe_u32", k_bfe, 1},
        {"v_alignbit_b32", k_alignbit, 1}, {"v_and_or_b32", k_andor, 1}, {"v_lshrrev_b64", k_shr64, 1},
        {"v_lshl_add_u64", k_lshladd64, 1}, {"v_add_co+addc", k_addco_pair, 2}, {"v_mov_b32", k_mov, 1},
        {"v_mov_b32_dpp", k_dpp, 1}, {"v_pk_mov_b32", k_pkmov, 1},
        {"mad+and", k_mad_and, 2}, {"mad+and+add", k_mad_2and, 3}, {"mad+shr64", k_mad_shr64, 2},
        {"mad+mul24", k_mad_mul24, 2}, {"mad+lshl_add64", k_mad_lshladd64, 2}, {"mad+mov", k_mad_mov, 2},
        {"2mad+and", k_2mad_and, 3}, {"mad+bfe", k_mad_bfe, 2},
    };
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int iters = 2000;
    unsigned long long *out, *clk;
    hipMalloc(&out, 64);
    hipMalloc(&clk, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("CUs %d nominal clock(kHz) %d\n", cus, prop.clockRate);
    const int wave_opts[] = {2, 3, 4};
    for (int wv : wave_opts) {
        const int blocks = cus * wv, threads = 256;   // 4 waves per block -> wv waves per SIMD
        printf("== %d waves/SIMD ==\n", wv);
        for (auto &k : ks) {
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, iters / 8, out, clk);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, iters, out, clk);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            unsigned long long c[2];
            hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
            const double slots_per_wave = (double)iters * UNROLL * CHAINS;
            // shader clock from s_memtime vs s_memrealtime (100 MHz) in block 0
            const double fclk = c[1] ? (double)c[0] / ((double)c[1] / 100e6) : 0;
            // cycles per slot per SIMD, from the wall time and the in-kernel clock
            const double cyc = (ms * 1e-3) * fclk / (slots_per_wave * wv);
            printf("%-18s %7.3f ms  fclk %.2f GHz  %.2f cyc/slot/SIMD  %.2f cyc/instr\n", k.name, ms, fclk / 1e9, cyc,
                   cyc / k.ops_per_slot);
        }
    }
    return 0;
}
