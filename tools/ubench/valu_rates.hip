// Throughput of single VALU instructions on gfx950 (whole chip, many waves):
// 8 independent chains per lane, ITERS iterations, inline asm so the compiler
// cannot fold or re-associate. Prints ns per wave-instruction per SIMD.
//
// Usage: valu_rates [W ...] [-op NAME]: one launch per (op, W waves per SIMD)
// (default W = 8). Round 5: W = 1/2/4/8/16 and packed
// controls, so that issue cycles per instruction against waves per SIMD can be
// read from counters (SQ_ACTIVE_INST_VALU, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE per
// dispatch, tools/ubench/valu_pmc.sh) as well as from the event clock; and the
// 64-bit compare forms the config-E sort network uses (u64 max as compare +
// two selects, against v_max_f64 / v_min_f64 on keys encoded as doubles).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define ITERS 4096
#define CHAIN8(INSN)                                                                                   \
    for (int i = 0; i < ITERS; ++i) {                                                                  \
        asm volatile(INSN " %0, %0, %8\n\t" INSN " %1, %1, %8\n\t" INSN " %2, %2, %8\n\t" INSN          \
                     " %3, %3, %8\n\t" INSN " %4, %4, %8\n\t" INSN " %5, %5, %8\n\t" INSN " %6, %6, %8\n\t" \
                     INSN " %7, %7, %8"                                                                 \
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)  \
                     : "s"(k));                                                                          \
    }

#define KERNEL(NAME, INSN)                                                                \
    __global__ void NAME(unsigned *out, unsigned k) {                                     \
        unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                   \
        CHAIN8(INSN)                                                                      \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
    }
KERNEL(k_add, "v_add_u32")
KERNEL(k_xor, "v_xor_b32")
KERNEL(k_mullo, "v_mul_lo_u32")
KERNEL(k_mul24, "v_mul_u32_u24")
KERNEL(k_mulhi, "v_mul_hi_u32")
#define CHAIN8_1(INSN)                                                                                   \
    for (int i = 0; i < ITERS; ++i) {                                                                    \
        asm volatile(INSN " %0, %0\n\t" INSN " %1, %1\n\t" INSN " %2, %2\n\t" INSN " %3, %3\n\t" INSN       \
                     " %4, %4\n\t" INSN " %5, %5\n\t" INSN " %6, %6\n\t" INSN " %7, %7"                          \
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));     \
    }
__global__ void k_ffbl(unsigned *out, unsigned k) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    CHAIN8_1("v_ffbl_b32")
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ k;
}
KERNEL(k_max, "v_max_u32")

// three-operand forms: dst = op(dst, dst, k)
#define CHAIN8_3(INSN, SUFFIX)                                                                                   \
    for (int i = 0; i < ITERS; ++i) {                                                                            \
        asm volatile(INSN " %0, %0, %0, %8" SUFFIX "\n\t" INSN " %1, %1, %1, %8" SUFFIX "\n\t" INSN            \
                     " %2, %2, %2, %8" SUFFIX "\n\t" INSN " %3, %3, %3, %8" SUFFIX "\n\t" INSN " %4, %4, %4, %8" \
                     SUFFIX "\n\t" INSN " %5, %5, %5, %8" SUFFIX "\n\t" INSN " %6, %6, %6, %8" SUFFIX "\n\t"     \
                     INSN " %7, %7, %7, %8" SUFFIX                                                               \
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)            \
                     : "s"(k));                                                                                  \
    }
#define KERNEL3(NAME, INSN, SUFFIX)                                                       \
    __global__ void NAME(unsigned *out, unsigned k) {                                     \
        unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                   \
        CHAIN8_3(INSN, SUFFIX)                                                            \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
    }
KERNEL3(k_bitop3, "v_bitop3_b32", " bitop3:0x82")
KERNEL3(k_mad24, "v_mad_u32_u24", "")
KERNEL3(k_max3, "v_max3_u32", "")
KERNEL3(k_fmaf3, "v_fma_f32", "")

// v_xor_b32 with SDWA src0 = WORD_1 (x ^= x >> 16)
#define CHAIN8_SDWA()                                                                                           \
    for (int i = 0; i < ITERS; ++i) {                                                                           \
        asm volatile(                                                                                           \
            "v_xor_b32_sdwa %0, %0, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"  \
            "v_xor_b32_sdwa %1, %1, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"  \
            "v_xor_b32_sdwa %2, %2, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"  \
            "v_xor_b32_sdwa %3, %3, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"  \
            "v_xor_b32_sdwa %4, %4, %4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"  \
            "v_xor_b32_sdwa %5, %5, %5 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"  \
            "v_xor_b32_sdwa %6, %6, %6 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"  \
            "v_xor_b32_sdwa %7, %7, %7 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"        \
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));                 \
    }
__global__ void k_xsdwa(unsigned *out, unsigned k) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    CHAIN8_SDWA()
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ k;
}


// 64-bit forms: dst = op(dst, dst, k) on VGPR pairs (f64 FMA, u64 compare + select)
#define KERNEL_F64(NAME, BODY)                                                                  \
    __global__ void NAME(unsigned *out, unsigned k) {                                           \
        double d0 = threadIdx.x, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, d4 = d0 + 4, d5 = d0 + 5, \
               d6 = d0 + 6, d7 = d0 + 7;                                                        \
        const double kd = (double)k * 1e-12;                                                    \
        for (int i = 0; i < ITERS; ++i) {                                                       \
            asm volatile(BODY(0) BODY(1) BODY(2) BODY(3) BODY(4) BODY(5) BODY(6) BODY(7)        \
                         : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), \
                           "+v"(d7)                                                             \
                         : "s"(kd));                                                            \
        }                                                                                       \
        out[blockIdx.x * blockDim.x + threadIdx.x] =                                            \
            (unsigned)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);                                  \
    }
#define FMA64(i) "v_fma_f64 %" #i ", %" #i ", %" #i ", %8\n\t"
#define ADD64(i) "v_add_f64 %" #i ", %" #i ", %8\n\t"
KERNEL_F64(k_fma64, FMA64)
KERNEL_F64(k_add64, ADD64)
// v_cvt_u32_f64 (saturating truncation), 8 independent chains through a u32 -> f64 round trip
__global__ void k_cvt64(unsigned *out, unsigned k) {
    double d0 = threadIdx.x, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, d4 = d0 + 4, d5 = d0 + 5, d6 = d0 + 6, d7 = d0 + 7;
    unsigned u0, u1, u2, u3, u4, u5, u6, u7;
    for (int i = 0; i < ITERS / 2; ++i) {
        asm volatile(
            "v_cvt_u32_f64 %8, %0\n\tv_cvt_u32_f64 %9, %1\n\tv_cvt_u32_f64 %10, %2\n\tv_cvt_u32_f64 %11, %3\n\t"
            "v_cvt_u32_f64 %12, %4\n\tv_cvt_u32_f64 %13, %5\n\tv_cvt_u32_f64 %14, %6\n\tv_cvt_u32_f64 %15, %7\n\t"
            "v_cvt_f64_u32 %0, %8\n\tv_cvt_f64_u32 %1, %9\n\tv_cvt_f64_u32 %2, %10\n\tv_cvt_f64_u32 %3, %11\n\t"
            "v_cvt_f64_u32 %4, %12\n\tv_cvt_f64_u32 %5, %13\n\tv_cvt_f64_u32 %6, %14\n\tv_cvt_f64_u32 %7, %15"
            : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7), "=v"(u0), "=v"(u1),
              "=v"(u2), "=v"(u3), "=v"(u4), "=v"(u5), "=v"(u6), "=v"(u7));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7) ^ k;
}
#define MAX64(i) "v_max_f64 %" #i ", %" #i ", %8\n\t"
#define MIN64(i) "v_min_f64 %" #i ", %" #i ", %8\n\t"
KERNEL_F64(k_max64, MAX64)
KERNEL_F64(k_min64, MIN64)
// u64 max the way the compiler emits umax64: v_cmp_gt_u64 + two v_cndmask_b32
// (the 3 instructions count as 3 wave-instructions in the per-instruction figure)
__global__ void k_umax64(unsigned *out, unsigned k) {
    unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    const unsigned long long kk = 0x9E3779B97F4A7C15ull ^ k;
    for (int i = 0; i < ITERS; ++i) {
        // (the empty asm keeps each value opaque, so every iteration emits the
        // compare and both selects; no instruction of its own)
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
        a0 = a0 > kk ? a0 : kk;
        a1 = a1 > kk ? a1 : kk;
        a2 = a2 > kk ? a2 : kk;
        a3 = a3 > kk ? a3 : kk;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3);
}
// packed controls: v_pk_fma_f32 (2 x f32 per lane), v_pk_add_u16
__global__ void k_pkfma(unsigned *out, unsigned k) {
    double d0 = threadIdx.x, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, d4 = d0 + 4, d5 = d0 + 5, d6 = d0 + 6, d7 = d0 + 7;
    const double kd = (double)k * 1e-12;
    for (int i = 0; i < ITERS; ++i) {
#define PKF(x) "v_pk_fma_f32 %" #x ", %" #x ", %" #x ", %8\n\t"
        asm volatile(PKF(0) PKF(1) PKF(2) PKF(3) PKF(4) PKF(5) PKF(6) PKF(7)
                     : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                     : "v"(kd));
#undef PKF
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
}
KERNEL(k_pkaddu16, "v_pk_add_u16")

// v_mad_u64_u32 (32x32 + 64 -> 64)
__global__ void k_mad64(unsigned *out, unsigned k) {
    unsigned long long a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
                       a7 = a0 + 7;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_mad_u64_u32 %0, vcc, %8, %8, %0\n\tv_mad_u64_u32 %1, vcc, %8, %8, %1\n\t"
            "v_mad_u64_u32 %2, vcc, %8, %8, %2\n\tv_mad_u64_u32 %3, vcc, %8, %8, %3\n\t"
            "v_mad_u64_u32 %4, vcc, %8, %8, %4\n\tv_mad_u64_u32 %5, vcc, %8, %8, %5\n\t"
            "v_mad_u64_u32 %6, vcc, %8, %8, %6\n\tv_mad_u64_u32 %7, vcc, %8, %8, %7"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "s"(k)
            : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}

int main(int argc, char **argv) {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const char *only = nullptr;
    int ws[16], nw = 0;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "-op") && i + 1 < argc) only = argv[++i];
        else if (nw < 16) ws[nw++] = atoi(argv[i]);
    }
    if (!nw) ws[nw++] = 8;
    const int threads = 64;
    unsigned *out;
    hipMalloc(&out, (size_t)cus * 4 * 32 * threads * 4);
    struct { const char *n; void (*f)(unsigned *, unsigned); int insts; } ks[] = {
        {"v_add_u32", k_add, 8}, {"v_xor_b32", k_xor, 8}, {"v_mul_lo_u32", k_mullo, 8}, {"v_mul_u32_u24", k_mul24, 8},
        {"v_mul_hi_u32", k_mulhi, 8}, {"v_ffbl_b32", k_ffbl, 8}, {"v_max_u32", k_max, 8},
        {"v_bitop3_b32", k_bitop3, 8}, {"v_mad_u32_u24", k_mad24, 8}, {"v_max3_u32", k_max3, 8}, {"v_fma_f32", k_fmaf3, 8},
        {"v_xor_b32_sdwa", k_xsdwa, 8}, {"v_fma_f64", k_fma64, 8}, {"v_add_f64", k_add64, 8},
        {"v_max_f64", k_max64, 8}, {"v_min_f64", k_min64, 8}, {"u64max(cmp+2cndmask)", k_umax64, 12},
        {"v_pk_fma_f32", k_pkfma, 8}, {"v_pk_add_u16", k_pkaddu16, 8},
        {"v_cvt_u32_f64+v_cvt_f64_u32", k_cvt64, 8}, {"v_mad_u64_u32", k_mad64, 8}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int wi = 0; wi < nw; ++wi) {
        const int W = ws[wi], blocks = cus * 4 * W;  // W waves per SIMD (one-wave workgroups)
        for (int rep = 0; rep < 2; ++rep)
            for (auto &k : ks) {
                if (only && strcmp(only, k.n)) continue;
                hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 0x9E3779B1u);
                hipEventRecord(a);
                hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 0x9E3779B1u);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                // (k_cvt64 runs ITERS/2 iterations of 16 instructions: the same count)
                const double wave_insts_per_simd = (double)W * ITERS * k.insts;
                if (rep)
                    printf("%-28s W=%-2d %8.3f ms  %.3f ns per wave-instruction per SIMD\n", k.n, W, ms,
                           ms * 1e6 / wave_insts_per_simd);
            }
    }
    return 0;
}
