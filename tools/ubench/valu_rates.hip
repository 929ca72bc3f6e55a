// Throughput of single VALU instructions on gfx950 (whole chip, many waves):
// 8 independent chains per lane, ITERS iterations, inline asm so the compiler
// cannot fold or re-associate. Prints ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

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

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 4 * 8, threads = 64;  // 8 waves per SIMD
    unsigned *out;
    hipMalloc(&out, blocks * threads * 4);
    struct { const char *n; void (*f)(unsigned *, unsigned); } ks[] = {
        {"v_add_u32", k_add}, {"v_xor_b32", k_xor}, {"v_mul_lo_u32", k_mullo}, {"v_mul_u32_u24", k_mul24},
        {"v_mul_hi_u32", k_mulhi}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep)
        for (auto &k : ks) {
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 0x9E3779B1u);
            hipEventRecord(a);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 0x9E3779B1u);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double wave_insts_per_simd = (double)blocks / (cus * 4) * ITERS * 8;
            if (rep) printf("%-16s %.3f ms  %.3f ns per wave-instruction per SIMD\n", k.n, ms,
                            ms * 1e6 / wave_insts_per_simd);
        }
    return 0;
}
