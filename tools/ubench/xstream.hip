// Cross-stream hand-off latency on one GPU: kernel A (stream 1) -> B (stream 2)
// via (0) a stream event, (1) an event created with hipEventReleaseToDevice,
// (2) hipStreamWaitValue32 on signal memory written by A.
// B's stream is kept busy by a kernel C that ends after (odd iterations) or
// before (even) A, to separate "waiting" from "barrier processing" cost.
// Timestamps come from rocprofv3 --kernel-trace (tools/ubench/xstream.py).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void k_busy(uint32_t cycles, uint32_t *flag, uint32_t val) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (flag && threadIdx.x == 0 && blockIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(flag, val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

#define CK(x)                                                          \
    do {                                                               \
        hipError_t e = (x);                                            \
        if (e != hipSuccess) {                                         \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));         \
            return 1;                                                  \
        }                                                              \
    } while (0)

int main(int argc, char **argv) {
    const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, mode == 1 ? (hipEventDisableTiming | hipEventReleaseToDevice)
                                              : hipEventDisableTiming));
    uint32_t *sig;
    CK(hipExtMallocWithFlags((void **)&sig, 8, hipMallocSignalMemory));
    CK(hipMemset(sig, 0, 8));
    CK(hipDeviceSynchronize());
    if (mode == 3) {  // the same pattern captured into a graph (fork/join through events), launched per iteration
        hipEvent_t fork;
        CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        hipGraphExec_t ge[2];
        for (int odd = 0; odd < 2; ++odd) {
            hipGraph_t g;
            CK(hipStreamBeginCapture(s2, hipStreamCaptureModeGlobal));
            CK(hipEventRecord(fork, s2));
            CK(hipStreamWaitEvent(s1, fork, 0));
            k_busy<<<1, 64, 0, s2>>>(odd ? 100000u : 12000u, nullptr, 0);
            k_busy<<<1, 64, 0, s1>>>(50000u, nullptr, 0);
            CK(hipEventRecord(ev, s1));
            CK(hipStreamWaitEvent(s2, ev, 0));
            k_busy<<<1, 64, 0, s2>>>(2000u, nullptr, 0);
            CK(hipStreamEndCapture(s2, &g));
            CK(hipGraphInstantiate(&ge[odd], g, nullptr, nullptr, 0));
        }
        for (int it = 1; it <= 200; ++it) {
            CK(hipGraphLaunch(ge[it & 1], s2));
            CK(hipDeviceSynchronize());
        }
        std::printf("mode %d done\n", mode);
        return 0;
    }
    for (int it = 1; it <= 200; ++it) {
        // C on s2: ~40 us (odd) or ~5 us (even); A on s1: ~20 us; then B on s2 after the hand-off
        k_busy<<<1, 64, 0, s2>>>(it & 1 ? 100000u : 12000u, nullptr, 0);
        k_busy<<<1, 64, 0, s1>>>(50000u, mode == 2 ? sig : nullptr, (uint32_t)it);
        if (mode == 2) {
            CK(hipStreamWaitValue32(s2, sig, (uint32_t)it, hipStreamWaitValueGte, 0xFFFFFFFFu));
        } else {
            CK(hipEventRecord(ev, s1));
            CK(hipStreamWaitEvent(s2, ev, 0));
        }
        k_busy<<<1, 64, 0, s2>>>(2000u, nullptr, 0);
        CK(hipDeviceSynchronize());
    }
    std::printf("mode %d done\n", mode);
    return 0;
}
