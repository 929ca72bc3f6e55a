// CopyPool (mini-kube-scheduler_amd/csrc/ms_copy_pool.h): every part of every job
// runs exactly once, jobs never overlap, helpers that went to sleep wake for the
// next job, and destruction joins spinning and sleeping helpers. Built under
// ThreadSanitizer by tests/test_host_cpp.py.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "ms_copy_pool.h"

int main() {
    int failed = 0;
    for (unsigned helpers : {0u, 1u, 3u, 7u}) {
        msgpu::CopyPool pool(helpers);
        std::vector<unsigned char> src(1 << 20), dst(1 << 20);
        for (size_t i = 0; i < src.size(); ++i) src[i] = (unsigned char)(i * 131u + helpers);
        for (int job = 0; job < 300; ++job) {
            if (job == 100 || job == 200)  // helpers asleep (spin window over) before these jobs
                std::this_thread::sleep_for(std::chrono::milliseconds(5));
            std::vector<std::atomic<int>> hits(pool.ways());
            const size_t n = src.size() - (size_t)job;
            std::memset(dst.data(), 0, dst.size());
            pool.run_parts([&](unsigned p, unsigned P) {
                hits[p].fetch_add(1);
                const size_t a = n * p / P, b = n * (p + 1) / P;
                std::memcpy(dst.data() + a, src.data() + a, b - a);
            });
            for (unsigned p = 0; p < pool.ways(); ++p) failed += hits[p].load() != 1;
            failed += std::memcmp(dst.data(), src.data(), n) != 0;
        }
    }
    for (int i = 0; i < 200; ++i) {  // a job posted before the helper threads have started
        msgpu::CopyPool pool(3);
        std::atomic<int> parts{0};
        pool.run_parts([&](unsigned, unsigned) { parts.fetch_add(1); });
        failed += parts.load() != 4;
    }
    {  // destroyed while its helpers sleep
        msgpu::CopyPool pool(2);
        pool.run_parts([](unsigned, unsigned) {});
        std::this_thread::sleep_for(std::chrono::milliseconds(3));
    }
    std::printf("%d failed\n", failed);
    return failed ? 1 : 0;
}
