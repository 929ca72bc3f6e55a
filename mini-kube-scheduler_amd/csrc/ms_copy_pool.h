// ms_copy_pool.h — helper threads for the host copies of a host-array call
// (ms_schedule_batch(_compact) on one shard): the caller's pageable pod array
// into the pinned staging K1 reads, and the pinned results back into the
// caller's array. The first chunk's copy-in and the last chunk's copy-out are
// on the call's critical path (the kernel cannot start before the first, the
// call cannot return before the last); one core moves ~35 GB/s, so 400 KB cost
// ~12 us each at config C. Split over the caller and `helpers` threads they run
// at memory bandwidth instead.
//
// Helpers spin on an epoch for a while after each job (back-to-back calls find
// them awake), then sleep on a condition variable. One job at a time: the
// caller holds the context's scheduling lock.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace msgpu {

class CopyPool {
  public:
    explicit CopyPool(unsigned helpers) {
        try {
            for (unsigned i = 0; i < helpers; ++i) th_.emplace_back([this, i] { run(i + 1); });
        } catch (...) {  // a thread could not be created: join the ones that were, then report
            shutdown();
            throw;
        }
    }
    ~CopyPool() { shutdown(); }
    CopyPool(const CopyPool &) = delete;
    CopyPool &operator=(const CopyPool &) = delete;

    unsigned ways() const { return (unsigned)th_.size() + 1u; }

    // fn(part, parts) for part = 0 .. ways()-1, the caller taking part 0; returns
    // when every part has finished.
    void run_parts(const std::function<void(unsigned, unsigned)> &fn) {
        job_ = &fn;
        done_.store(0, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> g(mu_);
            epoch_.fetch_add(1, std::memory_order_release);
        }
        if (sleeping_.load(std::memory_order_acquire)) cv_.notify_all();
        fn(0, ways());
        while (done_.load(std::memory_order_acquire) != (unsigned)th_.size()) std::this_thread::yield();
        job_ = nullptr;
    }

  private:
    void shutdown() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_.store(true, std::memory_order_relaxed);
            epoch_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto &t : th_)
            if (t.joinable()) t.join();
    }

    void run(unsigned part) {
        // (0, the epoch at construction, not a fresh load: a job posted before this
        // thread got here would otherwise be missed and its caller would wait forever)
        uint64_t seen = 0;
        for (;;) {
            // spin ~200 us for the next job, then sleep
            const auto t0 = std::chrono::steady_clock::now();
            uint64_t e;
            while ((e = epoch_.load(std::memory_order_acquire)) == seen) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) {
                    std::unique_lock<std::mutex> lk(mu_);
                    sleeping_.fetch_add(1, std::memory_order_acq_rel);
                    cv_.wait(lk, [&] { return epoch_.load(std::memory_order_acquire) != seen; });
                    sleeping_.fetch_sub(1, std::memory_order_acq_rel);
                }
            }
            seen = e;
            if (stop_.load(std::memory_order_relaxed)) return;
            (*job_)(part, ways());
            done_.fetch_add(1, std::memory_order_release);
        }
    }

    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::atomic<uint64_t> epoch_{0};
    std::atomic<unsigned> done_{0}, sleeping_{0};
    std::atomic<bool> stop_{false};
    const std::function<void(unsigned, unsigned)> *job_ = nullptr;
};

}  // namespace msgpu
