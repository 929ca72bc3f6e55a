// ms_ctx.h — the engine context behind the C ABI, shared by ms_capi.cpp (one
// device's node shard, deltas, staging, streams) and ms_comm.cpp (the RCCL
// communicator and node-sharded pipelines). Not part of the public boundary.
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "ms_copy_pool.h"
#include "ms_internal.h"

namespace msgpu {
struct CommState;
}

using msgpu::DRow;
using msgpu::NodeDelta;
using msgpu::NodeTable;

struct ms_ctx {
    ms_config cfg{};
    hipStream_t stream = nullptr;
    int num_cus = 0;
    NodeTable t{};
    // helper threads for the host copies of single-shard host-array calls
    // (ms_copy_pool.h; created on the first large call, joined when the context is deleted)
    std::unique_ptr<msgpu::CopyPool> copy_pool;

    // node deltas (informer goroutines) — guarded by delta_mu
    std::mutex delta_mu;
    std::vector<NodeDelta> pending;
    std::vector<uint8_t> present;  // host mirror of presence, updated at enqueue
    uint32_t present_count = 0;
    uint32_t rows_used = 0;  // high-water mark of upserted rows (sweep extent)
    // what the device table holds after the last flush: snapshots of the two
    // counters above taken with the drained deltas (under delta_mu), read only
    // by sched_mu holders
    uint32_t rows_dev = 0, present_dev = 0;

    // one scheduling caller at a time (minisched.go:28-30 runs one goroutine)
    std::mutex sched_mu;

    // staging (d_pods / d_res / h_pods / h_res hold stage_cap pods; the key and
    // flag scratch batch_cap; the compact records compact_cap)
    uint32_t batch_cap = 0, stage_cap = 0, compact_cap = 0;
    ms_pod_compact *d_podc = nullptr;
    ms_result_compact *d_resc = nullptr;
    ms_pod_rec *h_pods = nullptr;
    ms_result *h_res = nullptr;
    ms_pod_rec *d_pods = nullptr;
    ms_result *d_res = nullptr;
    unsigned long long *d_keys = nullptr;
    uint32_t *d_flags = nullptr;  // per-pod filter flags (set 1) / NodeAffinity anchors (set 2)
    uint32_t w_nn = 1, w_na = 1;  // score weights (MS_PLUGINS_NU_NN_NA)
    NodeDelta *h_deltas = nullptr;
    NodeDelta *d_deltas = nullptr;
    uint32_t delta_cap = 0;
    ms_pod_rec *d_one = nullptr;  // commit/uncommit staging

    // sequential engine scratch
    unsigned long long *d_tile_keys = nullptr;
    uint32_t *d_tile_flags = nullptr;
    unsigned long long *d_spec = nullptr;  // per-pod speculative winner key (atomicMax target)
    uint32_t *d_spec_flags = nullptr;      // per-pod flags of tiles with no feasible row (atomicOr target)
    unsigned long long *d_top4 = nullptr;  // per-pod global speculative top-4 keys
    int64_t *d_top4_rec = nullptr;         // their batch-start node records (validator layout)
    unsigned long long *d_top_ext = nullptr;  // ranks 4..7 per pod (the validator's slow pods)
    uint32_t *d_merge_tags = nullptr;         // per pod of both merge-output sets: the in-step merge's tag
    uint32_t *d_merge_ctr = nullptr;          // the in-step merge's sweep-done counter
    void *d_table = nullptr;                  // the node table's columns, one allocation (ms_create)
    uint32_t merge_tag = 0;                   // last in-step merge tag issued
    unsigned long long *d_tl = nullptr;       // MS_VSTAMPS: step timeline (MS_TIMELINE=<file> dumps it at ms_destroy)
    uint32_t *d_prev = nullptr;            // {count, rows} of the nodes each batch bound (x2)
    int64_t *d_prev_rec = nullptr;         // and their final records (x2)
    DRow *d_drow = nullptr;                // derived rows of the binary64 sweep (tile_cap * kFullWaveTile)
    // (every sequential-engine buffer above is double-buffered by batch parity)
    // ms_schedule_batch's chunked copies (schedule_chunked): H2D / D2H of host arrays beside the cycle
    hipStream_t copy_stream = nullptr;
    hipEvent_t ev_copy[4] = {nullptr, nullptr, nullptr, nullptr}, ev_cyc[4] = {nullptr, nullptr, nullptr, nullptr};
    uint32_t tile_cap = 0;  // tiles allocated per pod
    uint32_t *d_overflow = nullptr;
    ms_pod_compact *h_podz = nullptr;      // pinned compact pods / results the compact cycle's
    ms_result_compact *h_resz = nullptr;   // kernel reads and writes over PCIe (zero-copy)
    uint32_t z_cap = 0;
    // MS_PLUGINS_NU_TT_NN: segment summaries of the sweep (tt_bytes allocated)
    void *d_tt = nullptr;
    size_t tt_bytes = 0;
    // d_tt is one scratch for every TT cycle of the context: a cycle on another
    // stream than the previous one waits for ev_tt, recorded after that one's
    // combine (node-sharded submits run on caller / sweep streams that are not
    // chained through the context stream)
    hipEvent_t ev_tt = nullptr;
    hipStream_t tt_stream = nullptr;
    // MS_PLUGINS_NU_NN_NAM: the registered term sets as lookup tables (NamTab) and the
    // per-class passes' scratch of a chunk (nam_bytes allocated)
    void *d_terms = nullptr;
    uint32_t n_terms = 0, terms_cap = 0;
    void *d_nam = nullptr;
    size_t nam_bytes = 0;
    // node-sharded sequential mode: merged candidate lists (ms_seq_validate_device)
    ms_seq_cand *d_merged = nullptr;
    uint32_t *d_merged_flags = nullptr;


    // Ordering. Every piece of work that reads or writes the node table or the
    // context's scratch is totally ordered through the context stream: a call
    // on a caller stream first waits for the context stream (order_after_ctx_
    // stream), and its work is then chained back into the context stream
    // (chain_back), so later deltas, binds, read-backs and calls on any other
    // stream wait for it. ctx_seq counts enqueues on the context stream that a
    // caller stream has not necessarily seen; a caller stream ordered after it
    // at ctx_seq needs no new cross-stream wait (each costs ~6-10 us of idle
    // device time even when already signalled, tools/ubench/xstream).
    uint64_t ctx_seq = 0;
    // fence_seq counts the times the context stream was made to wait for the
    // communicator's in-flight sweeps (table readers on its internal streams,
    // comm_fence_reads); a stream ordered before the last fence must wait again
    uint64_t fence_seq = 0, ordered_fence = 0;
    hipStream_t ordered_stream = nullptr;
    uint64_t ordered_seq = 0;
    hipEvent_t ev_order = nullptr;
    hipEvent_t ev_back = nullptr;

    // RCCL communicator and the node-sharded pipelines (ms_comm.cpp); null
    // until ms_comm_init
    msgpu::CommState *comm = nullptr;

    // host phase times of the last ms_schedule_batch(_compact) call (ms_last_call_profile)
    uint64_t prof[MS_CALL_PHASES] = {};

    std::string err;
};

namespace msgpu {

// Records msg as the context's last error (or the thread's ms_create error).
int fail(ms_ctx *c, int code, const std::string &msg);

#define MS_HIP(c, call)                                                                          \
    do {                                                                                         \
        hipError_t e_ = (call);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return ::msgpu::fail((c), MS_E_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

inline uint32_t cdiv(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

// Host wall time of a host-array call split into MS_PH_* phases: lap(ph) adds
// the time since the previous lap to phase ph; the destructor records the
// call's total (every return path of the call).
class CallClock {
  public:
    using Clock = std::chrono::steady_clock;
    explicit CallClock(ms_ctx *c) : c_(c), t0_(Clock::now()), t_(t0_) {
        for (uint64_t &v : c_->prof) v = 0;
    }
    ~CallClock() { c_->prof[MS_PH_TOTAL] = ns(t0_, Clock::now()); }
    void lap(int ph) {
        const auto now = Clock::now();
        c_->prof[ph] += ns(t_, now);
        t_ = now;
    }
    void count(int ph, uint64_t k = 1) { c_->prof[ph] += k; }

  private:
    static uint64_t ns(Clock::time_point a, Clock::time_point b) {
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
    }
    ms_ctx *c_;
    Clock::time_point t0_, t_;
};

constexpr uint32_t kTopKCands = 4;  // ms_seq_cand entries per pod and shard (the validator's top-K)

// ms_capi.cpp (callers hold sched_mu)
int flush_locked(ms_ctx *c);
hipStream_t pick_stream(ms_ctx *c, void *s);
int order_after_ctx_stream(ms_ctx *c, hipStream_t s);
int chain_back(ms_ctx *c, hipStream_t s, bool recorded = false);
int ensure_tiles(ms_ctx *c, uint32_t n_tiles);
int ensure_stage(ms_ctx *c, uint32_t n);
// MS_PLUGINS_NU_TT_NN: this shard's merged per-pod summaries (MS_TT_SUMMARY_BYTES each) into out
int tt_summaries_locked(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *d_pods, void *out, hipStream_t s);
bool plugins_stateless(const ms_ctx *c);
// done (optional): recorded on s after the sweep (by the K1 dispatch itself when it is one launch)
int sweep_locked(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *d_pods, unsigned long long *keys, uint32_t *flags,
                 hipStream_t s, hipEvent_t done = nullptr);
int seq_candidates_locked(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, ms_seq_cand *cands_dev,
                          uint32_t *flags_dev, hipStream_t s);

// ms_comm.cpp
void comm_free(ms_ctx *c);
// ms_schedule_batch / ms_schedule_sequential_device on a context joined to a
// communicator (callers hold sched_mu; deltas flushed)
int comm_schedule_host(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods, int32_t mode, ms_result *out,
                       CallClock *ck);
// the same on pods already staged in c->d_pods (comm_stage(n) first), results in c->d_res
int comm_stage(ms_ctx *c, uint32_t n_pods);
int comm_cycle_staged(ms_ctx *c, uint32_t n_pods, int32_t mode);
int comm_schedule_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, ms_result *results_dev,
                         hipStream_t s);
void comm_rank_world(const ms_ctx *c, int32_t *rank, int32_t *world);
// Makes `writer` wait for the node-sharded sweeps still reading the table on the
// communicator's internal streams; returns 1 if it inserted waits, 0 if none
// were outstanding (or no communicator), < 0 on failure.
int comm_fence_reads(ms_ctx *c, hipStream_t writer);
// MS_PLUGINS_NU_TT_NN: the two-pass bit-sliced cycle (default) or, with
// MINISCHED_TT=v1, the per-pair summary sweep (read once per process).
int ensure_tt(ms_ctx *c, size_t need);

}  // namespace msgpu
