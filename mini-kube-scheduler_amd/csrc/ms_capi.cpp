// ms_capi.cpp — C ABI of the scheduling-cycle engine (include/minisched_gpu.h).
//
// Owns one device's node table (a shard of global ordinals), the node-delta
// queue fed by informer callbacks, pinned staging for the cgo caller, and the
// stream everything is ordered on. It never aborts: every HIP failure becomes
// MS_E_HIP with the message kept for ms_last_error.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "ms_ctx.h"

using namespace msgpu;


namespace msgpu {

namespace {
thread_local std::string g_create_err;

// validator counters: u32[6] (overflow, re-swept tiles, recomputes, pods, speculation misses,
// list scans), then u64[4] phase cycles in the MS_VSTAMPS diagnostic build
constexpr size_t kStatsBytes = 256;

}  // namespace

int fail(ms_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    else g_create_err = msg;
    return code;
}

constexpr int kSeqBufs = 3;         // sequential-engine batch buffer sets (pipeline depth <= 3)

void free_all(ms_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->cfg.device);
    comm_free(c);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->d_table) {  // the columns live in it
        (void)hipFree(c->d_table);
        c->d_table = nullptr;
        c->t.flags = c->t.digit = c->t.zone = c->t.label2 = nullptr;
        c->t.taints = nullptr;
        c->t.allowed_pods = c->t.pod_count = nullptr;
        c->t.alloc_cpu = c->t.alloc_mem = c->t.req_cpu = c->t.req_mem = c->t.nz_cpu = c->t.nz_mem = nullptr;
    }
    void *dev[] = {c->t.planes, c->t.zone, c->t.label2, c->d_terms, c->d_nam, c->t.flags, c->t.digit, c->t.allowed_pods, c->t.pod_count, c->t.alloc_cpu,
                   c->t.alloc_mem, c->t.req_cpu, c->t.req_mem, c->t.nz_cpu, c->t.nz_mem,
                   c->d_pods, c->d_res, c->d_keys, c->d_flags, c->d_deltas, c->d_one,
                   c->d_tile_keys, c->d_tile_flags, c->d_spec, c->d_spec_flags, c->d_top4, c->d_top4_rec, c->d_prev, c->d_prev_rec, c->d_overflow,
                   c->d_podc, c->d_resc,
                   c->d_merged, c->d_merged_flags, c->d_drow, c->d_top_ext, c->t.taints, c->d_tt,
                   c->d_merge_tags, c->d_merge_ctr};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    if (c->h_podz) (void)hipHostFree(c->h_podz);
    if (c->h_resz) (void)hipHostFree(c->h_resz);
    if (c->h_pods) (void)hipHostFree(c->h_pods);
    if (c->h_res) (void)hipHostFree(c->h_res);
    if (c->h_deltas) (void)hipHostFree(c->h_deltas);
    if (c->ev_order) (void)hipEventDestroy(c->ev_order);
    if (c->ev_back) (void)hipEventDestroy(c->ev_back);
    if (c->ev_tt) (void)hipEventDestroy(c->ev_tt);
    if (c->copy_stream) {
        (void)hipStreamSynchronize(c->copy_stream);
        (void)hipStreamDestroy(c->copy_stream);
    }
    // (the zero-copy path creates ev_cyc without a copy stream)
    for (int i = 0; i < 4; ++i) {
        if (c->ev_copy[i]) (void)hipEventDestroy(c->ev_copy[i]);
        if (c->ev_cyc[i]) (void)hipEventDestroy(c->ev_cyc[i]);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
}

int ensure_delta_cap(ms_ctx *c, uint32_t n) {
    if (n <= c->delta_cap) return MS_OK;
    uint32_t cap = std::max<uint32_t>(n, std::max<uint32_t>(1024, c->delta_cap * 2));
    if (c->h_deltas) (void)hipHostFree(c->h_deltas);
    if (c->d_deltas) (void)hipFree(c->d_deltas);
    c->h_deltas = nullptr;
    c->d_deltas = nullptr;
    c->delta_cap = 0;
    if (hipHostMalloc((void **)&c->h_deltas, sizeof(NodeDelta) * cap) != hipSuccess)
        return fail(c, MS_E_OOM, "pinned delta staging");
    if (hipMalloc((void **)&c->d_deltas, sizeof(NodeDelta) * cap) != hipSuccess)
        return fail(c, MS_E_OOM, "device delta staging");
    c->delta_cap = cap;
    return MS_OK;
}

// Drains the delta queue onto the stream (caller holds sched_mu).
int flush_locked(ms_ctx *c) {
    std::vector<NodeDelta> batch;
    {
        std::lock_guard<std::mutex> g(c->delta_mu);
        batch.swap(c->pending);
        c->rows_dev = c->rows_used;
        c->present_dev = c->present_count;
    }
    if (batch.empty()) return MS_OK;
    // the deltas land on the context stream: after the sweeps still reading the
    // table on the communicator's streams
    const int fenced = comm_fence_reads(c, c->stream);
    if (fenced < 0) return fenced;
    if (fenced) ++c->fence_seq;
    // later deltas to one row win: keep the last occurrence only
    std::unordered_map<uint32_t, uint32_t> last;
    last.reserve(batch.size() * 2);
    for (uint32_t i = 0; i < batch.size(); ++i) last[batch[i].local] = i;
    std::vector<NodeDelta> uniq;
    uniq.reserve(last.size());
    for (uint32_t i = 0; i < batch.size(); ++i)
        if (last[batch[i].local] == i) uniq.push_back(batch[i]);
    int rc = ensure_delta_cap(c, (uint32_t)uniq.size());
    if (rc) return rc;
    // the previous use of h_deltas must be complete before it is overwritten
    MS_HIP(c, hipStreamSynchronize(c->stream));
    std::memcpy(c->h_deltas, uniq.data(), sizeof(NodeDelta) * uniq.size());
    MS_HIP(c, hipMemcpyAsync(c->d_deltas, c->h_deltas, sizeof(NodeDelta) * uniq.size(),
                             hipMemcpyHostToDevice, c->stream));
    MS_HIP(c, launch_apply_deltas(c->t, c->d_deltas, (uint32_t)uniq.size(), c->stream));
    MS_HIP(c, launch_build_planes(c->t, c->d_deltas, (uint32_t)uniq.size(), c->stream));
    ++c->ctx_seq;
    return MS_OK;
}

hipStream_t pick_stream(ms_ctx *c, void *s) { return s ? (hipStream_t)s : c->stream; }

// Makes work later enqueued on s wait for everything already on the context stream.
int order_after_ctx_stream(ms_ctx *c, hipStream_t s) {
    const int fenced = comm_fence_reads(c, c->stream);
    if (fenced < 0) return fenced;
    if (fenced) ++c->fence_seq;
    if (s == c->stream) return MS_OK;
    if (s == c->ordered_stream && c->ordered_seq == c->ctx_seq && c->ordered_fence == c->fence_seq)
        return MS_OK;  // nothing new on the ctx stream
    if (!c->ev_order) MS_HIP(c, hipEventCreateWithFlags(&c->ev_order, hipEventDisableTiming));
    hipError_t e = hipEventRecord(c->ev_order, c->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, c->ev_order, 0);
    if (e != hipSuccess) return fail(c, MS_E_HIP, std::string("stream ordering: ") + hipGetErrorString(e));
    c->ordered_stream = s;
    c->ordered_seq = c->ctx_seq;
    c->ordered_fence = c->fence_seq;
    return MS_OK;
}

// After a call's last launch on caller stream s: the context stream waits for
// it, so later deltas, binds, read-backs and calls on other streams (which
// order after the context stream) come after this call's table and scratch
// accesses. s itself needs no new wait (ordered_seq is kept), another stream
// does (ordered_stream differs).
// recorded: ev_back was already recorded on s after the call's last launch
// (by that launch's own dispatch).
int chain_back(ms_ctx *c, hipStream_t s, bool recorded) {
    if (s == c->stream) return MS_OK;
    if (!c->ev_back) MS_HIP(c, hipEventCreateWithFlags(&c->ev_back, hipEventDisableTiming));
    hipError_t e = recorded ? hipSuccess : hipEventRecord(c->ev_back, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ev_back, 0);
    if (e != hipSuccess) return fail(c, MS_E_HIP, std::string("stream ordering: ") + hipGetErrorString(e));
    if (c->ordered_stream != s) {  // the ctx stream now holds s's work: other streams must wait for it
        ++c->ctx_seq;
        c->ordered_stream = s;
        c->ordered_seq = c->ctx_seq;
        c->ordered_fence = c->fence_seq;
    }
    return MS_OK;
}

// The in-step merge's counter (a counter, or one slot per sweep workgroup: at most 255).
hipError_t ctr_alloc(uint32_t **p) { return hipMalloc((void **)p, 1024); }

// Sequential-engine scratch for n_tiles tiles, kSeqBufs batches deep (the
// single-stream steps use two sets; the node-sharded candidates up to three).
int ensure_tiles(ms_ctx *c, uint32_t n_tiles) {
    if (n_tiles <= c->tile_cap) return MS_OK;
    MS_HIP(c, hipDeviceSynchronize());  // no batch still reads the old buffers
    void *old[] = {c->d_tile_keys, c->d_tile_flags, c->d_spec, c->d_spec_flags, c->d_top4, c->d_top4_rec, c->d_prev,
                   c->d_prev_rec, c->d_drow, c->d_top_ext, c->d_merge_tags, c->d_merge_ctr};
    for (void *q : old)
        if (q) (void)hipFree(q);
    c->d_tile_keys = nullptr;
    c->d_tile_flags = nullptr;
    c->d_spec = nullptr;
    c->d_spec_flags = nullptr;
    c->d_top4 = nullptr;
    c->d_top4_rec = nullptr;
    c->d_prev = nullptr;
    c->d_prev_rec = nullptr;
    c->d_drow = nullptr;
    c->d_top_ext = nullptr;
    c->d_merge_tags = nullptr;
    c->d_merge_ctr = nullptr;
    c->tile_cap = 0;
    // (ms_seq_candidates_device uses the same buffers for up to kSeqBufs * B pods)
    const size_t B = seq_batch_limit(), NB = kSeqBufs * B, n = NB * n_tiles;
    if (hipMalloc((void **)&c->d_tile_keys, n * seq_topk() * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc((void **)&c->d_tile_flags, n * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&c->d_spec, NB * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc((void **)&c->d_spec_flags, NB * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&c->d_top4, NB * seq_topk() * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc((void **)&c->d_top4_rec, NB * seq_topk() * seq_rec_fields() * sizeof(int64_t)) != hipSuccess ||
        hipMalloc((void **)&c->d_prev, 2 * (2 + seq_prev_cap()) * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&c->d_prev_rec, 2 * seq_prev_cap() * seq_rec_fields() * sizeof(int64_t)) != hipSuccess ||
        hipMalloc((void **)&c->d_drow, (size_t)n_tiles * kFullWaveTile * sizeof(DRow)) != hipSuccess ||
        hipMalloc((void **)&c->d_top_ext, NB * seq_topk() * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc((void **)&c->d_merge_tags, NB * sizeof(uint32_t)) != hipSuccess ||
        ctr_alloc(&c->d_merge_ctr) != hipSuccess)
        return fail(c, MS_E_OOM, "sequential-engine scratch");
    MS_HIP(c, hipMemsetAsync(c->d_merge_tags, 0, NB * sizeof(uint32_t), c->stream));
    MS_HIP(c, hipMemsetAsync(c->d_spec, 0, NB * sizeof(unsigned long long), c->stream));
    MS_HIP(c, hipMemsetAsync(c->d_spec_flags, 0, NB * sizeof(uint32_t), c->stream));
    MS_HIP(c, hipStreamSynchronize(c->stream));
    c->tile_cap = n_tiles;
    return MS_OK;
}

// Pods per speculative batch: fewer nodes touched per batch keeps the top-K
// lists valid; more pods amortise the two launches. MINISCHED_SEQ_BATCH
// overrides (tuning), clamped to the validator's LDS capacity.
uint32_t seq_batch(const ms_ctx *) {
    uint32_t b = seq_batch_limit();  // the build's batch (128: profiles/r01_e_batch_sweep.jsonl, r03o)
    if (const char *e = getenv("MINISCHED_SEQ_BATCH")) b = (uint32_t)std::max(1, atoi(e));
    return std::min(b, seq_batch_limit());
}

// Exact sequential engine: speculative per-tile top-K sweep + in-order
// validation, batch after batch on one stream.
int run_sequential(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *d_pods, ms_result *d_res, hipStream_t s) {
    const uint32_t rows = c->rows_dev;
    const uint32_t seed32 = seed32_of(c->cfg.seed);
    if (rows == 0) {  // no node listed: every pod is a FitError with an empty mask
        for (uint32_t s0 = 0; s0 < n_pods; s0 += c->batch_cap) {
            const uint32_t nb = std::min(c->batch_cap, n_pods - s0);
            MS_HIP(c, hipMemsetAsync(c->d_keys, 0, sizeof(unsigned long long) * nb, s));
            MS_HIP(c, launch_decode(d_pods + s0, nb, c->d_keys, nullptr, 0, d_res + s0, s));
        }
        return MS_OK;
    }
    if (rows > seq_max_rows())
        return fail(c, MS_E_CAPACITY, "resource-aware sequential mode supports at most " +
                                          std::to_string(seq_max_rows()) + " rows per context (shard the nodes)");
    // Tiles of the speculative sweep: one per CU beside the validator's where the
    // table allows (rows per tile a multiple of 16, 64..256): at 50k nodes 241
    // tiles of 208 rows on 241 CUs instead of 196 of 256 on 196 (round 6).
    NodeTable tq = c->t;
    {
        const uint32_t room = (uint32_t)std::max(2, c->num_cus) - 1u;
        const uint32_t tr = (cdiv(rows, room) + 15u) / 16u * 16u;
        tq.tile_rows = std::min<uint32_t>((uint32_t)kFullWaveTile, std::max<uint32_t>(64u, tr));
#ifdef MS_TILE_ROWS  // (A/B builds: a fixed tile height)
        tq.tile_rows = MS_TILE_ROWS;
#endif
    }
    const uint32_t n_tiles = cdiv(rows, tq.tile_rows);
    int rc = ensure_tiles(c, n_tiles);
    if (rc) return rc;
    // the engine's table copy carries the derived rows of the binary64 sweep,
    // rebuilt here (deltas and binds since the last run) and kept current by
    // the validator's write-back
    tq.drow = c->d_drow;
    MS_HIP(c, launch_build_drows(tq, rows, n_tiles * tq.tile_rows, s));
    // Step k = ONE launch (launch_seq_step): validation of batch k on workgroup
    // 0 while the other workgroups sweep batch k+1 and then merge its tile lists
    // (the in-step merge); batch k+1 treats batch k's binds as stale. No
    // cross-stream hand-off: each cost ~12 us per batch, and a validation launched
    // beside a sweep waited for a SIMD to drain (two-stream modes and a depth-2
    // step measured slower and removed in round 6: profiles/r02j_e_modes.txt,
    // r04w_e_fused2_ab.txt).
    const uint32_t B = seq_batch(c), SB = seq_batch_limit();
    // ranks 4..7 of the merge for the validator's slow pods (profiles/r03v_e_rank8_ab.txt)
    unsigned long long *const top_ext = c->d_top_ext;
    const size_t prev_words = 2 + seq_prev_cap(), prev_fields = (size_t)seq_prev_cap() * seq_rec_fields();
    const size_t cells_per_set = (size_t)SB * n_tiles, recs_per_set = (size_t)SB * seq_topk() * seq_rec_fields();
    {
        // Warm-up batches: the first 4,096 pods of the queue in batches of 64. On an
        // empty cluster every pod prefers the same emptiest nodes, so early batches
        // touch each other's speculative winners most (the slow-path burst of
        // batches 20-30); half-size batches there cut the re-sweeps to 0 and the
        // recomputes by 10 %: config E 39.7 -> 38.5 ms (profiles/r05l_e_ab.txt;
        // 4096:32 / 8192:32 / 16384:32 / 16384:64 / 32768:64 measured slower,
        // r05k_e_warm.txt). Round 6, with the validator's ranks 4..7 walk: none /
        // 4,096 / 8,192 pods 32.3 / 31.1 / 31.2 ms (profiles/r06j_e_warm_ab.txt).
#ifndef MS_WARM_PODS
#define MS_WARM_PODS 4096
#endif
        constexpr uint32_t kWarmPods = MS_WARM_PODS, kWarmBatch = 64;
        auto batch_at = [&](uint32_t s0) { return s0 < kWarmPods ? std::min(kWarmBatch, B) : B; };
        const uint32_t nb0 = std::min(batch_at(0), n_pods);
        const char *merge_env = getenv("MINISCHED_SEQ_MERGE");
        const std::string merge_mode = merge_env ? merge_env : "instep";
        const bool want_instep = merge_mode == "instep" || merge_mode == "fallback";
        if (want_instep) {
            // Tagged lists: no cell of either set may hold a tag from an earlier run
            // (or an earlier chunk of this call). Both sets, every pod slot: a
            // warm-up batch rewrites only its first pods, and a cell left from a
            // previous run whose 2-bit tag happened to match was taken as swept
            // (config E's second 65,536-pod chunk, pods 64..127 of its first
            // full-size batch: tests/test_gpu_fullsize.py, profiles/r05n_e_probe.txt).
            MS_HIP(c, hipMemsetAsync(c->d_merge_ctr, 0, 1024, s));
            MS_HIP(c, hipMemsetAsync(c->d_tile_keys, 0,
                                     (size_t)kSeqBufs * cells_per_set * seq_topk() * sizeof(unsigned long long), s));
            MS_HIP(c, hipMemsetAsync(c->d_tile_flags, 0, (size_t)kSeqBufs * cells_per_set * sizeof(uint32_t), s));
        }
        MS_HIP(c, launch_sweep_full_tiles(tq, rows, d_pods, nb0, seed32, c->d_tile_keys, c->d_tile_flags, n_tiles, s));
        MS_HIP(c, launch_topk_merge(c->d_tile_keys, c->d_tile_flags, nb0, n_tiles, c->d_top4, c->d_spec,
                                    c->d_spec_flags, tq, c->d_top4_rec, s, top_ext));
        // Batch k+1's merge inside step k (default since round 5, "instep"): the sweep
        // workgroups count themselves done on a device counter, then one wave per
        // pod merges the tile lists (written through, read L2-bypassing across the
        // XCDs) while the validator continues; a worker whose bounded wait runs out
        // leaves its pods untagged and the next validation merges them itself.
        // With the binary64 tile keys the sweep + merge path fits beside the
        // validator: config E 44.4 -> 40.5 ms against the merge launch
        // (profiles/r05c_e_ab.txt, r05f_e_sync_ab.txt). MINISCHED_SEQ_MERGE=launch:
        // a k_topk_merge launch after each step (A/B); "fallback": the in-step
        // workers skip (a test hook). Read per call (tests switch it); the lists
        // were cleared above.
        uint32_t k = 0, in_tag = 0, target = 0;
        for (uint32_t s0 = 0, nb = 0; s0 < n_pods; s0 += nb, ++k) {
            nb = std::min(batch_at(s0), n_pods - s0);
            const uint32_t cur = k & 1u, nxt = cur ^ 1u;
            const uint32_t s1 = s0 + nb, nn = s1 < n_pods ? std::min(batch_at(s1), n_pods - s1) : 0u;
            unsigned long long *tk = c->d_tile_keys + cells_per_set * seq_topk() * cur;
            unsigned long long *tk1 = c->d_tile_keys + cells_per_set * seq_topk() * nxt;
            uint32_t *tf = c->d_tile_flags + cells_per_set * cur, *tf1 = c->d_tile_flags + cells_per_set * nxt;
            SeqMergeIO mio;
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
            // diagnostic builds: timeline of steps 0 .. kTimelineSteps - 1 (MS_TIMELINE=<file>)
            static const bool want_tl = getenv("MS_TIMELINE") != nullptr;
            if (want_tl && !c->d_tl &&
                hipMalloc((void **)&c->d_tl, (size_t)kTimelineSteps * kTimelineWgs * 8 * 8) == hipSuccess)
                MS_HIP(c, hipMemsetAsync(c->d_tl, 0, (size_t)kTimelineSteps * kTimelineWgs * 8 * 8, s));
#endif
            mio.tl = c->d_tl;
            mio.tl_step = k;
            mio.in_tags = c->d_merge_tags + SB * cur;
            mio.in_tag = in_tag;
            mio.ctr = c->d_merge_ctr;
            mio.target = target;
            const bool in_step = want_instep && seq_step_merges(tq, n_tiles, nn);
            if (in_step) {
                if (++c->merge_tag == 0) ++c->merge_tag;  // (0: no tag)
                mio.top = c->d_top4 + (size_t)SB * seq_topk() * nxt;
                mio.spec = c->d_spec + SB * nxt;
                mio.spec_flags = c->d_spec_flags + SB * nxt;
                mio.recs = c->d_top4_rec + recs_per_set * nxt;
                mio.ext = top_ext + (size_t)SB * seq_topk() * nxt;
                mio.tags = c->d_merge_tags + SB * nxt;
                mio.tag = c->merge_tag;
                mio.skip = merge_mode == "fallback" ? 1 : 0;
            }
            MS_HIP(c, launch_seq_step(tq, rows, n_tiles, seed32, d_pods + s0, nb, tk, tf, c->d_spec + SB * cur,
                                      c->d_spec_flags + SB * cur, c->d_top4 + (size_t)SB * seq_topk() * cur,
                                      c->d_top4_rec + recs_per_set * cur,
                                      k ? c->d_prev + prev_words * nxt : nullptr,
                                      k ? c->d_prev_rec + prev_fields * nxt : nullptr, c->d_prev + prev_words * cur,
                                      c->d_prev_rec + prev_fields * cur, d_res + s0, c->d_overflow,
                                      nn ? d_pods + s1 : nullptr, nn, tk1, tf1, c->num_cus, s,
                                      top_ext + (size_t)SB * seq_topk() * cur, &mio));
            target = mio.target;
            in_tag = in_step ? mio.tag : 0u;
            if (nn && !in_step)
                MS_HIP(c, launch_topk_merge(tk1, tf1, nn, n_tiles, c->d_top4 + (size_t)SB * seq_topk() * nxt,
                                            c->d_spec + SB * nxt, c->d_spec_flags + SB * nxt, c->t,
                                            c->d_top4_rec + recs_per_set * nxt, s,
                                            top_ext + (size_t)SB * seq_topk() * nxt));
        }
        return MS_OK;
    }
}

// Plugin sets whose filters and scores read no mutable node state (NU, NN,
// NodeAffinity): a bind never changes a later pod's outcome, so chunks of a
// call, or the queue-order loop, equal one batched sweep.
bool plugins_stateless(const ms_ctx *c) { return c->cfg.plugin_set != MS_PLUGINS_NU_NRF_NN_LA; }

// Pod / result staging for at least n pods (grown on demand; hipFree
// synchronises the device, so no in-flight call still uses the old buffers).
int ensure_stage(ms_ctx *c, uint32_t n) {
    if (n <= c->stage_cap) return MS_OK;
    void *dev[] = {c->d_pods, c->d_res};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    if (c->h_pods) (void)hipHostFree(c->h_pods);
    if (c->h_res) (void)hipHostFree(c->h_res);
    c->d_pods = nullptr;
    c->d_res = nullptr;
    c->h_pods = nullptr;
    c->h_res = nullptr;
    c->stage_cap = 0;
    if (hipHostMalloc((void **)&c->h_pods, (size_t)n * sizeof(ms_pod_rec)) != hipSuccess ||
        hipHostMalloc((void **)&c->h_res, (size_t)n * sizeof(ms_result)) != hipSuccess ||
        hipMalloc((void **)&c->d_pods, (size_t)n * sizeof(ms_pod_rec)) != hipSuccess ||
        hipMalloc((void **)&c->d_res, (size_t)n * sizeof(ms_result)) != hipSuccess)
        return fail(c, MS_E_OOM, "pod staging");
    c->stage_cap = n;
    return MS_OK;
}

// MS_PLUGINS_NU_TT_NN scratch: `need` bytes (summaries or the two-pass cycle's).
int ensure_tt(ms_ctx *c, size_t need) {
    if (need <= c->tt_bytes) return MS_OK;
    // (growing: the previous scratch may still be read by work on the sweep,
    // collective or decode streams of a node-sharded cycle)
    if (c->d_tt) MS_HIP(c, hipDeviceSynchronize());
    if (c->d_tt) (void)hipFree(c->d_tt);
    c->d_tt = nullptr;
    c->tt_bytes = 0;
    if (hipMalloc(&c->d_tt, need) != hipSuccess) return fail(c, MS_E_OOM, "TaintToleration scratch");
    c->tt_bytes = need;
    return MS_OK;
}

// The batch's per-pod summaries of every row segment, merged in LIST order into
// out (this shard's summary), or finalised into results (the single-shard
// cycle; commit: the winners' NodeInfo.AddPod). Chunks of batch_cap pods.
// A single-shard cycle (results) runs the two-pass bit-sliced form (round 5,
// launch_tt2_cycle); the shard summaries (out, ms_tt_summaries_device) the
// per-pair summary sweep.
int tt_cycle_locked(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *d_pods, void *out, ms_result *results, int commit,
                    hipStream_t s) {
    const bool two_pass = !out;
    const uint32_t B = c->batch_cap, segs = tt_segments(c->rows_dev), cap = std::min(B, n_pods);
    int rc = ensure_tt(c, two_pass ? tt2_scratch_bytes(c->rows_dev, cap)
                                   : (size_t)segs * cap * MS_TT_SUMMARY_BYTES);
    if (rc) return rc;
    if (!c->ev_tt) MS_HIP(c, hipEventCreateWithFlags(&c->ev_tt, hipEventDisableTiming));
    // the previous cycle's sweep/combine on another stream still owns d_tt
    if (c->tt_stream && c->tt_stream != s) MS_HIP(c, hipStreamWaitEvent(s, c->ev_tt, 0));
    const uint32_t seed32 = seed32_of(c->cfg.seed);
    if (two_pass) MS_HIP(c, launch_tt2_planes(c->t, c->rows_dev, c->d_tt, s));
    for (uint32_t s0 = 0; s0 < n_pods; s0 += B) {
        const uint32_t nb = std::min(B, n_pods - s0);
        if (two_pass) {
            MS_HIP(c, launch_tt2_cycle(c->t, c->rows_dev, d_pods + s0, nb, seed32, c->d_tt, cap, results + s0, commit,
                                       s));
            continue;
        }
        MS_HIP(c, launch_tt_sweep(c->t, c->rows_dev, d_pods + s0, nb, seed32, c->d_tt, s));
        MS_HIP(c, launch_tt_combine(c->d_tt, nb, segs, d_pods + s0, nb, seed32,
                                    out ? static_cast<char *>(out) + (size_t)s0 * MS_TT_SUMMARY_BYTES : nullptr,
                                    out ? nullptr : results + s0, c->t, commit, s));
    }
    MS_HIP(c, hipEventRecord(c->ev_tt, s));
    c->tt_stream = s;
    return MS_OK;
}

int tt_summaries_locked(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *d_pods, void *out, hipStream_t s) {
    return tt_cycle_locked(c, n_pods, d_pods, out, nullptr, 0, s);
}

// MS_PLUGINS_NU_NN_NAM: pods per chunk and the per-class passes' layout. A chunk
// holds at most min(pods, 2 (n_sets + 1)) classes, and the per-class scores F
// take classes x rows bytes: chunks shrink so F stays within kNamFBudget (only
// with very many term sets; 64 sets at 50k rows: 130 classes, 6.5 MB).
constexpr size_t kNamFBudget = 512ull << 20;

uint32_t nam_chunk(const ms_ctx *c, uint32_t n_pods) {
    uint32_t nb = std::min(c->batch_cap, n_pods);
    const size_t rows = std::max<uint32_t>(64u, c->rows_dev);
    const uint32_t cls_sets = 2u * (c->n_terms + 1u);
    if ((size_t)std::min(nb, cls_sets) * rows > kNamFBudget)
        nb = std::max<uint32_t>(256u, (uint32_t)std::min<size_t>(nb, kNamFBudget / rows));
    return std::max(1u, nb);
}

NamLayout nam_layout_for(const ms_ctx *c, uint32_t nb) {
    return nam_layout(c->rows_dev, std::max(1u, std::min(nb, 2u * (c->n_terms + 1u))));
}

// Scratch for chunks of nb pods (NamLayout), plus one record (the later shards'
// table) and one byte (an earlier shard has a non-zero node) per pod. Every NAM
// call runs on the context stream or chains back into it, so one scratch serves
// them in order.
int ensure_nam(ms_ctx *c, uint32_t nb) {
    const size_t need = nam_scratch_bytes(nam_layout_for(c, nb), nb, c->n_terms) + (size_t)nb * (MS_NAM_SEG_BYTES + 1) + 512;
    if (need <= c->nam_bytes) return MS_OK;
    // (growing: a NodeAffinity call on a caller stream may still read the tables; as ensure_tt)
    if (c->d_nam) MS_HIP(c, hipDeviceSynchronize());
    if (c->d_nam) (void)hipFree(c->d_nam);
    c->d_nam = nullptr;
    c->nam_bytes = 0;
    if (hipMalloc(&c->d_nam, need) != hipSuccess) return fail(c, MS_E_OOM, "NodeAffinity scratch");
    c->nam_bytes = need;
    return MS_OK;
}
// The per-pod shard inputs (after: nb records, m_in: nb bytes) past the layout's scratch.
char *nam_after(ms_ctx *c, uint32_t nb) {
    const size_t o = (nam_scratch_bytes(nam_layout_for(c, nb), nb, c->n_terms) + 255u) & ~size_t(255);
    return static_cast<char *>(c->d_nam) + o;
}

// This shard's packed keys of nb pods into keys (scratch sized for the chunk):
// per class its rows' normalised scores under the later segments' and (after /
// m_in, node shards) the later shards' rescales, then per pod the best key.
int nam_keys_locked(ms_ctx *c, uint32_t nb, const ms_pod_rec *d_pods, const void *after, const uint8_t *m_in,
                    unsigned long long *keys, hipStream_t s) {
    if (c->rows_dev == 0) {
        MS_HIP(c, launch_fill_keys(keys, nb, 0ull, s));
        return MS_OK;
    }
    MS_HIP(c, launch_nam_keys(c->t, c->rows_dev, d_pods, nb, c->d_terms, c->n_terms, seed32_of(c->cfg.seed), c->w_nn,
                              c->w_na, after, m_in, c->present_dev ? 1u : 0u, nam_layout_for(c, nb), c->d_nam, keys,
                              s));
    return MS_OK;
}

// The single-shard NAM cycle: keys per chunk, decode, and with commit each
// winner's NodeInfo.AddPod (stateless: no later pod reads it).
int nam_cycle_locked(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *d_pods, ms_result *d_res, int commit,
                     hipStream_t s) {
    const uint32_t B = nam_chunk(c, n_pods);
    int rc = ensure_nam(c, B);
    if (rc) return rc;
    for (uint32_t s0 = 0; s0 < n_pods; s0 += B) {
        const uint32_t nb = std::min(B, n_pods - s0);
        rc = nam_keys_locked(c, nb, d_pods + s0, nullptr, nullptr, c->d_keys, s);
        if (rc) return rc;
        MS_HIP(c, launch_decode(d_pods + s0, nb, c->d_keys, nullptr, c->present_dev, d_res + s0, s));
        if (commit) MS_HIP(c, launch_apply_binds(c->t, d_pods + s0, nb, d_res + s0, s));
    }
    return MS_OK;
}

// This shard's keys (and filter flags for the resource-aware set) for a batch.
int sweep_locked(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *d_pods, unsigned long long *keys, uint32_t *flags,
                 hipStream_t s, hipEvent_t done) {
    const uint32_t seed32 = seed32_of(c->cfg.seed);
    if (c->cfg.plugin_set == MS_PLUGINS_NU_TT_NN)
        return fail(c, MS_E_INVAL, "TaintToleration shards combine by summaries (ms_tt_summaries_device), not keys");
    if (c->cfg.plugin_set == MS_PLUGINS_NU_NN_NAM)
        return fail(c, MS_E_INVAL, "multi-term NodeAffinity shards exchange rescale tables first "
                                   "(ms_nam_segment_device, ms_nam_keys_device)");
    if (c->cfg.plugin_set == MS_PLUGINS_NU_NN) {
        MS_HIP(c, launch_sweep_pp(c->t, c->rows_dev, d_pods, n_pods, seed32, keys, nullptr, c->present_dev,
                                  c->num_cus, s, 0, done));
        return MS_OK;
    } else if (c->cfg.plugin_set == MS_PLUGINS_NU_NN_NA) {
        MS_HIP(c, launch_fill_keys(keys, n_pods, c->present_dev ? kKeyListed : 0ull, s));
        MS_HIP(c, hipMemsetAsync(flags, 0, sizeof(uint32_t) * n_pods, s));
        MS_HIP(c, launch_sweep_na(c->t, c->rows_dev, d_pods, n_pods, seed32, c->w_nn, c->w_na, keys, flags,
                                  c->num_cus, s));
    } else {
        MS_HIP(c, launch_fill_keys(keys, n_pods, c->present_dev ? kKeyListed : 0ull, s));
        if (flags) MS_HIP(c, hipMemsetAsync(flags, 0, sizeof(uint32_t) * n_pods, s));
        MS_HIP(c, launch_sweep_full(c->t, c->rows_dev, d_pods, n_pods, seed32, keys, flags, c->num_cus, s));
    }
    if (done) MS_HIP(c, hipEventRecord(done, s));
    return MS_OK;
}

// Combined keys (+ flags / anchors) -> ms_result for this context's plugin set.
hipError_t decode_for(const ms_ctx *c, const ms_pod_rec *pods, uint32_t n, const unsigned long long *keys,
                      const uint32_t *flags, uint32_t present, ms_result *out, hipStream_t s) {
    if (c->cfg.plugin_set == MS_PLUGINS_NU_NN_NA)
        return launch_decode_na(pods, n, keys, flags, present, seed32_of(c->cfg.seed), c->w_nn, c->w_na, out, s);
    return launch_decode(pods, n, keys, flags, present, out, s);
}

// The stateless cycle of a batch on a single-shard context: filter + score +
// selectHost + decode into results; commit != 0 also commits every winner's
// bind (NodeInfo.AddPod). NU+NN with K1 pp is one fused launch for the whole
// batch, binds included (it needs key scratch only above kPpMaxFusedRows
// rows); otherwise batch_cap chunks are swept into the context's key/flag
// scratch, then decoded (and their binds applied).
// done (optional): recorded on s after the call's last launch (by the fused
// K1 dispatch itself when the cycle is that one launch).
int select_locked(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *d_pods, ms_result *d_res, hipStream_t s,
                  int commit = 0, hipEvent_t done = nullptr) {
    const uint32_t B = c->batch_cap;
    const bool fused = c->cfg.plugin_set == MS_PLUGINS_NU_NN;
    if (c->cfg.plugin_set == MS_PLUGINS_NU_NN_NAM) {
        int rc = nam_cycle_locked(c, n_pods, d_pods, d_res, commit, s);
        if (rc) return rc;
        if (done) MS_HIP(c, hipEventRecord(done, s));
        return MS_OK;
    }
    if (c->cfg.plugin_set == MS_PLUGINS_NU_TT_NN) {  // (stateless: binds in the combine launch)
        int rc = tt_cycle_locked(c, n_pods, d_pods, nullptr, d_res, commit, s);
        if (rc) return rc;
        if (done) MS_HIP(c, hipEventRecord(done, s));
        return MS_OK;
    }
    if (fused && c->rows_dev <= kPpMaxFusedRows) {
        MS_HIP(c, launch_sweep_pp(c->t, c->rows_dev, d_pods, n_pods, seed32_of(c->cfg.seed), nullptr, d_res,
                                  c->present_dev, c->num_cus, s, commit, done));
        return MS_OK;
    }
    // The resource-aware set reads Requested / pod_count: every chunk must be
    // decided before any bind of the call lands (MS_MODE_BATCHED), so
    // its binds are committed after the last chunk's decode.
    const bool late_commit = commit && !plugins_stateless(c);
    for (uint32_t s0 = 0; s0 < n_pods; s0 += B) {
        const uint32_t nb = std::min(B, n_pods - s0);
        if (fused) {
            MS_HIP(c, launch_sweep_pp(c->t, c->rows_dev, d_pods + s0, nb, seed32_of(c->cfg.seed), c->d_keys,
                                      d_res + s0, c->present_dev, c->num_cus, s, commit));
            continue;
        }
        const bool want_flags = c->cfg.plugin_set != MS_PLUGINS_NU_NN;
        int rc = sweep_locked(c, nb, d_pods + s0, c->d_keys, want_flags ? c->d_flags : nullptr, s);
        if (rc) return rc;
        MS_HIP(c, decode_for(c, d_pods + s0, nb, c->d_keys, want_flags ? c->d_flags : nullptr, c->present_dev,
                             d_res + s0, s));
        if (commit && !late_commit) MS_HIP(c, launch_apply_binds(c->t, d_pods + s0, nb, d_res + s0, s));
    }
    if (late_commit) MS_HIP(c, launch_apply_binds(c->t, d_pods, n_pods, d_res, s));
    if (done) MS_HIP(c, hipEventRecord(done, s));
    return MS_OK;
}

// Chunks of ms_schedule_batch's host-array cycle (NU+NN / NA sets, pageable
// copies): chunk i+1's H2D (copy stream; the runtime stages pageable memory on
// the calling thread, which here overlaps chunk i's fused cycle) and chunk i-1's
// D2H overlap chunk i on the context stream; one cross-stream wait per chunk.
constexpr uint32_t kE2eMinChunk = 16384, kE2eChunks = 2;

uint32_t e2e_chunks(uint32_t n) { return std::max(1u, std::min(kE2eChunks, n / kE2eMinChunk)); }

// The per-chunk events of the host-array paths, each created once whichever
// path (zero-copy or chunked copies) runs first (no leak when a
// context switches paths); copies: also the copy-stream events.
int ensure_chunk_events(ms_ctx *c, bool copies) {
    for (int i = 0; i < 4; ++i) {
        if (!c->ev_cyc[i]) MS_HIP(c, hipEventCreateWithFlags(&c->ev_cyc[i], hipEventDisableTiming));
        if (copies && !c->ev_copy[i]) MS_HIP(c, hipEventCreateWithFlags(&c->ev_copy[i], hipEventDisableTiming));
    }
    return MS_OK;
}

int schedule_chunked(ms_ctx *c, const ms_pod_rec *pods, uint32_t n, ms_result *out, uint32_t parts, CallClock &ck) {
    const hipStream_t s = c->stream;
    if (!c->copy_stream) {
        MS_HIP(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
        ck.lap(MS_PH_ALLOC);
    }
    int erc = ensure_chunk_events(c, true);
    if (erc) return erc;
    const hipStream_t cs = c->copy_stream;
    const uint32_t per = cdiv(n, parts);
    auto beg = [&](uint32_t i) { return std::min(n, i * per); };
    auto cnt = [&](uint32_t i) { return beg(i + 1) - beg(i); };
    ck.count(MS_PH_CHUNKS, parts);
    MS_HIP(c, hipMemcpyAsync(c->d_pods, pods, sizeof(ms_pod_rec) * cnt(0), hipMemcpyHostToDevice, s));
    ck.lap(MS_PH_STAGE_IN);
    for (uint32_t i = 0; i < parts; ++i) {
        if (i > 0) MS_HIP(c, hipStreamWaitEvent(s, c->ev_copy[i], 0));
        int rc = select_locked(c, cnt(i), c->d_pods + beg(i), c->d_res + beg(i), s, 1);
        if (rc) return rc;
        MS_HIP(c, hipEventRecord(c->ev_cyc[i], s));
        ck.lap(MS_PH_LAUNCH);
        if (i + 1 < parts) {
            MS_HIP(c, hipMemcpyAsync(c->d_pods + beg(i + 1), pods + beg(i + 1), sizeof(ms_pod_rec) * cnt(i + 1),
                                     hipMemcpyHostToDevice, cs));
            MS_HIP(c, hipEventRecord(c->ev_copy[i + 1], cs));
            ck.lap(MS_PH_STAGE_IN);
        }
        if (i > 0) {
            MS_HIP(c, hipStreamWaitEvent(cs, c->ev_cyc[i - 1], 0));
            MS_HIP(c, hipMemcpyAsync(out + beg(i - 1), c->d_res + beg(i - 1), sizeof(ms_result) * cnt(i - 1),
                                     hipMemcpyDeviceToHost, cs));
            ck.lap(MS_PH_STAGE_OUT);
        }
    }
    MS_HIP(c, hipMemcpyAsync(out + beg(parts - 1), c->d_res + beg(parts - 1), sizeof(ms_result) * cnt(parts - 1),
                             hipMemcpyDeviceToHost, s));
    ck.lap(MS_PH_STAGE_OUT);
    MS_HIP(c, hipStreamSynchronize(cs));
    MS_HIP(c, hipStreamSynchronize(s));
    ck.lap(MS_PH_WAIT);
    return MS_OK;
}

// Pinned coherent staging of compact records (the compact cycle's kernel reads
// the pods from and writes the results to it over PCIe), grown to n.
int ensure_zc(ms_ctx *c, uint32_t n) {
    if (n <= c->z_cap) return MS_OK;
    if (c->h_podz) (void)hipHostFree(c->h_podz);
    if (c->h_resz) (void)hipHostFree(c->h_resz);
    c->h_podz = nullptr;
    c->h_resz = nullptr;
    c->z_cap = 0;
    // coherent (fine-grained): the kernel's reads see this call's host copy and
    // its writes reach host memory with no cache maintenance between calls
    if (hipHostMalloc((void **)&c->h_podz, sizeof(ms_pod_compact) * n, hipHostMallocCoherent) != hipSuccess ||
        hipHostMalloc((void **)&c->h_resz, sizeof(ms_result_compact) * n, hipHostMallocCoherent) != hipSuccess)
        return fail(c, MS_E_OOM, "compact pinned staging");
    c->z_cap = n;
    return MS_OK;
}

// The single-shard NU+NN cycle of a host-array call without runtime (pageable)
// copies: chunk by chunk, the host writes the 8-B compact records K1 reads into
// pinned coherent memory (narrowing 40-B ms_pod_rec, or copying compact ones),
// the compact cycle kernel (one launch per chunk, binds included) reads them
// and writes 8-B results there over PCIe, and the host moves chunk i-1's
// results into the caller's array (widening to ms_result, or copying) while
// chunk i runs. For ms_schedule_batch the pageable copies this replaces cost
// 0.59 ms at config C (the blocking D2H alone ~0.42 ms of host time) and once
// took 7.3 ms (BENCH_r03 e2e.runs[4]; the A/B rerun caught a 6.7 ms pageable
// H2D in the call's stage_in phase, profiles/r04b_e2e_zc_ab.txt);
// MINISCHED_PAGEABLE_E2E=1 restores them (A/B). Chunks: one per 50k pods, at
// most 4. With the fixed-slot K1 (shorter kernels) config C's 100k pods in 2
// chunks overlap the host copies: 0.320 vs 0.328 ms compact, 0.362 vs 0.403 ms
// with 40/24-B records (profiles/r04zb_zc_parts.txt; 3 chunks 0.325 / 0.364;
// round 3, slot-search K1: 4 chunks of 25k cost as much kernel time as their
// overlap saved). MINISCHED_ZC_PARTS overrides the chunk count (1..4).
constexpr uint32_t kZcMinChunk = 50000;
constexpr uint32_t kZcParMin = 16384;  // pods per chunk from which the copies use the pool
template <typename PodIn, typename ResOut>
int schedule_zc(ms_ctx *c, const PodIn *pods, uint32_t n, ResOut *out, CallClock &ck) {
    static_assert(sizeof(ms_pod_compact) <= sizeof(PodIn), "compact pod = the first 8 B of a pod record");
    const hipStream_t s = c->stream;
    int rc = ensure_zc(c, n);
    if (rc) return rc;
    rc = ensure_chunk_events(c, false);
    if (rc) return rc;
    ck.lap(MS_PH_ALLOC);
    MS_HIP(c, hipStreamSynchronize(s));  // (no earlier call still reads h_podz)
    ck.lap(MS_PH_WAIT);
    const uint32_t parts = std::max(1u, std::min(4u, n / kZcMinChunk));
    const uint32_t per = cdiv(n, parts);
    auto beg = [&](uint32_t i) { return std::min(n, i * per); };
    // Host copies split over the caller and the copy pool's 3 helpers (7 measured
    // no better, profiles/r05v_e2e_ab.txt): the first chunk's copy-in and the last
    // one's copy-out are on the call's critical path.
    constexpr unsigned helpers = 3;
    if (per >= kZcParMin && !c->copy_pool) {
        try {  // (no helper threads, e.g. none can be created: the caller copies alone)
            c->copy_pool.reset(new CopyPool(helpers));
        } catch (...) {
            c->copy_pool.reset();
        }
    }
    CopyPool *pool = per >= kZcParMin ? c->copy_pool.get() : nullptr;
    auto par = [&](uint32_t lo, uint32_t hi, const std::function<void(uint32_t, uint32_t)> &fn) {
        if (!pool) {
            fn(lo, hi);
            return;
        }
        pool->run_parts([&](unsigned p, unsigned P) {
            fn(lo + (uint32_t)((uint64_t)(hi - lo) * p / P), lo + (uint32_t)((uint64_t)(hi - lo) * (p + 1) / P));
        });
    };
    auto move_out = [&](uint32_t i) {
        const ms_result_compact *r = c->h_resz;
        par(beg(i), beg(i + 1), [&](uint32_t a, uint32_t b) {
            if constexpr (std::is_same<ResOut, ms_result_compact>::value) {
                std::memcpy(out + a, r + a, sizeof(ms_result_compact) * (b - a));
            } else {
                for (uint32_t j = a; j < b; ++j) {
                    const ms_result_compact x = r[j];
                    out[j] = ms_result{x.node, (int32_t)x.code, (int64_t)x.score, (uint32_t)x.plugin_mask, 0u};
                }
            }
        });
    };
    ++c->ctx_seq;  // binds write the table on the context stream
    ck.count(MS_PH_CHUNKS, parts);
    for (uint32_t i = 0; i < parts; ++i) {
        ms_pod_compact *z = c->h_podz;
        par(beg(i), beg(i + 1), [&](uint32_t a, uint32_t b) {
            if constexpr (std::is_same<PodIn, ms_pod_compact>::value) {
                std::memcpy(z + a, pods + a, sizeof(ms_pod_compact) * (b - a));
            } else {
                for (uint32_t j = a; j < b; ++j) std::memcpy(&z[j], &pods[j], sizeof(ms_pod_compact));
            }
        });
        ck.lap(MS_PH_STAGE_IN);
        MS_HIP(c, launch_sweep_pp_compact(c->t, c->rows_dev, c->h_podz + beg(i), beg(i + 1) - beg(i),
                                          seed32_of(c->cfg.seed), c->h_resz + beg(i), c->present_dev, c->num_cus, s));
        MS_HIP(c, hipEventRecord(c->ev_cyc[i], s));
        ck.lap(MS_PH_LAUNCH);
        if (i > 0) {
            MS_HIP(c, hipEventSynchronize(c->ev_cyc[i - 1]));
            ck.lap(MS_PH_WAIT);
            move_out(i - 1);
            ck.lap(MS_PH_STAGE_OUT);
        }
    }
    MS_HIP(c, hipEventSynchronize(c->ev_cyc[parts - 1]));
    ck.lap(MS_PH_WAIT);
    move_out(parts - 1);
    ck.lap(MS_PH_STAGE_OUT);
    return MS_OK;
}

// This shard's speculative top-4 candidates with records, and its filter flags,
// for a batch of at most MS_SEQ_SHARD_BATCH_MAX pods (ms_seq_candidates_device;
// the in-library node-sharded sequential cycle).
int seq_candidates_locked(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, ms_seq_cand *cands_dev,
                          uint32_t *flags_dev, hipStream_t s) {
    const uint32_t rows = c->rows_dev;
    if (rows == 0) {  // no node listed: no candidates, no rejections
        MS_HIP(c, hipMemsetAsync(cands_dev, 0, sizeof(ms_seq_cand) * kTopKCands * n_pods, s));
        MS_HIP(c, hipMemsetAsync(flags_dev, 0, sizeof(uint32_t) * n_pods, s));
        return MS_OK;
    }
    if (rows > seq_max_rows())
        return fail(c, MS_E_CAPACITY, "ms_seq_candidates_device: at most " + std::to_string(seq_max_rows()) +
                                          " rows per context");
    const uint32_t n_tiles = cdiv(rows, kFullWaveTile);
    int rc = ensure_tiles(c, n_tiles);
    if (rc) return rc;
    const uint32_t seed32 = seed32_of(c->cfg.seed);
    MS_HIP(c, launch_sweep_full_tiles(c->t, rows, pods_dev, n_pods, seed32, c->d_tile_keys, c->d_tile_flags, n_tiles, s));
    MS_HIP(c, launch_topk_merge(c->d_tile_keys, c->d_tile_flags, n_pods, n_tiles, c->d_top4, c->d_spec,
                                c->d_spec_flags, c->t, nullptr, s));
    MS_HIP(c, launch_seq_pack_cands(c->t, c->d_top4, c->d_tile_flags, n_tiles, n_pods, cands_dev, flags_dev, s));
    return MS_OK;
}

bool valid_ctx(const ms_ctx *c) { return c != nullptr; }

}  // namespace msgpu

extern "C" {

int ms_abi_version(void) { return MS_ABI_VERSION; }

int ms_device_count(int *out) {
    if (!out) return MS_E_INVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *out = n;
    return MS_OK;
}

int ms_create(const ms_config *cfg, ms_ctx **out) {
    if (!cfg || !out) return fail(nullptr, MS_E_INVAL, "ms_create: null argument");
    *out = nullptr;
    if (cfg->plugin_set != MS_PLUGINS_NU_NN && cfg->plugin_set != MS_PLUGINS_NU_NRF_NN_LA &&
        cfg->plugin_set != MS_PLUGINS_NU_NN_NA && cfg->plugin_set != MS_PLUGINS_NU_TT_NN &&
        cfg->plugin_set != MS_PLUGINS_NU_NN_NAM)
        return fail(nullptr, MS_E_INVAL, "ms_create: unknown plugin_set");
    const uint32_t w0 = cfg->score_weight[0] ? cfg->score_weight[0] : 1u;
    const uint32_t w1 = cfg->score_weight[1] ? cfg->score_weight[1] : 1u;
    if (cfg->plugin_set != MS_PLUGINS_NU_NN_NA && cfg->plugin_set != MS_PLUGINS_NU_NN_NAM && (w0 != 1 || w1 != 1))
        return fail(nullptr, MS_E_INVAL, "ms_create: score weights apply to MS_PLUGINS_NU_NN_NA / _NAM only");
    if (w0 * 10u + w1 * 100u >= 2048u)
        return fail(nullptr, MS_E_INVAL, "ms_create: weighted score must stay below 2048 (packed key)");
    if (cfg->max_nodes == 0 || (uint64_t)cfg->node_base + cfg->max_nodes > (uint64_t)MS_MAX_ORDINAL + 1)
        return fail(nullptr, MS_E_INVAL, "ms_create: node range must be non-empty and end at or below 0xFFFFF");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(nullptr, MS_E_NODEV, "ms_create: no HIP device visible");
    if (cfg->device < 0 || cfg->device >= ndev) return fail(nullptr, MS_E_NODEV, "ms_create: device out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess)
        return fail(nullptr, MS_E_NODEV, "ms_create: hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(nullptr, MS_E_NODEV, std::string("ms_create: built for gfx950, device is ") + prop.gcnArchName);

    ms_ctx *c = new (std::nothrow) ms_ctx();
    if (!c) return fail(nullptr, MS_E_OOM, "ms_create: host allocation");
    c->cfg = *cfg;
    if (c->cfg.max_batch == 0) c->cfg.max_batch = 1u << 16;
    c->num_cus = prop.multiProcessorCount;
    c->w_nn = w0;
    c->w_na = w1;
    c->batch_cap = c->cfg.max_batch;
    c->present.assign(cfg->max_nodes, 0);

    auto bail = [&](int code, const char *what) {
        std::string m = std::string("ms_create: ") + what;
        free_all(c);
        delete c;
        return fail(nullptr, code, m);
    };
    if (hipSetDevice(cfg->device) != hipSuccess) return bail(MS_E_HIP, "hipSetDevice");
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(MS_E_HIP, "hipStreamCreate");
    const size_t n = cfg->max_nodes;
    NodeTable &t = c->t;
    t.cap = cfg->max_nodes;
    t.base = cfg->node_base;
#ifndef MS_TABLE_ONE_ALLOC
#define MS_TABLE_ONE_ALLOC 1
#endif
    bool ok;
    if (MS_TABLE_ONE_ALLOC) {
        // Every column in one allocation, 2 MB-rounded: the validator's write-back
        // stores one scattered row per lane into five of them each step, and
        // separate allocations spread those rows over many more translation entries.
        void **cols[] = {(void **)&t.flags,     (void **)&t.digit,     (void **)&t.zone,    (void **)&t.label2,
                         (void **)&t.taints,    (void **)&t.allowed_pods, (void **)&t.pod_count, (void **)&t.alloc_cpu,
                         (void **)&t.alloc_mem, (void **)&t.req_cpu,   (void **)&t.req_mem, (void **)&t.nz_cpu,
                         (void **)&t.nz_mem};
        const size_t bytes[] = {n + kColumnPad, n + kColumnPad, n + kColumnPad, n + kColumnPad, n * 4, n * 4, n * 4,
                                n * 8,          n * 8,          n * 8,          n * 8,          n * 8, n * 8};
        static_assert(sizeof(cols) / sizeof(cols[0]) == sizeof(bytes) / sizeof(bytes[0]), "one size per column");
        size_t off[sizeof(bytes) / sizeof(bytes[0])], total = 0;
        for (size_t i = 0; i < sizeof(bytes) / sizeof(bytes[0]); ++i) {
            off[i] = total;
            total += (bytes[i] + 255) & ~(size_t)255;
        }
        total = (total + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
        ok = hipMalloc(&c->d_table, total) == hipSuccess;
        if (ok)
            for (size_t i = 0; i < sizeof(bytes) / sizeof(bytes[0]); ++i)
                *cols[i] = static_cast<char *>(c->d_table) + off[i];
    } else {
        ok = hipMalloc((void **)&t.flags, n + kColumnPad) == hipSuccess &&
             hipMalloc((void **)&t.digit, n + kColumnPad) == hipSuccess &&
             hipMalloc((void **)&t.zone, n + kColumnPad) == hipSuccess &&
             hipMalloc((void **)&t.label2, n + kColumnPad) == hipSuccess &&
             hipMalloc((void **)&t.taints, n * 4) == hipSuccess &&
             hipMalloc((void **)&t.allowed_pods, n * 4) == hipSuccess &&
             hipMalloc((void **)&t.pod_count, n * 4) == hipSuccess &&
             hipMalloc((void **)&t.alloc_cpu, n * 8) == hipSuccess &&
             hipMalloc((void **)&t.alloc_mem, n * 8) == hipSuccess &&
             hipMalloc((void **)&t.req_cpu, n * 8) == hipSuccess &&
             hipMalloc((void **)&t.req_mem, n * 8) == hipSuccess &&
             hipMalloc((void **)&t.nz_cpu, n * 8) == hipSuccess &&
             hipMalloc((void **)&t.nz_mem, n * 8) == hipSuccess;
    }
    t.gcap = (uint32_t)((n + kGroupRows - 1) / kGroupRows);
    ok = ok && hipMalloc((void **)&t.planes, sizeof(uint32_t) * kPlanes * t.gcap) == hipSuccess;
    if (!ok) return bail(MS_E_OOM, "node table allocation");
    const size_t b = c->batch_cap;
    ok = ensure_stage(c, c->batch_cap) == MS_OK &&
         hipMalloc((void **)&c->d_keys, b * sizeof(unsigned long long)) == hipSuccess &&
         hipMalloc((void **)&c->d_flags, b * sizeof(uint32_t)) == hipSuccess &&
         hipMalloc((void **)&c->d_one, sizeof(ms_pod_rec)) == hipSuccess &&
         hipMalloc((void **)&c->d_overflow, kStatsBytes) == hipSuccess;
    if (!ok) return bail(MS_E_OOM, "staging allocation");
    if (launch_init_table(t, c->stream) != hipSuccess || launch_build_planes(t, nullptr, 0, c->stream) != hipSuccess)
        return bail(MS_E_HIP, "table init launch");
    if (hipMemsetAsync(c->d_overflow, 0, kStatsBytes, c->stream) != hipSuccess) return bail(MS_E_HIP, "memset");
    if (hipStreamSynchronize(c->stream) != hipSuccess) return bail(MS_E_HIP, "table init");
    *out = c;
    return MS_OK;
}

int ms_destroy(ms_ctx *c) {
    if (!c) return MS_E_INVAL;
#ifdef MS_VSTAMPS
    {
        uint32_t st[64] = {};
        (void)hipSetDevice(c->cfg.device);
        (void)hipStreamSynchronize(c->stream);
        if (hipMemcpy(st, c->d_overflow, kStatsBytes, hipMemcpyDeviceToHost) == hipSuccess) {
            const uint64_t *cy = reinterpret_cast<const uint64_t *>(st + 8);
            std::fprintf(stderr,
                         "MS_VSTAMPS pods=%u slow=%u tile_scans=%u misses=%u recomputes=%u resweeps=%u rounds=%u cycles: prologue=%llu "
                         "group=%llu prologue_loads=%llu slow=%llu rounds=%llu epilogue=%llu first_slow=%llu round_cand=%llu "
                         "round_claim=%llu | step waves (10 ns): validator=%llu sweep_sum=%llu sweep_waves=%llu | epilogue "
                         "parts: counters=%llu compaction=%llu writeback=%llu | in-step merge (10 ns, summed from each "
                         "workgroup's start): swept=%llu waited=%llu merged=%llu workers=%llu wg_counted=%llu\n",
                         st[3], st[5], st[6], st[4], st[2], st[1], st[7], (unsigned long long)cy[0], (unsigned long long)cy[1],
                         (unsigned long long)cy[2], (unsigned long long)cy[3], (unsigned long long)cy[4],
                         (unsigned long long)cy[5], (unsigned long long)cy[6], (unsigned long long)cy[7],
                         (unsigned long long)cy[8], (unsigned long long)cy[9], (unsigned long long)cy[10],
                         (unsigned long long)cy[11], (unsigned long long)cy[12], (unsigned long long)cy[13],
                         (unsigned long long)cy[14], (unsigned long long)cy[15], (unsigned long long)cy[16],
                         (unsigned long long)cy[17], (unsigned long long)cy[18], (unsigned long long)cy[19]);
        }
    }
#endif
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
    {
        const char *tlf = getenv("MS_TIMELINE");
        if (tlf && c->d_tl) {
            // (the last step kernels, on any stream, may still be writing the timeline)
            (void)hipDeviceSynchronize();
            std::vector<unsigned long long> tl((size_t)kTimelineSteps * kTimelineWgs * 8);
            if (hipMemcpy(tl.data(), c->d_tl, tl.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
                if (FILE *f = std::fopen(tlf, "wb")) {
                    std::fwrite(tl.data(), 8, tl.size(), f);
                    std::fclose(f);
                }
            }
            (void)hipFree(c->d_tl);
            c->d_tl = nullptr;
        }
    }
#endif
    if (c->d_tl) (void)hipFree(c->d_tl);
    free_all(c);
    delete c;
    return MS_OK;
}

const char *ms_last_error(const ms_ctx *c) { return c ? c->err.c_str() : g_create_err.c_str(); }

int ms_last_call_profile(const ms_ctx *c, ms_call_profile *out) {
    if (!valid_ctx(c) || !out) return MS_E_INVAL;
    // CallClock writes prof under sched_mu while a call runs: read it under the
    // same lock, so a concurrent reader never sees a torn profile
    std::lock_guard<std::mutex> g(const_cast<ms_ctx *>(c)->sched_mu);
    for (int i = 0; i < MS_CALL_PHASES; ++i) out->ns[i] = c->prof[i];
    return MS_OK;
}

int ms_get_info(const ms_ctx *c, ms_info *out) {
    if (!valid_ctx(c) || !out) return MS_E_INVAL;
    ms_ctx *m = const_cast<ms_ctx *>(c);
    std::lock_guard<std::mutex> g(m->delta_mu);
    out->max_nodes = c->cfg.max_nodes;
    out->node_base = c->cfg.node_base;
    out->present_nodes = c->present_count;
    out->pending_deltas = (uint32_t)c->pending.size();
    out->device = c->cfg.device;
    out->plugin_set = c->cfg.plugin_set;
    out->seed = c->cfg.seed;
    uint32_t st[4] = {0, 0, 0, 0};
    // counters are written on the (non-blocking) context stream
    if (hipSetDevice(c->cfg.device) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess ||
        hipMemcpy(st, c->d_overflow, sizeof(st), hipMemcpyDeviceToHost) != hipSuccess)
        return fail(m, MS_E_HIP, "ms_get_info: counter read-back");
    out->seq_pods = st[3];
    out->seq_resweep_tiles = st[1];
    out->seq_recomputes = st[2];
    out->_pad = st[0];  // non-zero would mean a validator capacity violation
    comm_rank_world(c, &out->comm_rank, &out->comm_world);
    return MS_OK;
}

int ms_nodes_upsert(ms_ctx *c, uint32_t n, const uint32_t *ord, const ms_node_rec *recs) {
    if (!valid_ctx(c) || (n && (!ord || !recs))) return MS_E_INVAL;
    std::lock_guard<std::mutex> g(c->delta_mu);
    for (uint32_t i = 0; i < n; ++i)
        if (ord[i] < c->cfg.node_base || ord[i] - c->cfg.node_base >= c->cfg.max_nodes)
            return fail(c, MS_E_CAPACITY, "ms_nodes_upsert: ordinal " + std::to_string(ord[i]) + " outside shard");
    for (uint32_t i = 0; i < n; ++i) {
        NodeDelta d;
        d.local = ord[i] - c->cfg.node_base;
        d.absent = 0;
        d.rec = recs[i];
        c->pending.push_back(d);
        if (!c->present[d.local]) {
            c->present[d.local] = 1;
            ++c->present_count;
        }
        c->rows_used = std::max(c->rows_used, d.local + 1);
    }
    return MS_OK;
}

int ms_nodes_delete(ms_ctx *c, uint32_t n, const uint32_t *ord) {
    if (!valid_ctx(c) || (n && !ord)) return MS_E_INVAL;
    std::lock_guard<std::mutex> g(c->delta_mu);
    for (uint32_t i = 0; i < n; ++i)
        if (ord[i] < c->cfg.node_base || ord[i] - c->cfg.node_base >= c->cfg.max_nodes)
            return fail(c, MS_E_CAPACITY, "ms_nodes_delete: ordinal " + std::to_string(ord[i]) + " outside shard");
    for (uint32_t i = 0; i < n; ++i) {
        NodeDelta d{};
        d.local = ord[i] - c->cfg.node_base;
        d.absent = 1;
        c->pending.push_back(d);
        if (c->present[d.local]) {
            c->present[d.local] = 0;
            --c->present_count;
        }
    }
    return MS_OK;
}

int ms_nodes_flush(ms_ctx *c) {
    if (!valid_ctx(c)) return MS_E_INVAL;
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    MS_HIP(c, hipStreamSynchronize(c->stream));
    return MS_OK;
}

int ms_nodes_read(ms_ctx *c, uint32_t first, uint32_t n, ms_node_rec *out) {
    if (!valid_ctx(c) || (n && !out)) return MS_E_INVAL;
    if (first < c->cfg.node_base || (uint64_t)first - c->cfg.node_base + n > c->cfg.max_nodes)
        return fail(c, MS_E_CAPACITY, "ms_nodes_read: range outside shard");
    if (n == 0) return MS_OK;
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    ms_node_rec *d = nullptr;
    MS_HIP(c, hipMalloc((void **)&d, sizeof(ms_node_rec) * n));
    hipError_t e = launch_read_rows(c->t, first - c->cfg.node_base, n, d, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(out, d, sizeof(ms_node_rec) * n, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(c, MS_E_HIP, std::string("ms_nodes_read: ") + hipGetErrorString(e));
    return MS_OK;
}

int ms_schedule_batch(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods, int32_t mode, ms_result *out) {
    if (!valid_ctx(c) || (n_pods && (!pods || !out))) return MS_E_INVAL;
    if (mode != MS_MODE_BATCHED && mode != MS_MODE_SEQUENTIAL) return fail(c, MS_E_INVAL, "unknown mode");
    if (n_pods == 0) return MS_OK;
    std::lock_guard<std::mutex> g(c->sched_mu);
    CallClock ck(c);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    ck.lap(MS_PH_LOCK_FLUSH);
    if (c->comm) return comm_schedule_host(c, n_pods, pods, mode, out, &ck);  // node-sharded over the communicator
    if (c->cfg.plugin_set == MS_PLUGINS_NU_NN && c->rows_dev <= kPpMaxFusedRows)
        return schedule_zc(c, pods, n_pods, out, ck);  // (NU+NN: both modes are the batched cycle + binds)
    const hipStream_t s = c->stream;
    ++c->ctx_seq;  // binds below write the table on the context stream
    uint32_t B = c->batch_cap;
    if (mode == MS_MODE_BATCHED && !plugins_stateless(c)) {
        // every pod of the call is decided on the same node state before any of
        // its binds lands: one pass over the whole call (header contract)
        rc = ensure_stage(c, n_pods);
        if (rc) return rc;
        ck.lap(MS_PH_ALLOC);
        B = n_pods;
    }
    // Host arrays go straight to the device (the runtime's own pageable-copy
    // path, 0.56 ms for config C's 4 MB in + 2.4 MB out + cycle, against 0.72 ms
    // through a single-threaded memcpy into the pinned staging buffers;
    // profiles/r02u_e2e_ab.txt). The call waits for its copies before it
    // returns, so no caller (cgo) pointer outlives it.
    for (uint32_t s0 = 0; s0 < n_pods; s0 += B) {
        const uint32_t nb = std::min(B, n_pods - s0);
        MS_HIP(c, hipStreamSynchronize(s));  // h_pods / h_res free to reuse
        ck.lap(MS_PH_WAIT);
        const bool seq_full = (mode == MS_MODE_SEQUENTIAL && c->cfg.plugin_set == MS_PLUGINS_NU_NRF_NN_LA);
        const uint32_t parts = plugins_stateless(c) ? e2e_chunks(nb) : 1u;
        if (parts > 1) {  // (NU+NN / NA: binds never change a later pod's keys, so chunks equal one batch)
            rc = schedule_chunked(c, pods + s0, nb, out + s0, parts, ck);
            if (rc) return rc;
            continue;
        }
        MS_HIP(c, hipMemcpyAsync(c->d_pods, pods + s0, sizeof(ms_pod_rec) * nb, hipMemcpyHostToDevice, s));
        ck.count(MS_PH_CHUNKS);
        ck.lap(MS_PH_STAGE_IN);
        if (seq_full) {
            rc = run_sequential(c, nb, c->d_pods, c->d_res, s);
            if (rc) return rc;
        } else {
            // NU+NN keys never read mutable node state, so the queue-order
            // loop equals the batched sweep; binds are committed after it.
            rc = select_locked(c, nb, c->d_pods, c->d_res, s, 1);
            if (rc) return rc;
        }
        ck.lap(MS_PH_LAUNCH);
        MS_HIP(c, hipMemcpyAsync(out + s0, c->d_res, sizeof(ms_result) * nb, hipMemcpyDeviceToHost, s));
        ck.lap(MS_PH_STAGE_OUT);
        MS_HIP(c, hipStreamSynchronize(s));
        ck.lap(MS_PH_WAIT);
    }
    return MS_OK;
}

int ms_schedule_batch_compact(ms_ctx *c, uint32_t n, const ms_pod_compact *pods, int32_t mode, ms_result_compact *out) {
    if (!valid_ctx(c) || (n && (!pods || !out))) return MS_E_INVAL;
    if (mode != MS_MODE_BATCHED && mode != MS_MODE_SEQUENTIAL) return fail(c, MS_E_INVAL, "unknown mode");
    if (!plugins_stateless(c))
        return fail(c, MS_E_INVAL, "ms_schedule_batch_compact: the resource-aware set needs ms_schedule_batch");
    if (n == 0) return MS_OK;
    std::lock_guard<std::mutex> g(c->sched_mu);
    CallClock ck(c);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    ck.lap(MS_PH_LOCK_FLUSH);
    // Single-shard NU+NN: one launch reading the pods from and writing the
    // results to pinned host memory (8 B each way per pod over PCIe, no copy
    // commands, no widen / narrow passes); the host copies the caller's arrays
    // in and out (the staged path below: node shards, larger tables).
    if (!c->comm && c->cfg.plugin_set == MS_PLUGINS_NU_NN && c->rows_dev <= kPpMaxFusedRows)
        return schedule_zc(c, pods, n, out, ck);
    rc = c->comm ? comm_stage(c, n) : ensure_stage(c, n);
    if (rc) return rc;
    if (n > c->compact_cap) {
        if (c->d_podc) (void)hipFree(c->d_podc);
        if (c->d_resc) (void)hipFree(c->d_resc);
        c->d_podc = nullptr;
        c->d_resc = nullptr;
        c->compact_cap = 0;
        if (hipMalloc((void **)&c->d_podc, sizeof(ms_pod_compact) * n) != hipSuccess ||
            hipMalloc((void **)&c->d_resc, sizeof(ms_result_compact) * n) != hipSuccess)
            return fail(c, MS_E_OOM, "compact staging");
        c->compact_cap = n;
    }
    ck.lap(MS_PH_ALLOC);
    const hipStream_t s = c->stream;
    // 8 B per pod in and out over PCIe; widened / narrowed on the device
    MS_HIP(c, hipMemcpyAsync(c->d_podc, pods, sizeof(ms_pod_compact) * n, hipMemcpyHostToDevice, s));
    ck.lap(MS_PH_STAGE_IN);
    MS_HIP(c, launch_pods_widen(c->d_podc, n, c->d_pods, s));
    if (c->comm) {
        rc = comm_cycle_staged(c, n, mode);
    } else {
        ++c->ctx_seq;  // binds write the table on the context stream
        rc = select_locked(c, n, c->d_pods, c->d_res, s, 1);  // (stateless sets: sequential == batched)
    }
    if (rc) return rc;
    MS_HIP(c, launch_results_narrow(c->d_res, n, c->d_resc, s));
    ck.lap(MS_PH_LAUNCH);
    MS_HIP(c, hipMemcpyAsync(out, c->d_resc, sizeof(ms_result_compact) * n, hipMemcpyDeviceToHost, s));
    ck.lap(MS_PH_STAGE_OUT);
    MS_HIP(c, hipStreamSynchronize(s));
    ck.lap(MS_PH_WAIT);
    return MS_OK;
}

static int bind_common(ms_ctx *c, uint32_t ordinal, const ms_pod_rec *pod, int sign) {
    if (!valid_ctx(c) || !pod) return MS_E_INVAL;
    if (ordinal < c->cfg.node_base || ordinal - c->cfg.node_base >= c->cfg.max_nodes)
        return fail(c, MS_E_CAPACITY, "bind: ordinal outside shard");
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    rc = comm_fence_reads(c, c->stream);  // (the bind writes the table: after in-flight sharded sweeps)
    if (rc < 0) return rc;
    if (rc) ++c->fence_seq;
    // the context stream already waits for earlier caller-stream work (chain_back)
    MS_HIP(c, hipMemcpyAsync(c->d_one, pod, sizeof(ms_pod_rec), hipMemcpyHostToDevice, c->stream));
    MS_HIP(c, launch_bind_one(c->t, ordinal - c->cfg.node_base, c->d_one, sign, c->stream));
    ++c->ctx_seq;
    MS_HIP(c, hipStreamSynchronize(c->stream));
    return MS_OK;
}

int ms_commit_bind(ms_ctx *c, uint32_t ordinal, const ms_pod_rec *pod) { return bind_common(c, ordinal, pod, +1); }
int ms_uncommit_bind(ms_ctx *c, uint32_t ordinal, const ms_pod_rec *pod) { return bind_common(c, ordinal, pod, -1); }

int ms_sweep_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, uint64_t *keys_dev, uint32_t *flags_dev,
                    void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !keys_dev))) return MS_E_INVAL;
    if ((c->cfg.plugin_set == MS_PLUGINS_NU_NRF_NN_LA || c->cfg.plugin_set == MS_PLUGINS_NU_NN_NA) && n_pods &&
        !flags_dev)
        return fail(c, MS_E_INVAL, "ms_sweep_device: flags required for the resource-aware / NodeAffinity plugin sets");
    if (n_pods == 0) return MS_OK;
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    hipStream_t s = pick_stream(c, stream);
    rc = order_after_ctx_stream(c, s);  // deltas were applied on the context stream
    if (rc) return rc;
    // on a caller stream the chain-back event is recorded by the sweep's own dispatch
    hipEvent_t back = nullptr;
    if (s != c->stream) {
        if (!c->ev_back) MS_HIP(c, hipEventCreateWithFlags(&c->ev_back, hipEventDisableTiming));
        back = c->ev_back;
    }
    rc = sweep_locked(c, n_pods, pods_dev, reinterpret_cast<unsigned long long *>(keys_dev), flags_dev, s, back);
    if (rc) return rc;
    return chain_back(c, s, back != nullptr);
}

int ms_select_batch_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, ms_result *results_dev,
                           void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !results_dev))) return MS_E_INVAL;
    if (c->comm)
        return fail(c, MS_E_INVAL, "ms_select_batch_device: single-shard call on a sharded context (ms_sharded_submit)");
    if (n_pods == 0) return MS_OK;
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    hipStream_t s = pick_stream(c, stream);
    rc = order_after_ctx_stream(c, s);
    if (rc) return rc;
    // on a caller stream the chain-back event is recorded by the cycle's own dispatch
    hipEvent_t back = nullptr;
    if (s != c->stream) {
        if (!c->ev_back) MS_HIP(c, hipEventCreateWithFlags(&c->ev_back, hipEventDisableTiming));
        back = c->ev_back;
    }
    rc = select_locked(c, n_pods, pods_dev, results_dev, s, 0, back);
    if (rc) return rc;
    return chain_back(c, s, back != nullptr);
}

int ms_decode_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, const uint64_t *keys_dev,
                     const uint32_t *flags_dev, uint32_t present_nodes, ms_result *results_dev, void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !keys_dev || !results_dev))) return MS_E_INVAL;
    MS_HIP(c, hipSetDevice(c->cfg.device));
    if (c->cfg.plugin_set == MS_PLUGINS_NU_NN_NA && n_pods && !flags_dev)
        return fail(c, MS_E_INVAL, "ms_decode_device: the NodeAffinity anchors (flags) are required for this plugin set");
    if (c->cfg.plugin_set == MS_PLUGINS_NU_TT_NN)
        return fail(c, MS_E_INVAL, "ms_decode_device: TaintToleration shards decode summaries (ms_tt_decode_device)");
    MS_HIP(c, decode_for(c, pods_dev, n_pods, reinterpret_cast<const unsigned long long *>(keys_dev), flags_dev,
                         present_nodes, results_dev, pick_stream(c, stream)));
    return MS_OK;
}

int ms_decode_device_jobs(ms_ctx *c, uint32_t n_jobs, const ms_decode_job *jobs, uint32_t present_nodes,
                          void *stream) {
    if (!valid_ctx(c) || n_jobs > MS_DECODE_MAX_JOBS || (n_jobs && !jobs)) return MS_E_INVAL;
    if (c->cfg.plugin_set == MS_PLUGINS_NU_TT_NN)
        return fail(c, MS_E_INVAL, "ms_decode_device_jobs: TaintToleration shards decode summaries (ms_tt_decode_device)");
    for (uint32_t i = 0; i < n_jobs; ++i)
        if (jobs[i].n_pods && (!jobs[i].pods || !jobs[i].keys || !jobs[i].results)) return MS_E_INVAL;
    if (n_jobs == 0) return MS_OK;
    MS_HIP(c, hipSetDevice(c->cfg.device));
    if (c->cfg.plugin_set == MS_PLUGINS_NU_NN_NA) {  // one launch per job
        for (uint32_t i = 0; i < n_jobs; ++i) {
            if (jobs[i].n_pods && !jobs[i].flags) return fail(c, MS_E_INVAL, "ms_decode_device_jobs: anchors required");
            MS_HIP(c, decode_for(c, jobs[i].pods, jobs[i].n_pods, reinterpret_cast<const unsigned long long *>(jobs[i].keys),
                                 jobs[i].flags, present_nodes, jobs[i].results, pick_stream(c, stream)));
        }
        return MS_OK;
    }
    MS_HIP(c, launch_decode_jobs(jobs, n_jobs, present_nodes, pick_stream(c, stream)));
    return MS_OK;
}

int ms_apply_binds_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, const ms_result *results_dev,
                          void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !results_dev))) return MS_E_INVAL;
    if (n_pods == 0) return MS_OK;
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    const hipStream_t s = pick_stream(c, stream);
    int rc = order_after_ctx_stream(c, s);  // after earlier sweeps and deltas
    if (rc) return rc;
    MS_HIP(c, launch_apply_binds(c->t, pods_dev, n_pods, results_dev, s));
    if (s == c->stream) {
        ++c->ctx_seq;  // table writes on the context stream
        return MS_OK;
    }
    return chain_back(c, s);
}

int ms_schedule_sequential_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, ms_result *results_dev,
                                  void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !results_dev))) return MS_E_INVAL;
    if (n_pods == 0) return MS_OK;
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    hipStream_t s = pick_stream(c, stream);
    rc = order_after_ctx_stream(c, s);  // deltas were applied on the context stream
    if (rc) return rc;
    if (c->comm) {
        rc = comm_schedule_device(c, n_pods, pods_dev, results_dev, s);  // node-sharded over the communicator
    } else if (c->cfg.plugin_set == MS_PLUGINS_NU_NRF_NN_LA) {
        rc = run_sequential(c, n_pods, pods_dev, results_dev, s);
    } else {
        // NU+NN: keys are independent of mutable state -> batched cycle + commit
        rc = select_locked(c, n_pods, pods_dev, results_dev, s, 1);
    }
    if (rc) return rc;
    if (s == c->stream) {
        ++c->ctx_seq;  // binds wrote the table on the context stream
        return MS_OK;
    }
    return chain_back(c, s);
}

int ms_seq_candidates_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, ms_seq_cand *cands_dev,
                             uint32_t *flags_dev, void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !cands_dev || !flags_dev))) return MS_E_INVAL;
    if (c->cfg.plugin_set != MS_PLUGINS_NU_NRF_NN_LA)
        return fail(c, MS_E_INVAL, "ms_seq_candidates_device: the resource-aware plugin set only");
    if (n_pods > MS_SEQ_SHARD_BATCH_MAX) return fail(c, MS_E_INVAL, "ms_seq_candidates_device: batch too large");
    if (n_pods == 0) return MS_OK;
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    hipStream_t s = pick_stream(c, stream);
    rc = order_after_ctx_stream(c, s);
    if (rc) return rc;
    rc = seq_candidates_locked(c, n_pods, pods_dev, cands_dev, flags_dev, s);
    if (rc) return rc;
    return chain_back(c, s);
}

int ms_seq_validate_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, uint32_t n_shards,
                           const ms_seq_cand *cands_all_dev, const uint32_t *flags_all_dev, ms_result *results_dev,
                           uint32_t *n_done_dev, void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !cands_all_dev || !flags_all_dev || !results_dev || !n_done_dev)))
        return MS_E_INVAL;
    if (c->cfg.plugin_set != MS_PLUGINS_NU_NRF_NN_LA)
        return fail(c, MS_E_INVAL, "ms_seq_validate_device: the resource-aware plugin set only");
    if (n_pods > MS_SEQ_SHARD_BATCH_MAX || n_shards == 0 || n_shards > MS_SEQ_MAX_SHARDS)
        return fail(c, MS_E_INVAL, "ms_seq_validate_device: batch or shard count out of range");
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    hipStream_t s = pick_stream(c, stream);
    if (n_pods == 0) {
        MS_HIP(c, hipMemsetAsync(n_done_dev, 0, sizeof(uint32_t), s));
        return MS_OK;
    }
    int rc = order_after_ctx_stream(c, s);  // (deltas are not drained here: the candidates' records must stay current)
    if (rc) return rc;
    if (!c->d_merged) {
        if (hipMalloc((void **)&c->d_merged, sizeof(ms_seq_cand) * kTopKCands * MS_SEQ_SHARD_BATCH_MAX) != hipSuccess ||
            hipMalloc((void **)&c->d_merged_flags, sizeof(uint32_t) * MS_SEQ_SHARD_BATCH_MAX) != hipSuccess)
            return fail(c, MS_E_OOM, "sharded validator scratch");
    }
    MS_HIP(c, launch_seq_validate_rep(c->t, n_pods, pods_dev, seed32_of(c->cfg.seed), n_shards, cands_all_dev,
                                      flags_all_dev, c->d_merged, c->d_merged_flags, results_dev, n_done_dev, s));
    if (s == c->stream) {
        ++c->ctx_seq;
        return MS_OK;
    }
    return chain_back(c, s);
}

int ms_tt_summaries_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, void *summaries_dev, void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !summaries_dev))) return MS_E_INVAL;
    if (c->cfg.plugin_set != MS_PLUGINS_NU_TT_NN)
        return fail(c, MS_E_INVAL, "ms_tt_summaries_device: the TaintToleration plugin set only");
    if (n_pods == 0) return MS_OK;
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    hipStream_t s = pick_stream(c, stream);
    rc = order_after_ctx_stream(c, s);
    if (rc) return rc;
    rc = tt_summaries_locked(c, n_pods, pods_dev, summaries_dev, s);
    if (rc) return rc;
    return chain_back(c, s);
}

int ms_tt_decode_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, uint32_t n_shards,
                        const void *summaries_all_dev, ms_result *results_dev, void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !summaries_all_dev || !results_dev))) return MS_E_INVAL;
    if (c->cfg.plugin_set != MS_PLUGINS_NU_TT_NN)
        return fail(c, MS_E_INVAL, "ms_tt_decode_device: the TaintToleration plugin set only");
    if (n_shards == 0) return fail(c, MS_E_INVAL, "ms_tt_decode_device: no shards");
    if (n_pods == 0) return MS_OK;
    MS_HIP(c, hipSetDevice(c->cfg.device));
    MS_HIP(c, launch_tt_combine(summaries_all_dev, n_pods, n_shards, pods_dev, n_pods, seed32_of(c->cfg.seed), nullptr,
                                results_dev, c->t, 0, pick_stream(c, stream)));
    return MS_OK;
}

// The two-pass TaintToleration cycle over node shards (ms_taint.hip launch_tt2_*):
// chunks of batch_cap pods; each call rebuilds the row planes on its stream.
static int tt2_shard_prologue(ms_ctx *c, uint32_t n_pods, const char *who, hipStream_t &s, bool planes = true) {
    if (c->cfg.plugin_set != MS_PLUGINS_NU_TT_NN)
        return fail(c, MS_E_INVAL, std::string(who) + ": the TaintToleration plugin set only");
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    rc = order_after_ctx_stream(c, s);
    if (rc) return rc;
    rc = ensure_tt(c, tt2_scratch_bytes(c->rows_dev, std::min(c->batch_cap, n_pods)));
    if (rc) return rc;
    if (!c->ev_tt) MS_HIP(c, hipEventCreateWithFlags(&c->ev_tt, hipEventDisableTiming));
    if (c->tt_stream && c->tt_stream != s) MS_HIP(c, hipStreamWaitEvent(s, c->ev_tt, 0));
    if (planes) MS_HIP(c, launch_tt2_planes(c->t, c->rows_dev, c->d_tt, s));
    return MS_OK;
}

static int tt2_shard_epilogue(ms_ctx *c, hipStream_t s) {
    MS_HIP(c, hipEventRecord(c->ev_tt, s));
    c->tt_stream = s;
    return chain_back(c, s);
}

int ms_tt_census_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, void *census_dev, void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !census_dev))) return MS_E_INVAL;
    if (n_pods == 0) return c->cfg.plugin_set == MS_PLUGINS_NU_TT_NN ? MS_OK : MS_E_INVAL;
    std::lock_guard<std::mutex> g(c->sched_mu);
    hipStream_t s = pick_stream(c, stream);
    int rc = tt2_shard_prologue(c, n_pods, "ms_tt_census_device", s);
    if (rc) return rc;
    const uint32_t B = c->batch_cap, cap = std::min(B, n_pods), seed32 = seed32_of(c->cfg.seed);
    for (uint32_t s0 = 0; s0 < n_pods; s0 += B) {
        const uint32_t nb = std::min(B, n_pods - s0);
        MS_HIP(c, launch_tt2_census_shard(c->t, c->rows_dev, pods_dev + s0, nb, seed32, c->d_tt, cap,
                                          static_cast<char *>(census_dev) + (size_t)s0 * MS_TT_CENSUS_BYTES, s));
    }
    return tt2_shard_epilogue(c, s);
}

int ms_tt_pick_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, uint32_t n_shards, uint32_t shard_index,
                      const void *census_all_dev, unsigned long long *keys_dev, void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !census_all_dev || !keys_dev))) return MS_E_INVAL;
    if (n_shards == 0 || shard_index >= n_shards)
        return fail(c, MS_E_INVAL, "ms_tt_pick_device: shard_index must be below n_shards");
    if (n_pods == 0) return c->cfg.plugin_set == MS_PLUGINS_NU_TT_NN ? MS_OK : MS_E_INVAL;
    std::lock_guard<std::mutex> g(c->sched_mu);
    hipStream_t s = pick_stream(c, stream);
    int rc = tt2_shard_prologue(c, n_pods, "ms_tt_pick_device", s);
    if (rc) return rc;
    const uint32_t B = c->batch_cap, cap = std::min(B, n_pods), seed32 = seed32_of(c->cfg.seed);
    for (uint32_t s0 = 0; s0 < n_pods; s0 += B) {
        const uint32_t nb = std::min(B, n_pods - s0);
        MS_HIP(c, launch_tt2_pick_shard(c->t, c->rows_dev, pods_dev + s0, nb, seed32, c->d_tt, cap,
                                        static_cast<const char *>(census_all_dev) + (size_t)s0 * MS_TT_CENSUS_BYTES,
                                        n_pods, n_shards, shard_index, keys_dev + s0, s));
    }
    return tt2_shard_epilogue(c, s);
}

int ms_tt_final_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, uint32_t n_shards,
                       const void *census_all_dev, const unsigned long long *keys_max_dev, ms_result *results_dev,
                       void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !census_all_dev || !keys_max_dev || !results_dev)))
        return MS_E_INVAL;
    if (n_shards == 0) return fail(c, MS_E_INVAL, "ms_tt_final_device: no shards");
    if (n_pods == 0) return c->cfg.plugin_set == MS_PLUGINS_NU_TT_NN ? MS_OK : MS_E_INVAL;
    std::lock_guard<std::mutex> g(c->sched_mu);
    hipStream_t s = pick_stream(c, stream);
    int rc = tt2_shard_prologue(c, n_pods, "ms_tt_final_device", s, false);  // (the final pass reads no planes)
    if (rc) return rc;
    const uint32_t B = c->batch_cap, cap = std::min(B, n_pods), seed32 = seed32_of(c->cfg.seed);
    for (uint32_t s0 = 0; s0 < n_pods; s0 += B) {
        const uint32_t nb = std::min(B, n_pods - s0);
        // (the scratch's plan records: ADVICE r5, its start holds the row planes)
        MS_HIP(c, launch_tt2_final_shard(c->t, c->rows_dev, pods_dev + s0, nb, seed32,
                                         tt2_plans(c->d_tt, c->rows_dev, cap), cap,
                                         static_cast<const char *>(census_all_dev) + (size_t)s0 * MS_TT_CENSUS_BYTES,
                                         n_pods, n_shards, keys_max_dev + s0, results_dev + s0, s));
    }
    return tt2_shard_epilogue(c, s);
}

// A term set in general form -> the device's lookup table (NamTab).
static NamTab nam_tab_of(const ms_nam_term_set_ext &x) {
    NamTab t{};
    for (int k = 0; k < MS_NAM_TERMS; ++k) {
        const ms_pref_term_ext &e = x.term[k];
        if (e.weight == 0) continue;
        for (uint32_t v = 0; v < 256u; ++v) {
            if ((e.mask[0][v >> 5] >> (v & 31u)) & 1u) t.z[v] |= (uint8_t)(1u << k);
            if ((e.mask[1][v >> 5] >> (v & 31u)) & 1u) t.l[v] |= (uint8_t)(1u << k);
        }
    }
    for (uint32_t m = 0; m < 16u; ++m) {
        uint32_t w = 0;
        for (int k = 0; k < MS_NAM_TERMS; ++k)
            if ((m >> k) & 1u) w += x.term[k].weight;
        t.wsum[m] = (uint16_t)w;
    }
    return t;
}

// ms_nam_term_set's {key, value} terms: In [value] (1..254) or Exists (0xFF) on
// one key, all ids on the other; value 0 ("unlabelled") never matches.
static ms_nam_term_set_ext nam_ext_of(const ms_nam_term_set &x) {
    ms_nam_term_set_ext e{};
    for (int k = 0; k < MS_NAM_TERMS; ++k) {
        const ms_pref_term &t = x.term[k];
        if (t.weight == 0 || t.value == 0) continue;
        ms_pref_term_ext &o = e.term[k];
        const int key = t.key ? 1 : 0;
        for (int w = 0; w < 8; ++w) o.mask[1 - key][w] = ~0u;
        if (t.value == 0xFFu) {
            for (int w = 0; w < 8; ++w) o.mask[key][w] = ~0u;
            o.mask[key][0] &= ~1u;
        } else {
            o.mask[key][t.value >> 5] |= 1u << (t.value & 31u);
        }
        o.weight = t.weight;
    }
    return e;
}

static int nam_install(ms_ctx *c, const std::vector<NamTab> &tabs, const char *who) {
    const uint32_t n_sets = (uint32_t)tabs.size();
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    MS_HIP(c, hipDeviceSynchronize());  // (no cycle still reads the previous table; a configuration call)
    if (n_sets > c->terms_cap) {
        if (c->d_terms) (void)hipFree(c->d_terms);
        c->d_terms = nullptr;
        c->terms_cap = 0;
        if (hipMalloc(&c->d_terms, (size_t)n_sets * sizeof(NamTab)) != hipSuccess)
            return fail(c, MS_E_OOM, std::string(who) + ": term table");
        c->terms_cap = n_sets;
    }
    if (n_sets) MS_HIP(c, hipMemcpy(c->d_terms, tabs.data(), (size_t)n_sets * sizeof(NamTab), hipMemcpyHostToDevice));
    c->n_terms = n_sets;
    return MS_OK;
}

int ms_nam_term_sets(ms_ctx *c, uint32_t n_sets, const ms_nam_term_set *sets) {
    if (!valid_ctx(c) || (n_sets && !sets) || n_sets > 0xFFFFu) return MS_E_INVAL;
    if (c->cfg.plugin_set != MS_PLUGINS_NU_NN_NAM)
        return fail(c, MS_E_INVAL, "ms_nam_term_sets: the multi-term NodeAffinity plugin set only");
    std::vector<NamTab> tabs(n_sets);
    for (uint32_t i = 0; i < n_sets; ++i) {
        for (int k = 0; k < MS_NAM_TERMS; ++k) {
            const ms_pref_term &x = sets[i].term[k];
            if (x.key > 1 || x.weight > 100)
                return fail(c, MS_E_INVAL, "ms_nam_term_sets: term key must be 0 or 1 and weight 0..100");
            // (value 0xFF is Exists; an In term names a value id 1..254, so a node label id
            // of 255 matches Exists only: ZoneIds hands out at most 254 ids)
        }
        tabs[i] = nam_tab_of(nam_ext_of(sets[i]));
    }
    return nam_install(c, tabs, "ms_nam_term_sets");
}

int ms_nam_term_sets_ext(ms_ctx *c, uint32_t n_sets, const ms_nam_term_set_ext *sets) {
    if (!valid_ctx(c) || (n_sets && !sets) || n_sets > 0xFFFFu) return MS_E_INVAL;
    if (c->cfg.plugin_set != MS_PLUGINS_NU_NN_NAM)
        return fail(c, MS_E_INVAL, "ms_nam_term_sets_ext: the multi-term NodeAffinity plugin set only");
    std::vector<NamTab> tabs(n_sets);
    for (uint32_t i = 0; i < n_sets; ++i) {
        for (int k = 0; k < MS_NAM_TERMS; ++k)
            if (sets[i].term[k].weight > 100) return fail(c, MS_E_INVAL, "ms_nam_term_sets_ext: weight 0..100");
        tabs[i] = nam_tab_of(sets[i]);
    }
    return nam_install(c, tabs, "ms_nam_term_sets_ext");
}

int ms_nam_segment_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, void *seg_dev, void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !seg_dev))) return MS_E_INVAL;
    if (c->cfg.plugin_set != MS_PLUGINS_NU_NN_NAM)
        return fail(c, MS_E_INVAL, "ms_nam_segment_device: the multi-term NodeAffinity plugin set only");
    if (n_pods == 0) return MS_OK;
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    hipStream_t s = pick_stream(c, stream);
    rc = order_after_ctx_stream(c, s);
    if (rc) return rc;
    const uint32_t B = nam_chunk(c, n_pods);
    rc = ensure_nam(c, B);
    if (rc) return rc;
    for (uint32_t s0 = 0; s0 < n_pods; s0 += B) {
        const uint32_t nb = std::min(B, n_pods - s0);
        char *out = static_cast<char *>(seg_dev) + (size_t)s0 * MS_NAM_SEG_BYTES;
        if (c->rows_dev == 0) {  // no rows: the identity map, no non-zero node
            MS_HIP(c, launch_nam_identity(out, nb, s));
            continue;
        }
        MS_HIP(c, launch_nam_segment(c->t, c->rows_dev, pods_dev + s0, nb, c->d_terms, c->n_terms,
                                     nam_layout_for(c, nb), c->d_nam, out, s));
    }
    return chain_back(c, s);
}

int ms_nam_keys_device(ms_ctx *c, uint32_t n_pods, const ms_pod_rec *pods_dev, uint32_t n_shards, uint32_t shard_index,
                       const void *segs_all_dev, unsigned long long *keys_dev, void *stream) {
    if (!valid_ctx(c) || (n_pods && (!pods_dev || !segs_all_dev || !keys_dev))) return MS_E_INVAL;
    if (c->cfg.plugin_set != MS_PLUGINS_NU_NN_NAM)
        return fail(c, MS_E_INVAL, "ms_nam_keys_device: the multi-term NodeAffinity plugin set only");
    if (n_shards == 0 || shard_index >= n_shards)
        return fail(c, MS_E_INVAL, "ms_nam_keys_device: shard_index must be below n_shards");
    if (n_pods == 0) return MS_OK;
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    int rc = flush_locked(c);
    if (rc) return rc;
    hipStream_t s = pick_stream(c, stream);
    rc = order_after_ctx_stream(c, s);
    if (rc) return rc;
    const uint32_t B = nam_chunk(c, n_pods);
    rc = ensure_nam(c, B);
    if (rc) return rc;
    char *after = nam_after(c, B);
    uint8_t *m_in = reinterpret_cast<uint8_t *>(after + (size_t)B * MS_NAM_SEG_BYTES);
    for (uint32_t s0 = 0; s0 < n_pods; s0 += B) {
        const uint32_t nb = std::min(B, n_pods - s0);
        // the later shards' tables composed, and whether an earlier shard has a non-zero node
        MS_HIP(c, launch_nam_compose(static_cast<const char *>(segs_all_dev) + (size_t)s0 * MS_NAM_SEG_BYTES, n_pods,
                                     n_shards, nb, (int32_t)shard_index, after, m_in, s));
        rc = nam_keys_locked(c, nb, pods_dev + s0, after, m_in, keys_dev + s0, s);
        if (rc) return rc;
    }
    return chain_back(c, s);
}

}  // extern "C"
