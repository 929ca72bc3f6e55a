// ms_comm.cpp — multi-GPU inside the C ABI (include/minisched_gpu.h, "multi-GPU
// inside the library"). A context joined to an RCCL communicator owns one node
// shard per rank and runs the node-sharded cycles with their collectives in the
// library, so the Go scheduleOne (/root/reference/minisched/minisched.go:32-85,
// called from one goroutine, :28-30) drives G GPUs through the same cgo calls
// it uses for one, with no RCCL binding of its own (SURVEY §8(b) Ownership).
//
// Batched cycle (config C; selectHost over the union of the shards,
// minisched.go:304-325): this shard's sweep of the batch (K1 pp, the
// NodeAffinity sweep or the resource sweep) -> ONE grouped ncclReduceScatter
// on the collective stream:
//   keys   uint64 MAX, G x per pods -> this rank's slice of per pods (the keys
//          embed the global ordinal, so MAX is the global argmax);
//          A pod with no feasible node on a shard has key 1 there when the
//          shard lists a node (kKeyListed), so the MAX also carries the NU+NN /
//          NodeAffinity FitError mask: F = 0 with a listed node means
//          NodeUnschedulable rejected every node;
//   flags  NodeResourcesFit set: uint8 MAX of the filter bytes (byte-wise OR =
//          FitError's UnschedulablePlugins over the cluster, :130-137);
//          NodeAffinity set: uint32 MAX of the normalise anchors;
// -> the decode of the slice on the caller's stream. Pipelined: the decodes of
// batch k are enqueued once `depth` later batches were submitted, so batch k's
// collective overlaps their sweeps (RCCL runs one communicator's collectives in
// issue order on the collective stream, so a drain waits for the newest only).
// The sweeps run on the caller's stream, the collectives on the collective
// stream and the decodes on a decode stream, so no sweep waits for a
// collective or a decode (one cross-queue wait per step: the collective on
// its sweep). The sweeps only read the node table; writers (deltas, binds) are
// fenced behind the in-flight ones (comm_fence_reads) instead of every sweep
// being chained into the context stream. MINISCHED_SHARD_STREAMS=2 alternates
// the sweeps over two internal streams instead (two independent streams on
// separate hardware queues overlap one sweep's ramp and tail with the next:
// 55.4 vs 42.9 us per 12.5k-row sweep, tools/probe_streams.py; but the
// library's streams share the process's hardware queues and the extra waits
// made the pipelined step slower: profiles/r03_step_streams_ab.json).
//
// Exact sequential cycle (config E): per window of W pods, every
// shard's speculative top-4 with records (ms_seq_candidates_device) -> one
// grouped ncclAllGather -> the replicated in-order validation on every rank,
// which commits the binds on its own nodes. The queue cursor lives on the
// device (k_seq_window_in / k_seq_window_out), so windows are issued without a
// host round trip; the host reads the cursor once per round of
// ceil(remaining / W) windows (every window decides at least one pod; one
// round suffices unless a window stops early).
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <new>

#include "ms_ctx.h"

// The RCCL entry points. `make comm-loopback` (tests only) builds this file with
// -DMS_COMM_LOOPBACK against an in-process rendezvous of G contexts on one GPU
// (ms_comm_loopback.h), so the world > 1 code below runs on a 1-GPU box; the
// product library calls RCCL itself.
#ifdef MS_COMM_LOOPBACK
#include "ms_comm_loopback.h"
#define CCL(fn) lb_##fn
#else
#define CCL(fn) fn
#endif

namespace msgpu {

namespace {

constexpr uint32_t kPipeMax = 8;  // batch buffer sets: pipeline depth + 1 <= kPipeMax
static_assert(kPipeMax <= kMaxSliceJobs, "a full drain is one slice-decode launch");
static_assert(sizeof(ncclUniqueId) == MS_COMM_ID_BYTES, "ms_comm_id holds an ncclUniqueId");

// One in-flight batch's combine buffers.
struct ShardSlot {
    unsigned long long *keys = nullptr;       // G x cap: this shard's maxima, pod order
    unsigned long long *keys_mine = nullptr;  // cap: the cluster's maxima of this rank's slice
    uint32_t *flags = nullptr, *flags_mine = nullptr;
    // MS_PLUGINS_NU_TT_NN, the two-pass form: this shard's census (G x cap records, pod
    // order), every shard's after the all-gather (G x G x cap, shard-major,
    // stride = the batch), and the slice's plans for the final pass
    void *cen_mine = nullptr, *cen_all = nullptr, *plans = nullptr;
    uint32_t cap = 0;       // pods per slice the buffers hold
    bool used = false;      // a batch went through this slot
    uint64_t dec_gen = 0;   // the drain that decoded its last batch
};

struct Pending {
    uint32_t slot, n, first, count;
    const ms_pod_rec *pods;  // the batch (decode reads pods + first)
    ms_result *results;      // this rank's slice
};

}  // namespace

struct CommState {
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1;
    hipStream_t cs = nullptr;  // collective stream
    hipStream_t ss[2] = {nullptr, nullptr};  // sweep streams, alternating batch by batch
    hipEvent_t ev_swept[kPipeMax] = {}, ev_comb[kPipeMax] = {};
    hipEvent_t ev_ag[kPipeMax] = {};  // TaintToleration two-pass: the slot's census all-gather
    hipEvent_t ev_in = nullptr, ev_ctx = nullptr;  // caller stream -> sweep stream, context stream -> sweep stream
    hipEvent_t ev_drained = nullptr;               // after the newest drain's decodes (decode stream)
    uint64_t drains = 0, cs_drain_seen = 0;        // drains enqueued / the newest the collective stream waited for
    bool two_streams = false;  // MINISCHED_SHARD_STREAMS=2: sweeps alternate over ss[0], ss[1] (A/B)
    bool reads_outstanding = false;                // sweeps since the last fence
    uint64_t ctx_seen = ~0ull;                     // ctx_seq the sweep streams were last ordered after
    hipStream_t ctx_seen_stream = nullptr;         // (and the caller's stream then)
    ShardSlot slot[kPipeMax];
    std::deque<Pending> pending;
    uint64_t submitted = 0;
    uint64_t x_comb_seen = 0;       // x_stream waited for the collectives of submissions < this
    hipStream_t x_stream = nullptr;
    uint32_t depth = 4, group = 4;
    hipStream_t ds = nullptr;           // decode stream (the drains; callers wait on it in ms_sharded_drain)
    hipEvent_t ev_ds = nullptr;
    // node-sharded exact sequential
    uint32_t seq_w = 0;
    ms_pod_rec *win_pods = nullptr;
    ms_result *win_res = nullptr;
    uint32_t *ctl = nullptr;    // {cursor, live, n_done, pad}
    uint32_t *h_ctl = nullptr;  // pinned read-back of the cursor
    ms_seq_cand *cands = nullptr, *cands_all = nullptr, *merged = nullptr;
    uint32_t *sflags = nullptr, *sflags_all = nullptr, *merged_flags = nullptr;
    uint64_t seq_windows = 0, seq_rounds = 0;
    // coalesced submits: a NU+NN submission whose sweep waits to share the next one's launch
    struct Stash {
        bool on = false;
        uint32_t n = 0, si = 0;
        const ms_pod_rec *pods = nullptr;
        ms_result *results = nullptr;
        hipStream_t X = nullptr;
    } stash;
    bool coalesce = true;
    // MINISCHED_HOST_PROF=1: host time of ms_sharded_submit's phases (ns), printed at ms_destroy
    bool host_prof = false;
    uint64_t hp[6] = {0, 0, 0, 0, 0, 0}, hp_calls = 0;
};

namespace {

#define MS_NCCL(c, call)                                                                          \
    do {                                                                                          \
        ncclResult_t r_ = (call);                                                                 \
        if (r_ != ncclSuccess)                                                                    \
            return fail((c), MS_E_RCCL, std::string(#call) + ": " + CCL(ncclGetErrorString)(r_));      \
    } while (0)

void free_slot(ShardSlot &sl) {
    void *p[] = {sl.keys, sl.keys_mine, sl.flags, sl.flags_mine, sl.cen_mine, sl.cen_all, sl.plans};
    for (void *q : p)
        if (q) (void)hipFree(q);
    sl = ShardSlot{};
}

// Buffers of a slot for slices of `per` pods (grown; the slot's previous batch
// has been drained, and hipFree waits for its decode).
int slot_ensure(ms_ctx *c, ShardSlot &sl, uint32_t per) {
    if (per <= sl.cap && sl.keys) return MS_OK;
    const size_t G = (size_t)c->comm->world;
    const uint32_t cap = std::max<uint32_t>(1024u, cdiv(per, 1024u) * 1024u);
    free_slot(sl);
    if (hipMalloc((void **)&sl.keys, G * cap * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc((void **)&sl.keys_mine, cap * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc((void **)&sl.flags, G * cap * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&sl.flags_mine, cap * sizeof(uint32_t)) != hipSuccess ||
        (c->cfg.plugin_set == MS_PLUGINS_NU_TT_NN &&
         (hipMalloc(&sl.cen_mine, G * cap * MS_TT_CENSUS_BYTES) != hipSuccess ||
          hipMalloc(&sl.cen_all, G * G * cap * MS_TT_CENSUS_BYTES) != hipSuccess ||
          hipMalloc(&sl.plans, cap * MS_TT_CENSUS_BYTES) != hipSuccess))) {
        free_slot(sl);
        return fail(c, MS_E_OOM, "sharded combine buffers");
    }
    sl.cap = cap;
    return MS_OK;
}

void slice_of(const CommState &m, uint32_t n, uint32_t &first, uint32_t &count) {
    const uint32_t per = cdiv(n, (uint32_t)m.world);
    first = std::min<uint32_t>(n, (uint32_t)m.rank * per);
    count = std::min<uint32_t>(n, first + per) - first;
}

// Decodes of the oldest k pending batches on the decode stream (after their
// combines). The caller's stream is not involved: a sweep stream that orders
// after the caller's stream would otherwise wait for these combines too.
int drain_locked(ms_ctx *c, size_t k) {
    CommState &m = *c->comm;
    const hipStream_t s = m.ds;
    k = std::min(k, m.pending.size());
    if (k == 0) return MS_OK;
    MS_HIP(c, hipStreamWaitEvent(s, m.ev_comb[m.pending[k - 1].slot], 0));  // collectives run in issue order
    if (c->cfg.plugin_set == MS_PLUGINS_NU_TT_NN) {  // the slice's plans + the MAX of the picks
        for (size_t i = 0; i < k; ++i) {
            const Pending &p = m.pending[i];
            const ShardSlot &sl = m.slot[p.slot];
            MS_HIP(c, launch_tt2_final_shard(c->t, c->rows_dev, p.pods + p.first, p.count, seed32_of(c->cfg.seed),
                                             sl.plans, p.count, static_cast<const char *>(sl.cen_all) +
                                                                    (size_t)p.first * MS_TT_CENSUS_BYTES,
                                             p.n, (uint32_t)m.world, sl.keys_mine, p.results, s));
        }
    } else if (c->cfg.plugin_set == MS_PLUGINS_NU_NN_NA) {
        for (size_t i = 0; i < k; ++i) {
            const Pending &p = m.pending[i];
            const ShardSlot &sl = m.slot[p.slot];
            MS_HIP(c, launch_decode_na(p.pods + p.first, p.count, sl.keys_mine, sl.flags_mine, 0, seed32_of(c->cfg.seed),
                                       c->w_nn, c->w_na, p.results, s));
        }
    } else {
        SliceJob jobs[kMaxSliceJobs];
        const bool nrf = c->cfg.plugin_set == MS_PLUGINS_NU_NRF_NN_LA;
        for (size_t i = 0; i < k; ++i) {
            const Pending &p = m.pending[i];
            const ShardSlot &sl = m.slot[p.slot];
            jobs[i] = SliceJob{p.pods + p.first, sl.keys_mine, nrf ? sl.flags_mine : nullptr, nullptr, p.results,
                               p.count, 0};
        }
        MS_HIP(c, launch_decode_slices(jobs, (uint32_t)k, s));
    }
    ++m.drains;
    for (size_t i = 0; i < k; ++i) m.slot[m.pending[i].slot].dec_gen = m.drains;
    MS_HIP(c, hipEventRecord(m.ev_drained, s));
    m.pending.erase(m.pending.begin(), m.pending.begin() + (long)k);
    return MS_OK;
}

// Everything pending decoded; then `s` waits for the decode stream.
int flush_stash(ms_ctx *c);

int drain_to(ms_ctx *c, hipStream_t s) {
    CommState &m = *c->comm;
    int rc = flush_stash(c);  // (a coalesced submission waiting for a partner)
    if (rc) return rc;
    rc = drain_locked(c, m.pending.size());
    if (rc) return rc;
    MS_HIP(c, hipEventRecord(m.ev_ds, m.ds));
    MS_HIP(c, hipStreamWaitEvent(s, m.ev_ds, 0));
    return MS_OK;
}

using HostClock = std::chrono::steady_clock;
inline void host_tick(CommState &m, int i, HostClock::time_point &t) {
    if (!m.host_prof) return;
    const auto now = HostClock::now();
    m.hp[i] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(now - t).count();
    t = now;
}

// Submissions whose sweep can share a launch with the next one: NU+NN K1
// sweeps of a shard one workgroup holds, on one sweep stream.
bool coalescable(const ms_ctx *c) {
    const CommState &m = *c->comm;
    return m.coalesce && !m.two_streams && c->cfg.plugin_set == MS_PLUGINS_NU_NN && c->rows_dev <= kPpMaxFusedRows;
}

// The sweep stream and slot of the next submission (the slot's buffers sized
// for n pods), ordered after: the caller's stream (its pods), the context
// stream when it wrote the table since (deltas, binds), and the slot's
// previous collective (it read the keys this sweep overwrites).
int prepare_locked(ms_ctx *c, uint32_t n, hipStream_t s, uint32_t &si, hipStream_t &X) {
    CommState &m = *c->comm;
    const uint32_t G = (uint32_t)m.world, per = cdiv(n, G);
    si = (uint32_t)(m.submitted % (m.depth + 1));
    const int xi = (int)(m.submitted & 1u);
    X = m.two_streams ? m.ss[xi] : s;
    ShardSlot &sl = m.slot[si];
    int rc = slot_ensure(c, sl, per);
    if (rc) return rc;
    if (X != s) {
        MS_HIP(c, hipEventRecord(m.ev_in, s));
        MS_HIP(c, hipStreamWaitEvent(X, m.ev_in, 0));
    }
    if (m.ctx_seen != c->ctx_seq || m.ctx_seen_stream != s) {
        MS_HIP(c, hipEventRecord(m.ev_ctx, c->stream));
        MS_HIP(c, hipStreamWaitEvent(X, m.ev_ctx, 0));
        if (m.two_streams) MS_HIP(c, hipStreamWaitEvent(m.ss[xi ^ 1], m.ev_ctx, 0));
        m.ctx_seen = c->ctx_seq;
        m.ctx_seen_stream = s;
    }
    // the slot's previous collective (submission k - depth - 1) read the keys
    // this sweep overwrites. Collectives complete in issue order, so one wait
    // covers all older ones: wait for submission k - L's and skip the next
    // waits it covers. L = 2 (two steps old, normally done, and never the one
    // the previous sweep feeds); with coalesced submits L = 3: k is the first
    // of a pair (then k - 1 and k - 2 are the previous pair, whose collectives
    // follow the previous launch) or k - 3's wait is already on X.
    if (sl.used) {
        const uint64_t k = m.submitted, prev = k - (m.depth + 1);
        const uint32_t L = coalescable(c) ? 3u : 2u;
        if (m.two_streams || m.depth + 1 <= L) {
            MS_HIP(c, hipStreamWaitEvent(X, m.ev_comb[si], 0));
        } else if (m.x_stream != X || m.x_comb_seen <= prev) {
            m.x_stream = X;
            MS_HIP(c, hipStreamWaitEvent(X, m.ev_comb[(k - L) % (m.depth + 1)], 0));
            m.x_comb_seen = k - L + 1;
        }
    }
    ++m.submitted;
    return MS_OK;
}

// The collective of slot si's batch on the collective stream, after the sweep
// event ev (that recorded the batch's sweep) and the drain that decoded the
// slot's previous batch; then the batch joins the pending list (and the oldest
// are decoded once more than `depth` wait).
int collective_locked(ms_ctx *c, uint32_t si, hipEvent_t ev, uint32_t n, const ms_pod_rec *pods, ms_result *results,
                      HostClock::time_point &tp) {
    CommState &m = *c->comm;
    ShardSlot &sl = m.slot[si];
    const uint32_t G = (uint32_t)m.world, per = cdiv(n, G);
    const int ps = c->cfg.plugin_set;
    // one wait covers a whole drain
    if (ev) MS_HIP(c, hipStreamWaitEvent(m.cs, ev, 0));
    if (sl.used && sl.dec_gen > m.cs_drain_seen) {
        MS_HIP(c, hipStreamWaitEvent(m.cs, m.ev_drained, 0));
        m.cs_drain_seen = m.drains;
    }
    sl.used = true;
    host_tick(m, 2, tp);  // events to the collective stream
    ncclResult_t r = ncclSuccess;
    if (ps == MS_PLUGINS_NU_NN || ps == MS_PLUGINS_NU_TT_NN) {  // the keys alone: one call
        r = CCL(ncclReduceScatter)(sl.keys, sl.keys_mine, per, ncclUint64, ncclMax, m.comm, m.cs);
    } else {
        r = CCL(ncclGroupStart)();
        if (r == ncclSuccess) r = CCL(ncclReduceScatter)(sl.keys, sl.keys_mine, per, ncclUint64, ncclMax, m.comm, m.cs);
        if (r == ncclSuccess && ps == MS_PLUGINS_NU_NRF_NN_LA)  // 0/1 bytes: uint8 MAX = OR
            r = CCL(ncclReduceScatter)(sl.flags, sl.flags_mine, (size_t)per * 4, ncclUint8, ncclMax, m.comm, m.cs);
        if (r == ncclSuccess && ps == MS_PLUGINS_NU_NN_NA)  // anchors < 2^21: uint32 MAX
            r = CCL(ncclReduceScatter)(sl.flags, sl.flags_mine, per, ncclUint32, ncclMax, m.comm, m.cs);
        const ncclResult_t r2 = CCL(ncclGroupEnd)();
        if (r == ncclSuccess) r = r2;
    }
    if (r != ncclSuccess) return fail(c, MS_E_RCCL, std::string("sharded combine: ") + CCL(ncclGetErrorString)(r));
    host_tick(m, 3, tp);  // the grouped reduce-scatter
    MS_HIP(c, hipEventRecord(m.ev_comb[si], m.cs));
    Pending p{si, n, 0, 0, pods, results};
    slice_of(m, n, p.first, p.count);
    m.pending.push_back(p);
    int rc = MS_OK;
    if (m.pending.size() > m.depth) rc = drain_locked(c, std::min<size_t>(m.group, m.pending.size()));
    host_tick(m, 4, tp);  // bookkeeping + drains
    return rc;
}

// The stashed submission's sweep alone, then its collective.
int flush_stash(ms_ctx *c) {
    CommState &m = *c->comm;
    if (!m.stash.on) return MS_OK;
    const CommState::Stash st = m.stash;
    m.stash.on = false;
    HostClock::time_point tp = m.host_prof ? HostClock::now() : HostClock::time_point();
    int rc = sweep_locked(c, st.n, st.pods, m.slot[st.si].keys, nullptr, st.X, m.ev_swept[st.si]);
    if (rc) return rc;
    m.reads_outstanding = true;
    return collective_locked(c, st.si, m.ev_swept[st.si], st.n, st.pods, st.results, tp);
}

// MS_PLUGINS_NU_TT_NN, two-pass: the census of this shard on X, the all-gather of
// every shard's on the collective stream, then the picks on X again (the table's
// readers stay on the sweep stream, behind the delta fence ev_swept). The shared
// two-pass scratch (d_tt) passes from sweep stream to sweep stream by ev_tt.
int tt2_sharded_sweep(ms_ctx *c, uint32_t si, uint32_t n, const ms_pod_rec *pods, hipStream_t X) {
    CommState &m = *c->comm;
    ShardSlot &sl = m.slot[si];
    const uint32_t seed32 = seed32_of(c->cfg.seed);
    int rc = ensure_tt(c, tt2_scratch_bytes(c->rows_dev, std::max(1u, n)));
    if (rc) return rc;
    if (!c->ev_tt) MS_HIP(c, hipEventCreateWithFlags(&c->ev_tt, hipEventDisableTiming));
    if (c->tt_stream && c->tt_stream != X) MS_HIP(c, hipStreamWaitEvent(X, c->ev_tt, 0));
    MS_HIP(c, launch_tt2_planes(c->t, c->rows_dev, c->d_tt, X));
    MS_HIP(c, launch_tt2_census_shard(c->t, c->rows_dev, pods, n, seed32, c->d_tt, std::max(1u, n), sl.cen_mine, X));
    MS_HIP(c, hipEventRecord(m.ev_swept[si], X));
    MS_HIP(c, hipStreamWaitEvent(m.cs, m.ev_swept[si], 0));
    if (sl.used && sl.dec_gen > m.cs_drain_seen) {  // the slot's previous final read cen_all
        MS_HIP(c, hipStreamWaitEvent(m.cs, m.ev_drained, 0));
        m.cs_drain_seen = m.drains;
    }
    const ncclResult_t r = CCL(ncclAllGather)(sl.cen_mine, sl.cen_all, (size_t)n * MS_TT_CENSUS_BYTES, ncclUint8,
                                              m.comm, m.cs);
    if (r != ncclSuccess) return fail(c, MS_E_RCCL, std::string("TaintToleration census all-gather: ") +
                                                        CCL(ncclGetErrorString)(r));
    MS_HIP(c, hipEventRecord(m.ev_ag[si], m.cs));
    MS_HIP(c, hipStreamWaitEvent(X, m.ev_ag[si], 0));
    MS_HIP(c, launch_tt2_pick_shard(c->t, c->rows_dev, pods, n, seed32, c->d_tt, std::max(1u, n), sl.cen_all, n,
                                    (uint32_t)m.world, (uint32_t)m.rank, sl.keys, X));
    MS_HIP(c, hipEventRecord(c->ev_tt, X));
    c->tt_stream = X;
    return MS_OK;
}

int submit_locked(ms_ctx *c, uint32_t n, const ms_pod_rec *pods, ms_result *results, hipStream_t s) {
    CommState &m = *c->comm;
    HostClock::time_point tp = m.host_prof ? HostClock::now() : HostClock::time_point();
    if (m.host_prof) ++m.hp_calls;
    const bool co = coalescable(c);
    if (!co) {
        int rc = flush_stash(c);
        if (rc) return rc;
    }
    uint32_t si = 0;
    hipStream_t X = nullptr;
    int rc = prepare_locked(c, n, s, si, X);
    if (rc) return rc;
    host_tick(m, 0, tp);  // ordering of the sweep stream
    if (co && (!m.stash.on || m.stash.X != X)) {
        // Coalesced submits (MINISCHED_SHARD_COALESCE=0 turns it off): this
        // batch's sweep waits for the next submission (or a drain / table
        // writer) and then shares ONE K1 launch with it, so the launch's ramp
        // and drain (~7.5 us at a 12.5k-row shard, tools/probe_fixed.py) are
        // paid once per two batches. Its collective starts after both sweeps.
        rc = flush_stash(c);
        if (rc) return rc;
        m.stash = CommState::Stash{true, n, si, pods, results, X};
        return MS_OK;
    }
    ShardSlot &sl = m.slot[si];
    if (co) {  // the stashed batch and this one in one launch
        const CommState::Stash st = m.stash;
        m.stash.on = false;
        MS_HIP(c, launch_sweep_pp2(c->t, c->rows_dev, st.pods, st.n, m.slot[st.si].keys, pods, n, sl.keys,
                                   seed32_of(c->cfg.seed), c->present_dev, c->num_cus, X, m.ev_swept[si]));
        host_tick(m, 1, tp);  // the sweep launch
        m.reads_outstanding = true;
        rc = collective_locked(c, st.si, m.ev_swept[si], st.n, st.pods, st.results, tp);
        if (rc) return rc;
        return collective_locked(c, si, nullptr, n, pods, results, tp);  // (cs already waits for the sweep)
    }
    const int ps = c->cfg.plugin_set;
    // (ev_swept recorded by the sweep's own dispatch for K1: no separate event
    // packet between consecutive sweeps on X)
    if (ps == MS_PLUGINS_NU_TT_NN) {
        // the two-pass form: this shard's census, every shard's by one all-gather,
        // then this shard's picks for every pod (keys, combined by the reduce-scatter)
        rc = tt2_sharded_sweep(c, si, n, pods, X);
        if (rc == MS_OK && hipEventRecord(m.ev_swept[si], X) != hipSuccess) rc = fail(c, MS_E_HIP, "event record");
    } else {
        rc = sweep_locked(c, n, pods, sl.keys, ps == MS_PLUGINS_NU_NN ? nullptr : sl.flags, X, m.ev_swept[si]);
    }
    if (rc) return rc;
    host_tick(m, 1, tp);  // the sweep launch
    m.reads_outstanding = true;
    return collective_locked(c, si, m.ev_swept[si], n, pods, results, tp);
}

// Sequential-window buffers for windows of w pods.
int seq_ensure(ms_ctx *c, uint32_t w) {
    CommState &m = *c->comm;
    if (w <= m.seq_w) return MS_OK;
    MS_HIP(c, hipDeviceSynchronize());
    void *old[] = {m.win_pods, m.win_res, m.ctl, m.cands, m.cands_all, m.merged, m.sflags, m.sflags_all, m.merged_flags};
    for (void *q : old)
        if (q) (void)hipFree(q);
    if (m.h_ctl) (void)hipHostFree(m.h_ctl);
    m.win_pods = nullptr;
    m.win_res = nullptr;
    m.ctl = m.h_ctl = m.sflags = m.sflags_all = m.merged_flags = nullptr;
    m.cands = m.cands_all = m.merged = nullptr;
    m.seq_w = 0;
    const size_t G = (size_t)m.world, K = kTopKCands;
    if (hipMalloc((void **)&m.win_pods, w * sizeof(ms_pod_rec)) != hipSuccess ||
        hipMalloc((void **)&m.win_res, w * sizeof(ms_result)) != hipSuccess ||
        hipMalloc((void **)&m.ctl, 4 * sizeof(uint32_t)) != hipSuccess ||
        hipHostMalloc((void **)&m.h_ctl, 4 * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&m.cands, w * K * sizeof(ms_seq_cand)) != hipSuccess ||
        hipMalloc((void **)&m.cands_all, G * w * K * sizeof(ms_seq_cand)) != hipSuccess ||
        hipMalloc((void **)&m.merged, w * K * sizeof(ms_seq_cand)) != hipSuccess ||
        hipMalloc((void **)&m.sflags, w * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&m.sflags_all, G * w * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc((void **)&m.merged_flags, w * sizeof(uint32_t)) != hipSuccess)
        return fail(c, MS_E_OOM, "sharded sequential buffers");
    m.seq_w = w;
    return MS_OK;
}

// Pods per window of the node-sharded exact sequential cycle: each window costs
// one all-gather of its candidates (W x 4 x 72 B per rank) and one validator
// launch. MINISCHED_SHARD_SEQ_BATCH overrides (1..256).
uint32_t seq_window() {
    uint32_t w = 128;
    if (const char *e = getenv("MINISCHED_SHARD_SEQ_BATCH")) w = (uint32_t)std::max(1, atoi(e));
    return std::min<uint32_t>(w, MS_SEQ_SHARD_BATCH_MAX);
}

int seq_sharded_locked(ms_ctx *c, uint32_t n, const ms_pod_rec *pods, ms_result *results, hipStream_t s) {
    CommState &m = *c->comm;
    const uint32_t W = seq_window();
    int rc = seq_ensure(c, W);
    if (rc) return rc;
    const uint32_t seed32 = seed32_of(c->cfg.seed);
    MS_HIP(c, hipMemsetAsync(m.ctl, 0, 4 * sizeof(uint32_t), s));
    const size_t cand_bytes = (size_t)W * kTopKCands * sizeof(ms_seq_cand);
    uint32_t known = 0;
    while (known < n) {
        const uint32_t r = cdiv(n - known, W);  // windows that may finish the queue
        for (uint32_t i = 0; i < r; ++i) {
            MS_HIP(c, launch_seq_window_in(pods, n, m.ctl, m.win_pods, W, s));
            rc = seq_candidates_locked(c, W, m.win_pods, m.cands, m.sflags, s);
            if (rc) return rc;
            ncclResult_t e = CCL(ncclGroupStart)();
            if (e == ncclSuccess) e = CCL(ncclAllGather)(m.cands, m.cands_all, cand_bytes, ncclUint8, m.comm, s);
            if (e == ncclSuccess) e = CCL(ncclAllGather)(m.sflags, m.sflags_all, W, ncclUint32, m.comm, s);
            const ncclResult_t e2 = CCL(ncclGroupEnd)();
            if (e == ncclSuccess) e = e2;
            if (e != ncclSuccess) return fail(c, MS_E_RCCL, std::string("sequential all-gather: ") + CCL(ncclGetErrorString)(e));
            MS_HIP(c, launch_seq_validate_rep(c->t, W, m.win_pods, seed32, (uint32_t)m.world, m.cands_all, m.sflags_all,
                                              m.merged, m.merged_flags, m.win_res, m.ctl + 2, s, m.ctl + 1));
            MS_HIP(c, launch_seq_window_out(m.win_res, m.ctl, results, n, s));
            ++m.seq_windows;
        }
        MS_HIP(c, hipMemcpyAsync(m.h_ctl, m.ctl, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        MS_HIP(c, hipStreamSynchronize(s));
        ++m.seq_rounds;
        const uint32_t now = m.h_ctl[0];
        if (now <= known || now > n) return fail(c, MS_E_HIP, "sharded sequential cycle made no progress");
        known = now;
    }
    return MS_OK;
}

// The batched cycle of all n pods with every result on every rank: submit +
// drain (this rank's slice into stage + first), one all-gather of the slices
// (in place: slices are contiguous in pod order), then this shard's binds.
int batched_all_locked(ms_ctx *c, uint32_t n, const ms_pod_rec *pods, ms_result *stage, hipStream_t s, bool commit) {
    CommState &m = *c->comm;
    uint32_t first = 0, count = 0;
    slice_of(m, n, first, count);
    const uint32_t per = cdiv(n, (uint32_t)m.world);
    int rc = submit_locked(c, n, pods, stage + first, s);
    if (rc) return rc;
    rc = drain_to(c, s);
    if (rc) return rc;
    // (a rank whose slice is short or empty sends entries past n: never read)
    const size_t bytes = (size_t)per * sizeof(ms_result);
    MS_NCCL(c, CCL(ncclAllGather)(reinterpret_cast<char *>(stage) + (size_t)m.rank * bytes, stage, bytes, ncclUint8, m.comm, s));
    if (commit) MS_HIP(c, launch_apply_binds(c->t, pods, n, stage, s));  // NodeInfo.AddPod on this shard's winners
    return MS_OK;
}

}  // namespace

void comm_rank_world(const ms_ctx *c, int32_t *rank, int32_t *world) {
    *rank = c->comm ? c->comm->rank : 0;
    *world = c->comm ? c->comm->world : 0;
}

int comm_fence_reads(ms_ctx *c, hipStream_t writer) {
    CommState *m = c->comm;
    if (m && m->stash.on) {  // the stashed batch's sweep reads the table before this writer
        const int rc = flush_stash(c);
        if (rc) return rc;
    }
    if (!m || !m->reads_outstanding) return 0;
    // every sweep in flight is the newest of its slot (a slot is swept again only
    // after the collective that read its previous sweep): wait for each slot's
    for (uint32_t i = 0; i < kPipeMax; ++i)
        if (m->slot[i].used) MS_HIP(c, hipStreamWaitEvent(writer, m->ev_swept[i], 0));
    m->reads_outstanding = false;
    return 1;
}

void comm_free(ms_ctx *c) {
    CommState *m = c->comm;
    if (!m) return;
    if (m->host_prof && m->hp_calls)
        std::fprintf(stderr, "MS_HOST_PROF submits=%llu us/submit: order=%.2f sweep=%.2f events=%.2f rccl=%.2f tail=%.2f\n",
                     (unsigned long long)m->hp_calls, m->hp[0] * 1e-3 / m->hp_calls, m->hp[1] * 1e-3 / m->hp_calls,
                     m->hp[2] * 1e-3 / m->hp_calls, m->hp[3] * 1e-3 / m->hp_calls, m->hp[4] * 1e-3 / m->hp_calls);
    for (hipStream_t q : m->ss)
        if (q) (void)hipStreamSynchronize(q);
    if (m->cs) (void)hipStreamSynchronize(m->cs);
    if (m->ds) (void)hipStreamSynchronize(m->ds);
    (void)hipDeviceSynchronize();
    if (m->comm) (void)CCL(ncclCommDestroy)(m->comm);
    for (uint32_t i = 0; i < kPipeMax; ++i) {
        free_slot(m->slot[i]);
        if (m->ev_swept[i]) (void)hipEventDestroy(m->ev_swept[i]);
        if (m->ev_comb[i]) (void)hipEventDestroy(m->ev_comb[i]);
        if (m->ev_ag[i]) (void)hipEventDestroy(m->ev_ag[i]);
    }
    if (m->ev_drained) (void)hipEventDestroy(m->ev_drained);
    if (m->ev_in) (void)hipEventDestroy(m->ev_in);
    if (m->ev_ds) (void)hipEventDestroy(m->ev_ds);
    if (m->ds) (void)hipStreamDestroy(m->ds);
    if (m->ev_ctx) (void)hipEventDestroy(m->ev_ctx);
    for (hipStream_t q : m->ss)
        if (q) (void)hipStreamDestroy(q);
    void *dev[] = {m->win_pods, m->win_res, m->ctl, m->cands, m->cands_all, m->merged, m->sflags, m->sflags_all,
                   m->merged_flags};
    for (void *q : dev)
        if (q) (void)hipFree(q);
    if (m->h_ctl) (void)hipHostFree(m->h_ctl);
    if (m->cs) (void)hipStreamDestroy(m->cs);
    delete m;
    c->comm = nullptr;
}

int comm_cycle_staged(ms_ctx *c, uint32_t n, int32_t mode) {
    CommState &m = *c->comm;
    const hipStream_t s = c->stream;
    ++c->ctx_seq;  // binds below write the table on the context stream
    if (mode == MS_MODE_SEQUENTIAL && !plugins_stateless(c)) return seq_sharded_locked(c, n, c->d_pods, c->d_res, s);
    (void)m;
    return batched_all_locked(c, n, c->d_pods, c->d_res, s, true);
}

int comm_stage(ms_ctx *c, uint32_t n) {
    CommState &m = *c->comm;
    int rc = drain_to(c, c->stream);  // device-resident batches in flight finish first
    if (rc) return rc;
    const uint32_t per = cdiv(n, (uint32_t)m.world);
    return ensure_stage(c, std::max<uint32_t>(n, per * (uint32_t)m.world));
}

int comm_schedule_host(ms_ctx *c, uint32_t n, const ms_pod_rec *pods, int32_t mode, ms_result *out, CallClock *ck) {
    const hipStream_t s = c->stream;
    int rc = comm_stage(c, n);
    if (rc) return rc;
    ck->lap(MS_PH_ALLOC);
    ck->count(MS_PH_CHUNKS);
    MS_HIP(c, hipMemcpyAsync(c->d_pods, pods, sizeof(ms_pod_rec) * n, hipMemcpyHostToDevice, s));
    ck->lap(MS_PH_STAGE_IN);
    rc = comm_cycle_staged(c, n, mode);
    if (rc) return rc;
    ck->lap(MS_PH_LAUNCH);
    MS_HIP(c, hipMemcpyAsync(out, c->d_res, sizeof(ms_result) * n, hipMemcpyDeviceToHost, s));
    ck->lap(MS_PH_STAGE_OUT);
    MS_HIP(c, hipStreamSynchronize(s));
    ck->lap(MS_PH_WAIT);
    return MS_OK;
}

int comm_schedule_device(ms_ctx *c, uint32_t n, const ms_pod_rec *pods_dev, ms_result *results_dev, hipStream_t s) {
    CommState &m = *c->comm;
    if (!plugins_stateless(c)) return seq_sharded_locked(c, n, pods_dev, results_dev, s);
    // NU+NN / NodeAffinity: the batched cycle with its binds (equal to the queue-order loop)
    const uint32_t per = cdiv(n, (uint32_t)m.world);
    int rc = drain_to(c, s);
    if (rc) return rc;
    rc = ensure_stage(c, per * (uint32_t)m.world);
    if (rc) return rc;
    rc = batched_all_locked(c, n, pods_dev, c->d_res, s, true);
    if (rc) return rc;
    MS_HIP(c, hipMemcpyAsync(results_dev, c->d_res, sizeof(ms_result) * n, hipMemcpyDeviceToDevice, s));
    return MS_OK;
}

namespace {

// The communicator's streams and events, then the rendezvous of the ranks.
int comm_setup(ms_ctx *c, CommState &m, const ms_comm_id *id, int32_t rank, int32_t world) {
    // The collective and decode streams get the highest priority: high-priority
    // streams are served by hardware queues of their own, so the caller's
    // (sweep) stream can never share a queue with them and serialise a
    // reduce-scatter or a decode behind the next sweep; their short kernels are
    // dispatched ahead of the sweep's pending workgroups (profiles/r03zc_comm_prio_ab.txt).
    int lo = 0, hi = 0;
    MS_HIP(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
    const int cprio = hi;
    MS_HIP(c, hipStreamCreateWithPriority(&m.cs, hipStreamNonBlocking, cprio));
    // (MINISCHED_SHARD_STREAMS=2 only) two sweep streams at normal priority (at the
    // highest, the collectives fell behind)
    if (m.two_streams)
        for (hipStream_t &q : m.ss) MS_HIP(c, hipStreamCreateWithPriority(&q, hipStreamNonBlocking, 0));
    MS_HIP(c, hipStreamCreateWithPriority(&m.ds, hipStreamNonBlocking, cprio));
    MS_HIP(c, hipEventCreateWithFlags(&m.ev_ds, hipEventDisableTiming));
    for (uint32_t i = 0; i < kPipeMax; ++i) {
        MS_HIP(c, hipEventCreateWithFlags(&m.ev_swept[i], hipEventDisableTiming));
        MS_HIP(c, hipEventCreateWithFlags(&m.ev_comb[i], hipEventDisableTiming));
        MS_HIP(c, hipEventCreateWithFlags(&m.ev_ag[i], hipEventDisableTiming));
    }
    MS_HIP(c, hipEventCreateWithFlags(&m.ev_drained, hipEventDisableTiming));
    MS_HIP(c, hipEventCreateWithFlags(&m.ev_in, hipEventDisableTiming));
    MS_HIP(c, hipEventCreateWithFlags(&m.ev_ctx, hipEventDisableTiming));
    ncclUniqueId uid;
    std::memcpy(&uid, id->internal, sizeof(uid));
    const ncclResult_t r = CCL(ncclCommInitRank)(&m.comm, world, uid, rank);
    if (r != ncclSuccess) {
        m.comm = nullptr;
        return fail(c, MS_E_RCCL, std::string("ncclCommInitRank: ") + CCL(ncclGetErrorString)(r));
    }
    return MS_OK;
}

}  // namespace

}  // namespace msgpu

using namespace msgpu;

extern "C" {

int ms_comm_id_create(ms_comm_id *out) {
    if (!out) return MS_E_INVAL;
    ncclUniqueId id;
    const ncclResult_t r = CCL(ncclGetUniqueId)(&id);
    if (r != ncclSuccess) return fail(nullptr, MS_E_RCCL, std::string("ncclGetUniqueId: ") + CCL(ncclGetErrorString)(r));
    std::memcpy(out->internal, &id, sizeof(id));
    return MS_OK;
}

int ms_comm_init(ms_ctx *c, const ms_comm_id *id, int32_t rank, int32_t world) {
    if (!c || !id || world < 1 || rank < 0 || rank >= world) return MS_E_INVAL;
    std::lock_guard<std::mutex> g(c->sched_mu);
    if (c->comm) return fail(c, MS_E_INVAL, "ms_comm_init: the context already has a communicator");
    MS_HIP(c, hipSetDevice(c->cfg.device));
    CommState *m = new (std::nothrow) CommState();
    if (!m) return fail(c, MS_E_OOM, "ms_comm_init: host allocation");
    m->rank = rank;
    m->world = world;
    m->depth = std::min<uint32_t>(m->depth, kPipeMax - 1);
    m->group = m->depth;
    if (const char *e = getenv("MINISCHED_SHARD_STREAMS")) m->two_streams = atoi(e) == 2;
    if (const char *e = getenv("MINISCHED_HOST_PROF")) m->host_prof = atoi(e) == 1;
    if (const char *e = getenv("MINISCHED_SHARD_COALESCE")) m->coalesce = atoi(e) != 0;
    // Attached before the streams exist (MS_HIP reports through the context);
    // every failure below goes through comm_free, so a context is either joined
    // or left without a communicator, never half-built.
    c->comm = m;
    const int rc = comm_setup(c, *m, id, rank, world);
    if (rc != MS_OK) comm_free(c);
    return rc;
}

int ms_sharded_slice(const ms_ctx *c, uint32_t n, uint32_t *first, uint32_t *count) {
    if (!c || !first || !count) return MS_E_INVAL;
    if (!c->comm) {
        *first = 0;
        *count = n;
        return MS_OK;
    }
    slice_of(*c->comm, n, *first, *count);
    return MS_OK;
}

int ms_sharded_submit(ms_ctx *c, uint32_t n, const ms_pod_rec *pods_dev, ms_result *results_dev, void *stream) {
    if (!c || (n && !pods_dev)) return MS_E_INVAL;
    if (!c->comm) return fail(c, MS_E_INVAL, "ms_sharded_submit: the context has no communicator (ms_comm_init)");
    if (n == 0) return MS_OK;
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    uint32_t first = 0, count = 0;
    slice_of(*c->comm, n, first, count);
    if (count && !results_dev) return fail(c, MS_E_INVAL, "ms_sharded_submit: results_dev is required");
    int rc = flush_locked(c);
    if (rc) return rc;
    return submit_locked(c, n, pods_dev, results_dev, pick_stream(c, stream));
}

int ms_sharded_drain(ms_ctx *c, void *stream) {
    if (!c) return MS_E_INVAL;
    if (!c->comm) return fail(c, MS_E_INVAL, "ms_sharded_drain: the context has no communicator (ms_comm_init)");
    std::lock_guard<std::mutex> g(c->sched_mu);
    MS_HIP(c, hipSetDevice(c->cfg.device));
    return drain_to(c, pick_stream(c, stream));
}

}  // extern "C"
