// ms_taint.hip — plugin set MS_PLUGINS_NU_TT_NN: Filter[NodeUnschedulable,
// TaintToleration]; Score[NodeNumber, TaintToleration], TaintToleration's
// ScoreExtensions = DefaultNormalizeScore(MaxNodeScore, reverse=true)
// (k8s@v1.22.0 plugins/tainttoleration/taint_toleration.go, restated) run by
// RunScorePlugins' in-loop hook exactly as written
// (/root/reference/minisched/minisched.go:164-185).
//
// The hook rewrites the WHOLE list after every node, unscored entries
// included, with one map per step (v -> 100 - floor(100 v / M), M the list
// maximum; all 100 when M = 0). With per-node counts <= 8 (at most 8
// PreferNoSchedule taint ids) every step from the fourth to the next-to-last
// is the flip v -> 100 - v (oracle/ms_oracle.c tt_closed derives and checks
// this), so a node's final score depends only on its raw count c, the parity
// of its rank among the pod's feasible nodes in LIST order, the feasible count
// F, the first three and the last feasible node. Per pod the sweep therefore
// keeps a summary of a LIST-ordered segment of rows:
//   F, the filter flags, the first three and the last feasible node
//   (c, NodeNumber match, tie-break hash), and per class (c, rank parity) of the
//   other feasible nodes the best (NodeNumber match, hash) pair;
// summaries of consecutive segments merge associatively (tt_merge_into: ranks of
// the later segment shift by the earlier one's F), so row segments of one
// context and node shards of several GPUs combine the same way, and the
// finalisation (tt_finalize) applies the closed form and selectHost's argmax.
#include <algorithm>

#include "ms_device.h"

namespace msgpu {

namespace {

constexpr int kTtClasses = 18;  // c in 0..8 x rank parity
constexpr uint32_t kTtThreads = 256;   // pods per sweep workgroup (one per lane)
#ifndef MS_TT_TILE
#define MS_TT_TILE 1024
#endif
constexpr uint32_t kTtTile = MS_TT_TILE;  // rows staged in LDS per pass (2048 -> 1024: 8.24 -> 6.92 ms at 50k x 100k)
constexpr uint32_t kTtSegRows = 2048;  // minimum rows per segment
constexpr uint32_t kTtMaxSegs = 16;
constexpr uint32_t kTtCombineThreads = 128;  // k_tt_combine: one pod per thread, its running summary in LDS

// Segment summary of one pod (MS_TT_SUMMARY_BYTES). Special entries pack
// c << 40 | NodeNumber match << 32 | hash; class entries match << 32 | hash.
struct TtSummary {
    uint32_t n;      // feasible nodes in the segment
    uint32_t flags;  // MS_MASK_* of the filters that rejected a node of the segment
    uint32_t occ;    // occupied classes: bit 2c + parity
    uint32_t _pad;
    u64 first[3];    // local feasible ranks 0..2 (valid below n)
    u64 last;        // local rank n - 1 (valid when n > 0)
    u64 cls[kTtClasses];  // best entry of class (c, parity of the local rank) over ranks 3 .. n-2
};
static_assert(sizeof(TtSummary) == MS_TT_SUMMARY_BYTES, "TtSummary layout");

__device__ __forceinline__ uint32_t ent_c(u64 e) { return (uint32_t)(e >> 40) & 0xFFu; }
__device__ __forceinline__ u64 ent_key(u64 e) { return e & 0x1FFFFFFFFull; }  // match << 32 | hash

__device__ __forceinline__ void cls_put(TtSummary &r, uint32_t c, uint32_t par, u64 key) {
    const uint32_t k = 2u * c + par;
    if (!((r.occ >> k) & 1u) || key > r.cls[k]) r.cls[k] = key;
    r.occ |= 1u << k;
}

// r <- r merged with b, b following r in LIST order (in place: r lives in LDS
// in k_tt_combine, where its dynamically indexed classes need no scratch).
__device__ __forceinline__ void tt_merge_into(TtSummary &r, const TtSummary &b) {
    const uint32_t an = r.n;
    const u64 alast = r.last;
    r.n = an + b.n;
    r.flags |= b.flags;
    // b's classes, their parity shifted by a.n
    const uint32_t sh = an & 1u;
#pragma unroll
    for (int k = 0; k < kTtClasses; ++k)
        if ((b.occ >> k) & 1u) cls_put(r, (uint32_t)k >> 1, ((uint32_t)k & 1u) ^ sh, b.cls[k]);
    // the explicit entries of both: merged rank g -> first[g], last, or a class
    auto place = [&](u64 e, uint32_t g) {
        if (g < 3u) r.first[g] = e;
        if (g + 1u == r.n) r.last = e;
        if (g >= 3u && g + 1u < r.n) cls_put(r, ent_c(e), g & 1u, ent_key(e));
    };
    if (an > 3u) place(alast, an - 1u);  // (a's first three kept their ranks)
    for (uint32_t i = 0; i < 3u && i < b.n; ++i) place(b.first[i], an + i);
    if (b.n > 3u) place(b.last, an + b.n - 1u);
    if (b.n == 0u) r.last = alast;
}

__device__ __forceinline__ int32_t tt_map(int32_t m, int32_t v) { return m == 0 ? 100 : 100 - (100 * v) / m; }

// Final TaintToleration scores and selectHost over the merged summary of every
// segment of the cluster, in LIST order (oracle/ms_oracle.c tt_closed).
__device__ __forceinline__ ms_result tt_finalize(const TtSummary &r, const ms_pod_rec &pod, uint32_t seed32) {
    ms_result out;
    out._pad = 0;
    const uint32_t F = r.n;
    if (F == 0u) {  // FitError (minisched.go:143-148)
        out.node = -1;
        out.code = MS_CODE_UNSCHEDULABLE;
        out.score = 0;
        out.plugin_mask = r.flags;
        return out;
    }
    if (pod.name_digit < 0) {  // NodeNumber.Score fails (nodenumber.go:74-77)
        out.node = -1;
        out.code = MS_CODE_ERROR;
        out.score = 0;
        out.plugin_mask = 0;
        return out;
    }
    const uint32_t A = tb_pod(seed32, pod.ordinal);
    u64 best = 0;
    auto offer = [&](u64 key, int32_t v) {  // key = match << 32 | hash
        const uint32_t h = (uint32_t)key;
        const uint32_t score = 10u * (uint32_t)(key >> 32) + (uint32_t)v;
        best = umax64(best, make_key(score, h, tb_unhash(A, h)));
    };
    if (F <= 4u) {  // the loop itself over the (at most four) entries
        u64 e[4] = {r.first[0], r.first[1], r.first[2], r.last};
        int32_t s[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < F; ++k) {
            s[k] = (int32_t)ent_c(e[k]);
            int32_t m = 0;
            for (uint32_t i = 0; i < F; ++i) m = max(m, s[i]);
            for (uint32_t i = 0; i < F; ++i) s[i] = tt_map(m, s[i]);
        }
        for (uint32_t k = 0; k < F; ++k) offer(ent_key(e[k]), s[k]);
    } else {
        int32_t s[3], u = 0;  // entries 0..2 and the unscored entries after step 2
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            s[k] = (int32_t)ent_c(r.first[k]);
            int32_t m = u;
            for (int i = 0; i <= k; ++i) m = max(m, s[i]);
            for (int i = 0; i <= k; ++i) s[i] = tt_map(m, s[i]);
            u = tt_map(m, u);
        }
        const bool nf_odd = ((F - 4u) & 1u) != 0u;  // flips of steps 3 .. F-2
        const int32_t c_last = (int32_t)ent_c(r.last);
        int32_t p[3], m_last = c_last;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            p[k] = nf_odd ? 100 - s[k] : s[k];
            m_last = max(m_last, p[k]);
        }
        // class (c, parity q): rank j flipped F-2-j times after its own step (100 - c)
        auto pcls = [&](uint32_t k) {
            const int32_t c = (int32_t)(k >> 1);
            return ((k & 1u) == (F & 1u)) ? 100 - c : c;
        };
        for (uint32_t k = 0; k < (uint32_t)kTtClasses; ++k)
            if ((r.occ >> k) & 1u) m_last = max(m_last, pcls(k));
#pragma unroll
        for (int k = 0; k < 3; ++k) offer(ent_key(r.first[k]), tt_map(m_last, p[k]));
        offer(ent_key(r.last), tt_map(m_last, c_last));
        for (uint32_t k = 0; k < (uint32_t)kTtClasses; ++k)
            if ((r.occ >> k) & 1u) offer(r.cls[k], tt_map(m_last, pcls(k)));
    }
    out.node = (int32_t)(0xFFFFFu - (uint32_t)(best & 0xFFFFFu));
    out.code = MS_CODE_SUCCESS;
    out.score = (int64_t)(best >> 52);
    out.plugin_mask = 0;
    return out;
}

// Row word staged in LDS: digit (15 = none) | unschedulable << 4 | absent << 5 |
// NoSchedule taint ids << 8 | PreferNoSchedule ids << 16.
__device__ __forceinline__ uint32_t row_word(const NodeTable &t, uint32_t r) {
    const uint8_t f = t.flags[r];
    const uint32_t d = t.digit[r];
    const uint32_t tn = t.taints[r];
    return (d <= 9u ? d : 15u) | ((f & kNodeUnschedulable) ? 16u : 0u) | ((f & kNodeAbsent) ? 32u : 0u) |
           ((tn & 0xFFu) << 8) | (((tn >> 8) & 0xFFu) << 16);
}

// grid (pod blocks, segments): lane = pod, rows of the segment streamed through
// LDS in LIST order; the pod's per-class best hashes live in LDS (dynamic class
// index), their NodeNumber match bits in a register.
__global__ __launch_bounds__(kTtThreads) void k_tt_sweep(NodeTable t, uint32_t n_rows, uint32_t seg_rows,
                                                         const ms_pod_rec *__restrict__ pods, uint32_t n_pods,
                                                         uint32_t seed32, TtSummary *__restrict__ out) {
    __shared__ uint32_t tile[kTtTile];
    // per-class best: the hash in LDS, the NodeNumber match bit in a register
    // (bit k of clsm), so the workgroup's LDS is 22 KB (7 per CU)
    __shared__ uint32_t clsh[kTtClasses][kTtThreads];
    const uint32_t tid = threadIdx.x;
    const uint32_t p = blockIdx.x * kTtThreads + tid;
    const uint32_t seg = blockIdx.y;
    const uint32_t r0 = seg * seg_rows, r1 = min(n_rows, r0 + seg_rows);
    ms_pod_rec pod = {};
    if (p < n_pods) pod = pods[p];
    const uint32_t A = tb_pod(seed32, pod.ordinal);
    const uint32_t tolu = pod.tolerates_unschedulable ? 1u : 0u;
    const uint32_t tolh = pod.pref_zone, tols = pod.pref_weight;  // tol_hard / tol_soft (minisched_gpu.h)
    const uint32_t pd = pod.name_digit >= 0 && pod.name_digit <= 9 ? (uint32_t)pod.name_digit : 14u;
    uint32_t n = 0, flags = 0, occ = 0, clsm = 0;
    u64 f0 = 0, f1 = 0, f2 = 0, last = 0;
    for (uint32_t base = r0; base < r1; base += kTtTile) {
        const uint32_t nt = min(kTtTile, r1 - base);
        __syncthreads();
        for (uint32_t i = tid; i < nt; i += kTtThreads) tile[i] = row_word(t, base + i);
        __syncthreads();
        for (uint32_t i = 0; i < nt; ++i) {
            const uint32_t w = tile[i];  // (LDS broadcast: every lane reads the same row)
            if (w & 32u) continue;       // not in the LIST
            if ((w & 16u) && !tolu) {    // NodeUnschedulable rejects (first failure)
                flags |= MS_MASK_NODE_UNSCHEDULABLE;
                continue;
            }
            if ((w >> 8) & 0xFFu & ~tolh) {  // TaintToleration.Filter rejects
                flags |= MS_MASK_TAINT_TOLERATION;
                continue;
            }
            const uint32_t c = (uint32_t)__popc((w >> 16) & 0xFFu & ~tols);
            const uint32_t nn = (w & 15u) == pd ? 1u : 0u;
            const uint32_t ord = t.base + base + i;
            const u64 e = ((u64)c << 40) | ((u64)nn << 32) | tb_hash(A, ord);
            if (n >= 4u) {  // the previous feasible node (rank n-1 >= 3) is not the last: into its class
                const uint32_t k = 2u * ent_c(last) + ((n - 1u) & 1u);
                const uint32_t vm = (uint32_t)(last >> 32) & 1u, vh = (uint32_t)last, om = (clsm >> k) & 1u;
                if (!((occ >> k) & 1u) || vm > om || (vm == om && vh > clsh[k][tid])) {
                    clsh[k][tid] = vh;
                    clsm = (clsm & ~(1u << k)) | (vm << k);
                }
                occ |= 1u << k;
            }
            f0 = n == 0u ? e : f0;
            f1 = n == 1u ? e : f1;
            f2 = n == 2u ? e : f2;
            last = e;
            ++n;
        }
    }
    if (p >= n_pods) return;
    TtSummary &o = out[(size_t)seg * n_pods + p];
    o.n = n;
    o.flags = flags;
    o.occ = occ;
    o._pad = 0;
    o.first[0] = f0;
    o.first[1] = f1;
    o.first[2] = f2;
    o.last = last;
    for (int k = 0; k < kTtClasses; ++k)
        o.cls[k] = ((occ >> k) & 1u) ? ((u64)((clsm >> k) & 1u) << 32 | clsh[k][tid]) : 0ull;
}

// Per pod: the merge of n_segs summaries in LIST order (segment s at
// in[s * stride + p]), then either the merged summary (out) or its result
// (results; commit: NodeInfo.AddPod on the winner, which the table owns).
__global__ void k_tt_combine(const TtSummary *__restrict__ in, uint32_t stride, uint32_t n_segs,
                             const ms_pod_rec *__restrict__ pods, uint32_t n_pods, uint32_t seed32,
                             TtSummary *__restrict__ out, ms_result *__restrict__ results, NodeTable t, int commit) {
    __shared__ TtSummary acc[kTtCombineThreads];
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pods) return;
    TtSummary &r = acc[threadIdx.x];
    r = in[p];
    for (uint32_t s = 1; s < n_segs; ++s) tt_merge_into(r, in[(size_t)s * stride + p]);
    if (out) {
        out[p] = r;
        return;
    }
    const ms_result res = tt_finalize(r, pods[p], seed32);
    results[p] = res;
    if (commit && res.code == MS_CODE_SUCCESS) {
        const uint32_t node = (uint32_t)res.node;
        if (node >= t.base && node - t.base < t.cap) add_pod(t, node - t.base, pods[p], +1);
    }
}

inline uint32_t cdiv(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

}  // namespace

uint32_t tt_segments(uint32_t n_rows, uint32_t *seg_rows) {
    uint32_t sr = std::max(kTtSegRows, cdiv(std::max(n_rows, 1u), kTtMaxSegs));
    sr = cdiv(sr, kTtTile) * kTtTile;
    if (seg_rows) *seg_rows = sr;
    return std::max(1u, cdiv(n_rows, sr));
}

hipError_t launch_tt_sweep(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                           uint32_t seed32, void *summaries, hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    uint32_t sr = 0;
    const uint32_t segs = tt_segments(n_rows, &sr);
    hipLaunchKernelGGL(k_tt_sweep, dim3(cdiv(n_pods, kTtThreads), segs), dim3(kTtThreads), 0, s, t, n_rows, sr, pods,
                       n_pods, seed32, static_cast<TtSummary *>(summaries));
    return hipGetLastError();
}

hipError_t launch_tt_combine(const void *in, uint32_t stride, uint32_t n_segs, const ms_pod_rec *pods, uint32_t n_pods,
                             uint32_t seed32, void *out, ms_result *results, const NodeTable &t, int commit,
                             hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    if (n_segs == 0 || (!out && !results)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_tt_combine, dim3(cdiv(n_pods, kTtCombineThreads)), dim3(kTtCombineThreads), 0, s, static_cast<const TtSummary *>(in), stride,
                       n_segs, pods, n_pods, seed32, static_cast<TtSummary *>(out), results, t, commit);
    return hipGetLastError();
}

}  // namespace msgpu
