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

// ---- bit-sliced two-pass cycle (round 5) ------------------------------------
// The closed form needs the per-class best hashes only for the classes that can
// win, and which classes can win follows from the class OCCUPANCY alone: with
// F > 4 every class (c, rank parity q) scores tt_map(m_last, pcls) with pcls =
// 100 - c (q == F & 1) or c, all 18 values distinct and tt_map strictly
// decreasing for m_last <= 100, so the best total S* = max(explicit entries,
// 10 nn + class score) is reached by at most one class among the classes with a
// NodeNumber-matching row (W1, those rows) and one among the classes without
// (W0). So:
//   census  per (pod, row segment): F, filter flags, the first three and the last
//           feasible row, and the occupancy of the 18 classes over all middle rows
//           (occ) and over the NodeNumber-matching ones (occ1): bit planes of 32
//           rows, every filter, count and class a few v_bitop3 per word;
//   plan    per pod: the segments merged in LIST order (tt2_merge, the occupancy
//           form of tt_merge_into), the closed form: S*, W1, W0 and the best
//           explicit entry, or the result itself when no class can win;
//   pick    per (pod, segment): the maximum tie-break hash over the middle rows
//           of W1 (matching rows) and W0, global rank parity from the earlier
//           segments' counts: only those rows are hashed;
//   final   per pod: the explicit entry against the segments' picks.
// Row planes (k_tt2_planes, once per cycle): per 32-row word, 24 u32 — present,
// unschedulable, the 8 NoSchedule and 8 PreferNoSchedule taint ids, the 4 bits
// of the name digit (15: none), and a mask of the non-zero planes (read with
// scalar loads: a word is the same for every lane, the pods differ per lane).
constexpr uint32_t kTt2Planes = 24;
enum : uint32_t { kPlPres = 0, kPlUns = 1, kPlHard = 2, kPlSoft = 10, kPlDigit = 18, kPlNz = 22 };
constexpr uint32_t kTt2Threads = 256;  // pods per census / pick workgroup (lane = pod)
constexpr uint32_t kEntNone = 0xFFFFFFFFu;

struct TtCensus {  // 32 B per (segment, pod)
    uint32_t n, flags;
    uint32_t occ, occ1;  // bit 2c + q: a middle row of class (c, q) / one matching NodeNumber
    uint32_t first[3], last;  // entries: ordinal | nn << 21 | c << 24 (kEntNone: none)
};
static_assert(sizeof(TtCensus) == MS_TT_CENSUS_BYTES, "TtCensus layout (ms_tt_census_device)");
struct TtPlan {  // 32 B per pod
    uint32_t mode;  // 0: the plan kernel wrote the result, 1: pick
    uint32_t score; // S*
    uint32_t w1, w0;  // winning class bits (W1: matching rows only)
    uint32_t F, _pad;
    u64 best;       // best explicit entry at S* (make_key), 0: none
};
static_assert(sizeof(TtPlan) == MS_TT_CENSUS_BYTES, "plans buffers are sized in census records (ms_comm.cpp)");

__device__ __forceinline__ uint32_t ent_pack(uint32_t row, uint32_t c, uint32_t nn) { return row | nn << 21 | c << 24; }
__device__ __forceinline__ uint32_t ent_row(uint32_t e) { return e & 0x1FFFFFu; }
__device__ __forceinline__ uint32_t ent_nn(uint32_t e) { return (e >> 21) & 1u; }
__device__ __forceinline__ uint32_t ent_cc(uint32_t e) { return (e >> 24) & 0xFu; }

template <typename F>
constexpr uint32_t truth3(F f) {  // v_bitop3 table, S0 the most significant index bit
    uint32_t t = 0;
    for (int i = 0; i < 8; ++i)
        if (f((i >> 2) & 1, (i >> 1) & 1, i & 1)) t |= 1u << i;
    return t;
}
constexpr uint32_t kXor3 = truth3([](int a, int b, int c) { return (a ^ b ^ c) != 0; });
constexpr uint32_t kMaj3 = truth3([](int a, int b, int c) { return a + b + c >= 2; });
constexpr uint32_t kXnorAnd3 = truth3([](int a, int b, int c) { return c && a == b; });  // c & ~(a ^ b)
constexpr uint32_t kAndOr = truth3([](int a, int b, int c) { return (a && b) || c; });   // (a & b) | c
constexpr uint32_t kAndNotOr = truth3([](int a, int b, int c) { return (a && !b) || c; }); // (a & ~b) | c
// c & (a, b) == (0, 0) / (0, 1) / (1, 0) / (1, 1)
constexpr uint32_t kSel00 = truth3([](int a, int b, int c) { return c && !a && !b; });
constexpr uint32_t kSel01 = truth3([](int a, int b, int c) { return c && !a && b; });
constexpr uint32_t kSel10 = truth3([](int a, int b, int c) { return c && a && !b; });
constexpr uint32_t kSel11 = truth3([](int a, int b, int c) { return c && a && b; });
#define TT_BITOP3(a, b, c, imm) ((uint32_t)__builtin_amdgcn_bitop3_b32((a), (b), (c), (imm)))

// Per-lane pod masks: 0 / ~0 per taint id (not tolerated: ~0) and digit bit.
struct TtLane {
    uint32_t tolu_n;           // ~0 unless the pod tolerates node.kubernetes.io/unschedulable
    uint32_t hm[8], sm[8];     // NoSchedule / PreferNoSchedule id i NOT tolerated
    uint32_t dm[4];            // name digit bit b (non-digit pods: 14, which no row has)
    uint32_t A;
};

__device__ __forceinline__ TtLane tt_lane(const ms_pod_rec &pod, uint32_t seed32) {
    TtLane q;
    q.tolu_n = pod.tolerates_unschedulable ? 0u : ~0u;
    const uint32_t tolh = pod.pref_zone, tols = pod.pref_weight;  // tol_hard / tol_soft (minisched_gpu.h)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        q.hm[i] = ((tolh >> i) & 1u) ? 0u : ~0u;
        q.sm[i] = ((tols >> i) & 1u) ? 0u : ~0u;
    }
    const uint32_t pd = pod.name_digit >= 0 && pod.name_digit <= 9 ? (uint32_t)pod.name_digit : 14u;
#pragma unroll
    for (int b = 0; b < 4; ++b) q.dm[b] = ((pd >> b) & 1u) ? ~0u : 0u;
    q.A = tb_pod(seed32, pod.ordinal);
    return q;
}

// One 32-row word for one pod: feasible rows, their PreferNoSchedule counts c
// as bit planes c0..c3, the NodeNumber-matching feasible rows N; the filter
// rejections accumulate into fnu / ftt (first failure per row).
struct TtWord {
    uint32_t feas, c0, c1, c2, c3, N;
};
__device__ __forceinline__ TtWord tt_word(const uint32_t *__restrict__ pl, const TtLane &q, uint32_t &fnu,
                                          uint32_t &ftt) {
    const uint32_t nz = (uint32_t)__builtin_amdgcn_readfirstlane((int)pl[kPlNz]);
    const uint32_t pres = pl[kPlPres];
    uint32_t hard = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (nz & (1u << (kPlHard + i))) hard = TT_BITOP3(pl[kPlHard + i], q.hm[i], hard, kAndOr);
    const uint32_t nu = pl[kPlUns] & q.tolu_n;
    fnu |= pres & nu;
    ftt = TT_BITOP3(pres & hard, nu, ftt, kAndNotOr);
    TtWord o;
    o.feas = pres & ~(nu | hard);
    // c = popcount of the untolerated PreferNoSchedule ids: carry-save adders over
    // the 8 masked planes (groups of all-zero planes skipped, wave-uniform)
    uint32_t sa = 0, ka = 0, sb = 0, kb = 0, sc = 0, kc = 0;
    if (nz & (7u << kPlSoft)) {
        const uint32_t x0 = pl[kPlSoft + 0] & q.sm[0], x1 = pl[kPlSoft + 1] & q.sm[1], x2 = pl[kPlSoft + 2] & q.sm[2];
        sa = TT_BITOP3(x0, x1, x2, kXor3);
        ka = TT_BITOP3(x0, x1, x2, kMaj3);
    }
    if (nz & (7u << (kPlSoft + 3))) {
        const uint32_t x3 = pl[kPlSoft + 3] & q.sm[3], x4 = pl[kPlSoft + 4] & q.sm[4], x5 = pl[kPlSoft + 5] & q.sm[5];
        sb = TT_BITOP3(x3, x4, x5, kXor3);
        kb = TT_BITOP3(x3, x4, x5, kMaj3);
    }
    if (nz & (3u << (kPlSoft + 6))) {
        const uint32_t x6 = pl[kPlSoft + 6] & q.sm[6], x7 = pl[kPlSoft + 7] & q.sm[7];
        sc = x6 ^ x7;
        kc = x6 & x7;
    }
    o.c0 = TT_BITOP3(sa, sb, sc, kXor3);
    const uint32_t kd = TT_BITOP3(sa, sb, sc, kMaj3);
    const uint32_t se = TT_BITOP3(ka, kb, kc, kXor3), ke = TT_BITOP3(ka, kb, kc, kMaj3);
    o.c1 = se ^ kd;
    const uint32_t kf = se & kd;
    o.c2 = ke ^ kf;
    o.c3 = ke & kf;
    uint32_t N = o.feas;
#pragma unroll
    for (int b = 0; b < 4; ++b) N = TT_BITOP3(pl[kPlDigit + b], q.dm[b], N, kXnorAnd3);
    o.N = N;
    return o;
}

// Rows of odd rank among the word's feasible rows, the word's first feasible row
// having rank n: bit i of the inclusive prefix parity X is popcount(feas & bits
// 0..i) & 1, so row i's rank parity is X_i ^ 1 ^ (n & 1).
__device__ __forceinline__ uint32_t tt_odd_rows(uint32_t feas, uint32_t n) {
    uint32_t x = feas;
    x ^= x << 1;
    x ^= x << 2;
    x ^= x << 4;
    x ^= x << 8;
    x ^= x << 16;
    return (n & 1u) ? x : ~x;
}

__device__ __forceinline__ uint32_t tt_c_at(const TtWord &w, uint32_t b) {
    return ((w.c0 >> b) & 1u) | ((w.c1 >> b) & 1u) << 1 | ((w.c2 >> b) & 1u) << 2 | ((w.c3 >> b) & 1u) << 3;
}

__device__ __forceinline__ uint32_t swap_parity(uint32_t occ) {  // 18 class bits: 2c <-> 2c + 1
    return ((occ & 0x15555u) << 1) | ((occ >> 1) & 0x15555u);
}

// grid (pod blocks, segments of seg_words words): lane = pod.
__global__ __launch_bounds__(kTt2Threads) void k_tt2_census(const uint32_t *__restrict__ planes, uint32_t n_words,
                                                            uint32_t seg_words, const ms_pod_rec *__restrict__ pods,
                                                            uint32_t n_pods, uint32_t seed32, uint32_t node_base,
                                                            TtCensus *__restrict__ out) {
    const uint32_t p = blockIdx.x * kTt2Threads + threadIdx.x;
    const uint32_t w0 = blockIdx.y * seg_words, w1 = min(n_words, w0 + seg_words);
    ms_pod_rec pod = {};
    if (p < n_pods) pod = pods[p];
    const TtLane q = tt_lane(pod, seed32);
    uint32_t n = 0, fnu = 0, ftt = 0, f0 = kEntNone, f1 = kEntNone, f2 = kEntNone, last = kEntNone;
    uint32_t pend = 0, pend1 = 0;  // class bit of the tentative last row (rank >= 3), and if it matches
    uint32_t acc[9][2], acc1[9][2];
#pragma unroll
    for (int v = 0; v < 9; ++v) acc[v][0] = acc[v][1] = acc1[v][0] = acc1[v][1] = 0;
    uint32_t occ = 0, occ1 = 0;
    for (uint32_t w = w0; w < w1; ++w) {
        const uint32_t *pl = planes + (size_t)w * kTt2Planes;
        if (!__builtin_amdgcn_readfirstlane((int)pl[kPlPres])) continue;  // no listed row
        const TtWord x = tt_word(pl, q, fnu, ftt);
        if (!x.feas) continue;
        const uint32_t Q = tt_odd_rows(x.feas, n);
        const uint32_t cnt = (uint32_t)__popc(x.feas);
        uint32_t M = x.feas;  // middle rows: ranks 3 .. (not the tentative last)
        if (n < 3u) {  // ranks 0..2: explicit entries
            uint32_t m = x.feas, k = n;
            while (k < 3u && m) {
                const uint32_t b = first_slot(m);
                const uint32_t e = ent_pack(node_base + w * 32u + b, tt_c_at(x, b), (x.N >> b) & 1u);
                f0 = k == 0u ? e : f0;
                f1 = k == 1u ? e : f1;
                f2 = k == 2u ? e : f2;
                M &= ~(1u << b);
                m &= m - 1u;
                ++k;
            }
        }
        // the word's top feasible row is the tentative last; the previous one is a middle row
        const uint32_t t = 31u - (uint32_t)__clz(x.feas);
        M &= ~(1u << t);
        occ |= pend;
        occ1 |= pend1;
        const uint32_t ct = tt_c_at(x, t), nt = (x.N >> t) & 1u;
        last = ent_pack(node_base + w * 32u + t, ct, nt);
        pend = n + cnt - 1u >= 3u ? 1u << (2u * ct + ((Q >> t) & 1u)) : 0u;
        pend1 = nt ? pend : 0u;
        n += cnt;
        // the middle rows' classes: c == v from the count planes, by rank parity
        const uint32_t l0 = TT_BITOP3(x.c1, x.c0, M, kSel00), l1 = TT_BITOP3(x.c1, x.c0, M, kSel01);
        const uint32_t l2 = TT_BITOP3(x.c1, x.c0, M, kSel10), l3 = TT_BITOP3(x.c1, x.c0, M, kSel11);
        const uint32_t QN = Q & x.N, EN = x.N & ~Q;
        constexpr uint32_t kHi00 = kSel00, kHi01 = kSel01, kHi10 = kSel10;
        const uint32_t eq[9] = {
            TT_BITOP3(x.c3, x.c2, l0, kHi00), TT_BITOP3(x.c3, x.c2, l1, kHi00), TT_BITOP3(x.c3, x.c2, l2, kHi00),
            TT_BITOP3(x.c3, x.c2, l3, kHi00), TT_BITOP3(x.c3, x.c2, l0, kHi01), TT_BITOP3(x.c3, x.c2, l1, kHi01),
            TT_BITOP3(x.c3, x.c2, l2, kHi01), TT_BITOP3(x.c3, x.c2, l3, kHi01), TT_BITOP3(x.c3, x.c2, l0, kHi10)};
#pragma unroll
        for (int v = 0; v < 9; ++v) {
            acc[v][0] = TT_BITOP3(eq[v], Q, acc[v][0], kAndNotOr);
            acc[v][1] = TT_BITOP3(eq[v], Q, acc[v][1], kAndOr);
            acc1[v][0] = TT_BITOP3(eq[v], EN, acc1[v][0], kAndOr);
            acc1[v][1] = TT_BITOP3(eq[v], QN, acc1[v][1], kAndOr);
        }
    }
    if (p >= n_pods) return;
#pragma unroll
    for (int v = 0; v < 9; ++v)
#pragma unroll
        for (int par = 0; par < 2; ++par) {
            occ |= acc[v][par] ? 1u << (2 * v + par) : 0u;
            occ1 |= acc1[v][par] ? 1u << (2 * v + par) : 0u;
        }
    TtCensus o;
    o.n = n;
    o.flags = (fnu ? (uint32_t)MS_MASK_NODE_UNSCHEDULABLE : 0u) | (ftt ? (uint32_t)MS_MASK_TAINT_TOLERATION : 0u);
    o.occ = occ;
    o.occ1 = occ1;
    o.first[0] = f0;
    o.first[1] = f1;
    o.first[2] = f2;
    o.last = last;
    out[(size_t)blockIdx.y * n_pods + p] = o;
}

// r <- r merged with b (b follows r in LIST order), occupancy form of tt_merge_into.
__device__ __forceinline__ void tt2_merge(TtCensus &r, const TtCensus &b) {
    const uint32_t an = r.n, alast = r.last;
    r.n = an + b.n;
    r.flags |= b.flags;
    const bool sh = (an & 1u) != 0;
    r.occ |= sh ? swap_parity(b.occ) : b.occ;
    r.occ1 |= sh ? swap_parity(b.occ1) : b.occ1;
    auto place = [&](uint32_t e, uint32_t g) {
        if (g == 0u) r.first[0] = e;
        if (g == 1u) r.first[1] = e;
        if (g == 2u) r.first[2] = e;
        if (g + 1u == r.n) r.last = e;
        if (g >= 3u && g + 1u < r.n) {
            const uint32_t k = 1u << (2u * ent_cc(e) + (g & 1u));
            r.occ |= k;
            if (ent_nn(e)) r.occ1 |= k;
        }
    };
    if (an > 3u) place(alast, an - 1u);
    if (b.n > 0u) place(b.first[0], an);
    if (b.n > 1u) place(b.first[1], an + 1u);
    if (b.n > 2u) place(b.first[2], an + 2u);
    if (b.n > 3u) place(b.last, an + b.n - 1u);
    if (b.n == 0u) r.last = alast;
}

__device__ __forceinline__ void tt2_store(ms_result *results, uint32_t p, const ms_result &res, const NodeTable &t,
                                          const ms_pod_rec &pod, int commit) {
    if (!results) return;
    results[p] = res;
    if (commit && res.code == MS_CODE_SUCCESS) {
        const uint32_t node = (uint32_t)res.node;
        if (node >= t.base && node - t.base < t.cap) add_pod(t, node - t.base, pod, +1);
    }
}

// Per pod: the segments merged, then the closed form (tt_finalize's, classes by
// occupancy): the result when no class can win, else the pick plan.
// census: n_segs records per pod in LIST order (segments of one context, or the
// node shards' records), record s of pod p at census[s * stride + p]; results
// null: the plan only (a shard's pick).
__global__ void k_tt2_plan(const TtCensus *__restrict__ census, uint32_t n_segs, uint32_t stride,
                           const ms_pod_rec *__restrict__ pods, uint32_t n_pods, uint32_t seed32,
                           TtPlan *__restrict__ plans, ms_result *__restrict__ results, NodeTable t, int commit) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pods) return;
    TtCensus r = census[p];
    for (uint32_t s = 1; s < n_segs; ++s) tt2_merge(r, census[(size_t)s * stride + p]);
    const ms_pod_rec pod = pods[p];
    TtPlan plan = {};
    ms_result out;
    out._pad = 0;
    out.plugin_mask = 0;
    const uint32_t F = r.n;
    if (F == 0u) {  // FitError (minisched.go:143-148)
        out.node = -1;
        out.code = MS_CODE_UNSCHEDULABLE;
        out.score = 0;
        out.plugin_mask = r.flags;
        plans[p] = plan;
        tt2_store(results, p, out, t, pod, 0);
        return;
    }
    if (pod.name_digit < 0) {  // NodeNumber.Score fails (nodenumber.go:74-77)
        out.node = -1;
        out.code = MS_CODE_ERROR;
        out.score = 0;
        plans[p] = plan;
        tt2_store(results, p, out, t, pod, 0);
        return;
    }
    const uint32_t A = tb_pod(seed32, pod.ordinal);
    auto key_of = [&](uint32_t e, uint32_t score) {
        const uint32_t ord = ent_row(e);  // (a global ordinal)
        return make_key(score, tb_hash(A, ord), ord);
    };
    u64 best = 0;
    if (F <= 4u) {  // the loop itself over the (at most four) entries
        const uint32_t e[4] = {r.first[0], r.first[1], r.first[2], r.last};
        int32_t s[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < F; ++k) {
            s[k] = (int32_t)ent_cc(e[k]);
            int32_t m = 0;
            for (uint32_t i = 0; i < F; ++i) m = max(m, s[i]);
            for (uint32_t i = 0; i < F; ++i) s[i] = tt_map(m, s[i]);
        }
        for (uint32_t k = 0; k < F; ++k) best = umax64(best, key_of(e[k], 10u * ent_nn(e[k]) + (uint32_t)s[k]));
    } else {
        int32_t s[3], u = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            s[k] = (int32_t)ent_cc(r.first[k]);
            int32_t m = u;
            for (int i = 0; i <= k; ++i) m = max(m, s[i]);
            for (int i = 0; i <= k; ++i) s[i] = tt_map(m, s[i]);
            u = tt_map(m, u);
        }
        const bool nf_odd = ((F - 4u) & 1u) != 0u;
        const int32_t c_last = (int32_t)ent_cc(r.last);
        int32_t pv[3], m_last = c_last;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            pv[k] = nf_odd ? 100 - s[k] : s[k];
            m_last = max(m_last, pv[k]);
        }
        auto pcls = [&](uint32_t k) {
            const int32_t c = (int32_t)(k >> 1);
            return ((k & 1u) == (F & 1u)) ? 100 - c : c;
        };
        for (uint32_t k = 0; k < 18u; ++k)
            if ((r.occ >> k) & 1u) m_last = max(m_last, pcls(k));
        uint32_t tot[4];
#pragma unroll
        for (int k = 0; k < 3; ++k) tot[k] = 10u * ent_nn(r.first[k]) + (uint32_t)tt_map(m_last, pv[k]);
        tot[3] = 10u * ent_nn(r.last) + (uint32_t)tt_map(m_last, c_last);
        uint32_t S = max(max(tot[0], tot[1]), max(tot[2], tot[3]));
        for (uint32_t k = 0; k < 18u; ++k)
            if ((r.occ >> k) & 1u) S = max(S, ((r.occ1 >> k) & 1u ? 10u : 0u) + (uint32_t)tt_map(m_last, pcls(k)));
        const uint32_t e4[4] = {r.first[0], r.first[1], r.first[2], r.last};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (tot[k] == S) best = umax64(best, key_of(e4[k], S));
        uint32_t w1 = 0, w0 = 0;
        for (uint32_t k = 0; k < 18u; ++k) {
            if (!((r.occ >> k) & 1u)) continue;
            const bool m1 = ((r.occ1 >> k) & 1u) != 0;
            if ((m1 ? 10u : 0u) + (uint32_t)tt_map(m_last, pcls(k)) == S) {
                if (m1) w1 |= 1u << k;
                else w0 |= 1u << k;
            }
        }
        if (w1 | w0) {
            plan.mode = 1;
            plan.score = S;
            plan.w1 = w1;
            plan.w0 = w0;
            plan.F = F;
            plan.best = best;
            plans[p] = plan;
            return;
        }
    }
    plans[p] = plan;
    out.node = (int32_t)(0xFFFFFu - (uint32_t)(best & 0xFFFFFu));
    out.code = MS_CODE_SUCCESS;
    out.score = (int64_t)(best >> 52);
    tt2_store(results, p, out, t, pod, commit);
}

// grid (pod blocks, segments): per (pod, segment) the best key at S* among the
// middle rows of the winning classes (0: none), ranks global.
__global__ __launch_bounds__(kTt2Threads) void k_tt2_pick(const uint32_t *__restrict__ planes, uint32_t n_words,
                                                          uint32_t seg_words, const ms_pod_rec *__restrict__ pods,
                                                          uint32_t n_pods, uint32_t seed32,
                                                          const uint32_t *__restrict__ cnt, uint32_t cnt_words,
                                                          const uint32_t *__restrict__ base_in,
                                                          const TtPlan *__restrict__ plans, uint32_t node_base,
                                                          u64 *__restrict__ keys) {
    const uint32_t p = blockIdx.x * kTt2Threads + threadIdx.x;
    const uint32_t seg = blockIdx.y;
    const uint32_t w0 = seg * seg_words, w1 = min(n_words, w0 + seg_words);
    TtPlan plan = {};
    if (p < n_pods) plan = plans[p];
    const bool active = plan.mode == 1u;
    if (__ballot(active) == 0) {
        if (p < n_pods) keys[(size_t)seg * n_pods + p] = 0;
        return;  // (wave-uniform)
    }
    ms_pod_rec pod = {};
    if (active) pod = pods[p];
    const TtLane q = tt_lane(pod, seed32);
    // feasible rows before this segment (global ranks): the earlier node shards'
    // (base_in) and this context's earlier segments' (cnt: word 0 of records of
    // cnt_words words, [segment][pod])
    uint32_t n = (active && base_in) ? base_in[p] : 0u;
    if (active)
        for (uint32_t s = 0; s < seg; ++s) n += cnt[((size_t)s * n_pods + p) * cnt_words];
    const uint32_t F = plan.F;
    // the (at most one) winning class with a matching row and the (at most one)
    // without (k_tt2_plan: the 18 class scores are distinct), as per-lane masks:
    // c's bits 0 / ~0, the parity as an XOR on the odd-rank mask, validity
    const uint32_t k1 = plan.w1 ? first_slot(plan.w1) : 0u, k0 = plan.w0 ? first_slot(plan.w0) : 0u;
    const uint32_t v1 = plan.w1 ? ~0u : 0u, v0 = plan.w0 ? ~0u : 0u;
    const uint32_t q1x = (k1 & 1u) ? 0u : ~0u, q0x = (k0 & 1u) ? 0u : ~0u;
    uint32_t c1b[4], c0b[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        c1b[b] = ((k1 >> (1 + b)) & 1u) ? ~0u : 0u;
        c0b[b] = ((k0 >> (1 + b)) & 1u) ? ~0u : 0u;
    }
    u64 best = 0;
    uint32_t fnu = 0, ftt = 0;
    for (uint32_t w = w0; w < w1; ++w) {
        const uint32_t *pl = planes + (size_t)w * kTt2Planes;
        if (!__builtin_amdgcn_readfirstlane((int)pl[kPlPres])) continue;
        TtWord x = tt_word(pl, q, fnu, ftt);
        if (!active) x.feas = 0;
        if (!x.feas) continue;
        const uint32_t Q = tt_odd_rows(x.feas, n);
        const uint32_t cnt = (uint32_t)__popc(x.feas);
        // rows of the winning classes: count bits equal to c, parity, (W1) a NodeNumber match
        uint32_t m1 = (Q ^ q1x) & x.N & v1, m0 = (Q ^ q0x) & v0;
        m1 = TT_BITOP3(x.c0, c1b[0], m1, kXnorAnd3);
        m0 = TT_BITOP3(x.c0, c0b[0], m0, kXnorAnd3);
        m1 = TT_BITOP3(x.c1, c1b[1], m1, kXnorAnd3);
        m0 = TT_BITOP3(x.c1, c0b[1], m0, kXnorAnd3);
        m1 = TT_BITOP3(x.c2, c1b[2], m1, kXnorAnd3);
        m0 = TT_BITOP3(x.c2, c0b[2], m0, kXnorAnd3);
        m1 = TT_BITOP3(x.c3, c1b[3], m1, kXnorAnd3);
        m0 = TT_BITOP3(x.c3, c0b[3], m0, kXnorAnd3);
        uint32_t cand = x.feas & (m1 | m0);
        if (n < 3u) {  // global ranks 0..2 are explicit entries
            uint32_t m = x.feas;
            for (uint32_t k = n; k < 3u && m; ++k) {
                cand &= ~(m & (0u - m));
                m &= m - 1u;
            }
        }
        if (n + cnt == F) cand &= ~(0x80000000u >> __clz(x.feas));  // the global last row
        n += cnt;
        while (cand) {
            const uint32_t b = first_slot(cand);
            const uint32_t ord = node_base + w * 32u + b;
            best = umax64(best, make_key(plan.score, tb_hash(q.A, ord), ord));
            cand &= cand - 1u;
        }
    }
    if (p < n_pods) keys[(size_t)seg * n_pods + p] = best;
}

__global__ void k_tt2_final(const TtPlan *__restrict__ plans, const u64 *__restrict__ keys, uint32_t n_segs,
                            const ms_pod_rec *__restrict__ pods, uint32_t n_pods, ms_result *__restrict__ results,
                            NodeTable t, int commit) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pods) return;
    const TtPlan plan = plans[p];
    if (plan.mode != 1u) return;
    u64 best = plan.best;
    for (uint32_t s = 0; s < n_segs; ++s) best = umax64(best, keys[(size_t)s * n_pods + p]);
    ms_result out;
    out._pad = 0;
    out.plugin_mask = 0;
    out.node = (int32_t)(0xFFFFFu - (uint32_t)(best & 0xFFFFFu));
    out.code = MS_CODE_SUCCESS;
    out.score = (int64_t)(best >> 52);
    tt2_store(results, p, out, t, pods[p], commit);
}

// grid (pod blocks, segments): the feasible-row count per (segment, pod) alone
// (a shard's pick needs its segments' rank offsets, not their census).
__global__ __launch_bounds__(kTt2Threads) void k_tt2_count(const uint32_t *__restrict__ planes, uint32_t n_words,
                                                           uint32_t seg_words, const ms_pod_rec *__restrict__ pods,
                                                           uint32_t n_pods, uint32_t *__restrict__ out) {
    const uint32_t p = blockIdx.x * kTt2Threads + threadIdx.x;
    const uint32_t w0 = blockIdx.y * seg_words, w1 = min(n_words, w0 + seg_words);
    ms_pod_rec pod = {};
    if (p < n_pods) pod = pods[p];
    const TtLane q = tt_lane(pod, 0u);
    uint32_t n = 0;
    for (uint32_t w = w0; w < w1; ++w) {
        const uint32_t *pl = planes + (size_t)w * kTt2Planes;
        const uint32_t nz = (uint32_t)__builtin_amdgcn_readfirstlane((int)pl[kPlNz]);
        const uint32_t pres = pl[kPlPres];
        if (!__builtin_amdgcn_readfirstlane((int)pres)) continue;
        uint32_t hard = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (nz & (1u << (kPlHard + i))) hard = TT_BITOP3(pl[kPlHard + i], q.hm[i], hard, kAndOr);
        n += (uint32_t)__popc(pres & ~((pl[kPlUns] & q.tolu_n) | hard));
    }
    if (p < n_pods) out[(size_t)blockIdx.y * n_pods + p] = n;
}

// Per pod: the feasible nodes of the shards before `shard` (census_all records,
// [shard][pod] with stride) -- this shard's global rank offset.
__global__ void k_tt2_shard_base(const TtCensus *__restrict__ census_all, uint32_t stride, uint32_t shard,
                                 uint32_t n_pods, uint32_t *__restrict__ base) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pods) return;
    uint32_t n = 0;
    for (uint32_t s = 0; s < shard; ++s) n += census_all[(size_t)s * stride + p].n;
    base[p] = n;
}

// Per pod: this shard's key for the cross-shard uint64 MAX: the best of its
// segments' picks and the plan's explicit entry (the same on every shard), 0
// when the plan decided the pod outright (the final pass redoes that).
__global__ void k_tt2_keymax(const TtPlan *__restrict__ plans, const u64 *__restrict__ seg_keys, uint32_t n_segs,
                             uint32_t n_pods, u64 *__restrict__ keys) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pods) return;
    const TtPlan plan = plans[p];
    u64 best = 0;
    if (plan.mode == 1u) {
        best = plan.best;
        for (uint32_t s = 0; s < n_segs; ++s) best = umax64(best, seg_keys[(size_t)s * n_pods + p]);
    }
    keys[p] = best;
}

// Per pod: the merge of a context's segment records into one (a node shard's census).
__global__ void k_tt2_merge_segs(const TtCensus *__restrict__ census, uint32_t n_segs, uint32_t n_pods,
                                 TtCensus *__restrict__ out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pods) return;
    TtCensus r = census[p];
    for (uint32_t s = 1; s < n_segs; ++s) tt2_merge(r, census[(size_t)s * n_pods + p]);
    out[p] = r;
}

// One thread per row: 64 rows of a wave -> 2 words of planes by ballot.
__global__ __launch_bounds__(256) void k_tt2_planes(NodeTable t, uint32_t n_rows, uint32_t n_words,
                                                    uint32_t *__restrict__ planes) {
    __shared__ u64 bal[4][kTt2Planes];
    const uint32_t r = blockIdx.x * 256u + threadIdx.x, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t v = r < n_rows ? row_word(t, r) : 32u;  // (past the table: absent)
    const bool pres = !(v & 32u);
    u64 b[22];
    b[kPlPres] = __ballot(pres);
    b[kPlUns] = __ballot((v & 16u) != 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        b[kPlHard + i] = __ballot(((v >> (8 + i)) & 1u) != 0);
        b[kPlSoft + i] = __ballot(((v >> (16 + i)) & 1u) != 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) b[kPlDigit + i] = __ballot(((v >> i) & 1u) != 0);
    if (lane == 0) {
#pragma unroll
        for (int j = 0; j < 22; ++j) bal[wv][j] = b[j];
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    const uint32_t j = lane & 31u;
    const u64 bj = j < 22u ? bal[wv][j] : 0ull;
    const uint32_t half = lane < 32u ? (uint32_t)bj : (uint32_t)(bj >> 32);
    const u64 nzb = __ballot(half != 0u && j < 22u);
    // lanes 0..31: the word of rows (r & ~63) .. +31, lanes 32..63 the next; lane j & 31 = plane
    const uint32_t wbase = ((r & ~63u) >> 5) + (lane < 32u ? 0u : 1u);
    if (wbase < n_words && j < kTt2Planes) {
        uint32_t val = half;
        if (j == kPlNz) val = lane < 32u ? (uint32_t)nzb : (uint32_t)(nzb >> 32);
        if (j == kPlNz + 1) val = 0u;
        planes[(size_t)wbase * kTt2Planes + j] = val;
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

uint32_t tt2_words(uint32_t n_rows) { return cdiv(std::max(n_rows, 1u), 32u); }

// Two-pass scratch (d_tt): the row planes, then per chunk of up to max_pods pods
// the census [segs][pods], the plans [pods] and the picks [segs][pods].
// The two-pass scratch (d_tt): the row planes, then per chunk of up to max_pods
// pods the census [segs][pods], the plans [pods], the picks [segs][pods], and
// for node shards the segments' counts [segs][pods] and the shard offsets [pods].
struct Tt2Scratch {
    uint32_t *planes;
    TtCensus *census;
    TtPlan *plans;
    u64 *keys;
    uint32_t *counts, *base;
    size_t bytes;
};
Tt2Scratch tt2_layout(void *scratch, uint32_t n_rows, uint32_t max_pods) {
    const size_t segs = tt_segments(n_rows), m = max_pods;
    char *b = static_cast<char *>(scratch);
    Tt2Scratch x;
    size_t o = 0;
    x.planes = reinterpret_cast<uint32_t *>(b + o);
    o += (size_t)tt2_words(n_rows) * kTt2Planes * 4;
    x.census = reinterpret_cast<TtCensus *>(b + o);
    o += segs * m * sizeof(TtCensus);
    x.plans = reinterpret_cast<TtPlan *>(b + o);
    o += m * sizeof(TtPlan);
    x.keys = reinterpret_cast<u64 *>(b + o);
    o += segs * m * sizeof(u64);
    x.counts = reinterpret_cast<uint32_t *>(b + o);
    o += segs * m * 4;
    x.base = reinterpret_cast<uint32_t *>(b + o);
    o += m * 4;
    x.bytes = o;
    return x;
}

size_t tt2_scratch_bytes(uint32_t n_rows, uint32_t max_pods) { return tt2_layout(nullptr, n_rows, max_pods).bytes; }

hipError_t launch_tt2_planes(const NodeTable &t, uint32_t n_rows, void *scratch, hipStream_t s) {
    const uint32_t nw = tt2_words(n_rows);
    hipLaunchKernelGGL(k_tt2_planes, dim3(cdiv(nw * 32u, 256u)), dim3(256), 0, s, t, n_rows, nw,
                       static_cast<uint32_t *>(scratch));
    return hipGetLastError();
}

hipError_t launch_tt2_cycle(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                            uint32_t seed32, void *scratch, uint32_t max_pods, ms_result *results, int commit,
                            hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    if (n_pods > max_pods || !results) return hipErrorInvalidValue;
    uint32_t sr = 0;
    const uint32_t segs = tt_segments(n_rows, &sr), nw = tt2_words(n_rows), sw = sr / 32u;
    const Tt2Scratch x = tt2_layout(scratch, n_rows, max_pods);
    const dim3 grid(cdiv(n_pods, kTt2Threads), segs);
    hipLaunchKernelGGL(k_tt2_census, grid, dim3(kTt2Threads), 0, s, x.planes, nw, sw, pods, n_pods, seed32, t.base,
                       x.census);
    hipLaunchKernelGGL(k_tt2_plan, dim3(cdiv(n_pods, 128u)), dim3(128), 0, s, x.census, segs, n_pods, pods, n_pods,
                       seed32, x.plans, results, t, commit);
    hipLaunchKernelGGL(k_tt2_pick, grid, dim3(kTt2Threads), 0, s, x.planes, nw, sw, pods, n_pods, seed32,
                       reinterpret_cast<const uint32_t *>(x.census), (uint32_t)(sizeof(TtCensus) / 4),
                       (const uint32_t *)nullptr, x.plans, t.base, x.keys);
    hipLaunchKernelGGL(k_tt2_final, dim3(cdiv(n_pods, 128u)), dim3(128), 0, s, x.plans, x.keys, segs, pods, n_pods,
                       results, t, commit);
    return hipGetLastError();
}

// Node shards (ms_tt_census_device / ms_tt_pick_device / ms_tt_final_device): the
// row planes must be current (launch_tt2_planes earlier on s).
hipError_t launch_tt2_census_shard(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                                   uint32_t seed32, void *scratch, uint32_t max_pods, void *census_out,
                                   hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    if (n_pods > max_pods) return hipErrorInvalidValue;
    uint32_t sr = 0;
    const uint32_t segs = tt_segments(n_rows, &sr), nw = tt2_words(n_rows), sw = sr / 32u;
    const Tt2Scratch x = tt2_layout(scratch, n_rows, max_pods);
    hipLaunchKernelGGL(k_tt2_census, dim3(cdiv(n_pods, kTt2Threads), segs), dim3(kTt2Threads), 0, s, x.planes, nw, sw,
                       pods, n_pods, seed32, t.base, x.census);
    hipLaunchKernelGGL(k_tt2_merge_segs, dim3(cdiv(n_pods, 128u)), dim3(128), 0, s, x.census, segs, n_pods,
                       static_cast<TtCensus *>(census_out));
    return hipGetLastError();
}

hipError_t launch_tt2_pick_shard(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                                 uint32_t seed32, void *scratch, uint32_t max_pods, const void *census_all,
                                 uint32_t stride, uint32_t n_shards, uint32_t shard, unsigned long long *keys_out,
                                 hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    if (n_pods > max_pods || shard >= n_shards) return hipErrorInvalidValue;
    uint32_t sr = 0;
    const uint32_t segs = tt_segments(n_rows, &sr), nw = tt2_words(n_rows), sw = sr / 32u;
    const Tt2Scratch x = tt2_layout(scratch, n_rows, max_pods);
    const TtCensus *ca = static_cast<const TtCensus *>(census_all);
    const dim3 grid(cdiv(n_pods, kTt2Threads), segs), g1(cdiv(n_pods, 128u));
    hipLaunchKernelGGL(k_tt2_plan, g1, dim3(128), 0, s, ca, n_shards, stride, pods, n_pods, seed32, x.plans,
                       (ms_result *)nullptr, t, 0);
    hipLaunchKernelGGL(k_tt2_count, grid, dim3(kTt2Threads), 0, s, x.planes, nw, sw, pods, n_pods, x.counts);
    hipLaunchKernelGGL(k_tt2_shard_base, g1, dim3(128), 0, s, ca, stride, shard, n_pods, x.base);
    hipLaunchKernelGGL(k_tt2_pick, grid, dim3(kTt2Threads), 0, s, x.planes, nw, sw, pods, n_pods, seed32,
                       (const uint32_t *)x.counts, 1u, (const uint32_t *)x.base, x.plans, t.base, x.keys);
    hipLaunchKernelGGL(k_tt2_keymax, g1, dim3(128), 0, s, x.plans, x.keys, segs, n_pods,
                       reinterpret_cast<u64 *>(keys_out));
    return hipGetLastError();
}

void *tt2_plans(void *scratch, uint32_t n_rows, uint32_t max_pods) {
    return tt2_layout(scratch, n_rows, max_pods).plans;
}

hipError_t launch_tt2_final_shard(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                                  uint32_t seed32, void *plans_buf, uint32_t max_pods, const void *census_all,
                                  uint32_t stride, uint32_t n_shards, const unsigned long long *keys_max,
                                  ms_result *results, hipStream_t s) {
    (void)n_rows;
    if (n_pods == 0) return hipSuccess;
    if (n_pods > max_pods || !results || !plans_buf) return hipErrorInvalidValue;
    TtPlan *plans = static_cast<TtPlan *>(plans_buf);  // (n_pods records)
    const dim3 g1(cdiv(n_pods, 128u));
    hipLaunchKernelGGL(k_tt2_plan, g1, dim3(128), 0, s, static_cast<const TtCensus *>(census_all), n_shards, stride,
                       pods, n_pods, seed32, plans, results, t, 0);
    hipLaunchKernelGGL(k_tt2_final, g1, dim3(128), 0, s, plans, reinterpret_cast<const u64 *>(keys_max), 1u, pods,
                       n_pods, results, t, 0);
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
