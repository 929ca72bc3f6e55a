// ms_affinity.hip — plugin set MS_PLUGINS_NU_NN_NAM: Filter[NodeUnschedulable];
// Score[NodeNumber, NodeAffinity with several preferred terms], NodeAffinity's
// ScoreExtensions = DefaultNormalizeScore(MaxNodeScore, reverse=false)
// (k8s@v1.22.0 plugins/nodeaffinity/node_affinity.go, helper/normalize_score.go;
// restated) run by RunScorePlugins' in-loop hook exactly as written
// (/root/reference/minisched/minisched.go:164-185).
//
// With several terms a raw score (the sum of the matching terms' weights)
// reaches 400. Once an entry is non-zero the list maximum is 100 after every
// step, so step i is the identity when r_i <= 100 and otherwise rescales every
// EARLIER entry by f_{r_i}(v) = floor(100 v / r_i) (entry i ends at 100); the
// first non-zero node (the anchor) starts at 100. Node j's final score is
// T_{>j}(v_j): v_j = 100 for the anchor and for r_j > 100, else r_j, and T_{>j}
// the composition of the rescales of every later feasible node (oracle/
// ms_oracle.c nam_closed). Compositions of such maps on 0..100 are 101-entry
// tables that compose associatively, so a LIST-ordered row segment summarises
// as ONE table (its rescales composed) plus "has a non-zero node".
//
// Round 6: pod CLASSES. A node's NodeAffinity score depends on the pod only
// through its term set and, via NodeUnschedulable's feasibility, its toleration
// bit: pods with the same (term set, toleration) -- a class -- see the same
// feasible list, the same raw scores and so the same normalised scores. So the
// in-loop hook runs once per class, not per pod:
//   k_nam_classes  one workgroup: the batch's classes (dense ids), each pod's
//                  class, a representative pod per class, the pods in (class,
//                  name digit) order;
//   k_nam_seg      per (segment, class): the segment's composed rescale table
//                  (forward over its rows, T <- f_r o T at each rescale);
//   k_nam_fscore   per (segment, class): T_{>j} from the later segments (and
//                  later node shards), then the segment's rows in REVERSE order
//                  writing every row's normalised NodeAffinity score F[c][row]
//                  (0..100; 0xFF infeasible), the anchor decided by whether an
//                  earlier segment or shard has a non-zero node; and the
//                  maximum of F per node-digit class (atomicMax);
//   k_nam_pick     per pod (lane = pod, pods in class-digit order): the best
//                  total S* = max(w_na F + w_nn NodeNumber) follows from its
//                  class's maxima; then every (pod, row) pair is tested, four
//                  rows per bit operation (the row's F against the value that
//                  reaches S* given whether its name digit is the pod's), and
//                  only the rows reaching S* are hashed for selectHost's
//                  tie-break. Every pair is evaluated; only the hash is skipped
//                  where it cannot win.
// Terms (ABI 7, ms_nam_term_set_ext) are per-key value-id sets; the host turns
// each set into a lookup table (NamTab: per value id a 4-bit "these terms' sets
// hold it" mask per key, and the weight sum of every 4-bit term mask), so a
// row's raw score is wsum[z[zone] & l[label2]] for any operators.
#include <algorithm>

#include "ms_device.h"

namespace msgpu {

namespace {

constexpr uint32_t kNamTile = 1024;      // rows staged in LDS per pass
constexpr uint32_t kNamStride = 108;     // bytes per lane table in LDS: 27 words (odd: per-lane gathers spread banks)
constexpr uint32_t kNamTabStride = 548;  // bytes per lane term table in LDS: 137 words (odd)
constexpr uint32_t kNamComposeThreads = 128;
constexpr uint32_t kNamClsThreads = 1024;
constexpr uint32_t kNamPickRows = 32;  // rows per k_nam_pick step: two 16-B loads of F and two of the digit mask
constexpr uint32_t kNamSortCap = 65536;  // (class, digit) buckets the class sort takes (else batch order)
constexpr uint32_t kNamPickParts = 4;    // row parts per pod in a k_nam_pick workgroup (one per wave)
constexpr uint32_t kNamDigits = 11;      // node name digit 0..9, 10 = none

struct NamSeg {
    uint8_t T[101];  // the composed rescale map on 0..100
    uint8_t any;     // a feasible node of the segment has a non-zero raw score
    uint8_t _pad[2];
};
static_assert(sizeof(NamSeg) == MS_NAM_SEG_BYTES, "NamSeg layout");
static_assert(sizeof(NamTab) == 544 && kNamTabStride >= sizeof(NamTab), "NamTab layout");

// Row word staged in LDS: bit 0 absent, bit 1 unschedulable, zone << 8,
// label2 << 16, digit << 24 (15 = none).
__device__ __forceinline__ uint32_t nam_row_word(const NodeTable &t, uint32_t r) {
    const uint8_t f = t.flags[r];
    const uint32_t d = t.digit[r];
    return ((f & kNodeAbsent) ? 1u : 0u) | ((f & kNodeUnschedulable) ? 2u : 0u) | ((uint32_t)t.zone[r] << 8) |
           ((uint32_t)t.label2[r] << 16) | ((d <= 9u ? d : 15u) << 24);
}

__device__ __forceinline__ bool nam_feasible(uint32_t w, uint32_t tol) { return (w & (tol ? 1u : 3u)) == 0u; }

// NodeAffinity.Score of a row word under a term table in LDS.
__device__ __forceinline__ uint32_t nam_raw(uint32_t w, const uint8_t *tab) {
    const uint32_t m = tab[(w >> 8) & 0xFFu] & tab[256u + ((w >> 16) & 0xFFu)];
    return reinterpret_cast<const uint16_t *>(tab + 512)[m & 15u];
}

// Class key (term set, toleration) of a pod: set ids past n_sets count as no terms.
__device__ __forceinline__ uint32_t nam_key(const ms_pod_rec &p, uint32_t n_sets) {
    uint32_t sid = (uint32_t)p.pref_zone | (uint32_t)p.pref_weight << 8;
    if (sid > n_sets) sid = 0;
    return sid * 2u + (p.tolerates_unschedulable ? 1u : 0u);
}
__device__ __forceinline__ uint32_t nam_pod_digit(const ms_pod_rec &p) {
    return p.name_digit >= 0 && p.name_digit <= 9 ? (uint32_t)p.name_digit : 10u;
}

// The identity map in a lane's LDS table.
__device__ __forceinline__ void table_identity(uint8_t *row) {
    for (uint32_t v = 0; v <= 100u; v += 4u) {
        const uint32_t x = v | (v + 1u) << 8 | (v + 2u) << 16 | (v + 3u) << 24;
        *reinterpret_cast<uint32_t *>(row + v) = x;
    }
}

// floor(100 v / r) for v <= 100 (r > 100) as a multiply-high by m = floor((2^32 - 1) / r) + 1
// (one division per rescale, not per entry): m exceeds 2^32 / r by at most 1, so the
// product overshoots 100 v / r by at most 10^4 / 2^32 < 1 / r, less than the gap from any
// fraction k / r (k < r) to the next integer: the floor is exact.
__device__ __forceinline__ uint32_t div_magic(uint32_t r) { return 0xFFFFFFFFu / r + 1u; }
__device__ __forceinline__ uint32_t f_r(uint32_t v, uint32_t m) { return __umulhi(100u * v, m); }

// f_r o T on table `row` (every lane of the wave: entries lane, lane + 64).
__device__ __forceinline__ void table_post(uint8_t *row, uint32_t r, uint32_t lane) {
    const uint32_t m = div_magic(r);
    for (uint32_t v = lane; v <= 100u; v += 64u) row[v] = (uint8_t)f_r(row[v], m);
}

// T o f_r on table `row` (reads of both passes before the writes).
__device__ __forceinline__ void table_pre(uint8_t *row, uint32_t r, uint32_t lane) {
    const uint32_t v0 = lane, v1 = lane + 64u, m = div_magic(r);
    const uint8_t a = row[f_r(v0, m)];
    const uint8_t b = v1 <= 100u ? row[f_r(v1, m)] : 0;
    __builtin_amdgcn_wave_barrier();
    row[v0] = a;
    if (v1 <= 100u) row[v1] = b;
    __builtin_amdgcn_wave_barrier();
}

// The batch's classes (round 6), in five small launches:
//   k_nam_mark    used[key] = 1 for every pod's class key (used zeroed before);
//   k_nam_index   one workgroup: dense class ids in key order (used[key] becomes
//                 the class id), ctl[0] = the class count, cls_key[c], and the
//                 (class, name digit) bucket counters zeroed when they fit;
//   k_nam_count   pcls[p], and each bucket's pod count;
//   k_nam_offsets one workgroup: the buckets' start offsets (exclusive scan)
//                 into bstart and bcur;
//   k_nam_scatter perm = the pods in bucket order (class, then digit), and
//                 rep[c] = a pod of class c (its first bucket's first pod).
// With more buckets than kNamSortCap the pods keep batch order and rep[c] is
// the lowest pod index of the class (atomicMin in k_nam_count).
__global__ void k_nam_mark(const ms_pod_rec *__restrict__ pods, uint32_t n, uint32_t n_sets,
                           uint32_t *__restrict__ used) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) used[nam_key(pods[i], n_sets)] = 1u;
}

__global__ __launch_bounds__(kNamClsThreads) void k_nam_index(uint32_t n_sets, uint32_t *__restrict__ used,
                                                               uint32_t *__restrict__ ctl,
                                                               uint32_t *__restrict__ cls_key,
                                                               uint32_t *__restrict__ rep,
                                                               uint32_t *__restrict__ bcnt) {
    __shared__ uint32_t part[kNamClsThreads];
    const uint32_t tid = threadIdx.x, NT = kNamClsThreads;
    const uint32_t n_keys = 2u * (n_sets + 1u);
    const uint32_t per = (n_keys + NT - 1u) / NT, k0 = min(n_keys, tid * per), k1 = min(n_keys, k0 + per);
    uint32_t s = 0;
    for (uint32_t k = k0; k < k1; ++k) s += used[k];
    part[tid] = s;
    __syncthreads();
    if (tid == 0) {
        uint32_t a = 0;
        for (uint32_t t = 0; t < NT; ++t) {
            const uint32_t v = part[t];
            part[t] = a;
            a += v;
        }
        ctl[0] = a;
        ctl[1] = a * kNamDigits <= kNamSortCap ? 1u : 0u;  // sorted
    }
    __syncthreads();
    uint32_t c = part[tid];
    for (uint32_t k = k0; k < k1; ++k)
        if (used[k]) {
            cls_key[c] = k;
            rep[c] = 0xFFFFFFFFu;
            used[k] = c++;  // (used[] now maps a key to its class)
        }
    __syncthreads();
    const uint32_t nb = ctl[1] ? ctl[0] * kNamDigits : 0u;
    for (uint32_t b = tid; b < nb; b += NT) bcnt[b] = 0u;
}

__global__ void k_nam_count(const ms_pod_rec *__restrict__ pods, uint32_t n, uint32_t n_sets,
                            const uint32_t *__restrict__ used, const uint32_t *__restrict__ ctl,
                            uint32_t *__restrict__ pcls, uint32_t *__restrict__ rep, uint32_t *__restrict__ bcnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ms_pod_rec p = pods[i];
    const uint32_t cl = used[nam_key(p, n_sets)];
    pcls[i] = cl;
    if (ctl[1]) atomicAdd(&bcnt[cl * kNamDigits + nam_pod_digit(p)], 1u);
    else atomicMin(&rep[cl], i);
}

__global__ __launch_bounds__(kNamClsThreads) void k_nam_offsets(const uint32_t *__restrict__ ctl,
                                                                 uint32_t *__restrict__ bcnt,
                                                                 uint32_t *__restrict__ bstart) {
    __shared__ uint32_t part[kNamClsThreads];
    if (!ctl[1]) return;  // (workgroup-uniform)
    const uint32_t tid = threadIdx.x, NT = kNamClsThreads, nb = ctl[0] * kNamDigits;
    const uint32_t per = (nb + NT - 1u) / NT, b0 = min(nb, tid * per), b1 = min(nb, b0 + per);
    uint32_t s = 0;
    for (uint32_t b = b0; b < b1; ++b) s += bcnt[b];
    part[tid] = s;
    __syncthreads();
    if (tid == 0) {
        uint32_t a = 0;
        for (uint32_t t = 0; t < NT; ++t) {
            const uint32_t v = part[t];
            part[t] = a;
            a += v;
        }
    }
    __syncthreads();
    uint32_t a = part[tid];
    for (uint32_t b = b0; b < b1; ++b) {
        const uint32_t v = bcnt[b];
        bcnt[b] = a;  // (the scatter's running cursor)
        bstart[b] = a;
        a += v;
    }
}

__global__ void k_nam_scatter(const ms_pod_rec *__restrict__ pods, uint32_t n, const uint32_t *__restrict__ ctl,
                              const uint32_t *__restrict__ pcls, uint32_t *__restrict__ bcnt,
                              uint32_t *__restrict__ perm) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    perm[ctl[1] ? atomicAdd(&bcnt[pcls[i] * kNamDigits + nam_pod_digit(pods[i])], 1u) : i] = i;
}

__global__ void k_nam_rep(const uint32_t *__restrict__ ctl, const uint32_t *__restrict__ bstart,
                          const uint32_t *__restrict__ perm, uint32_t *__restrict__ rep) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (!ctl[1] || c >= ctl[0]) return;
    rep[c] = perm[bstart[c * kNamDigits]];  // (class c's buckets are contiguous and not all empty)
}

// A lane's class: its key's term table into the lane's LDS slot (kNamTabStride
// apart: an odd word stride, so the per-lane lookups spread over the banks); all
// 34 16-B loads issued before the stores. No terms: an all-zero table (raw 0).
__device__ __forceinline__ void load_class_tab(uint8_t *tabs, const NamTab *__restrict__ sets,
                                               const uint32_t *__restrict__ cls_key, uint32_t c, bool live,
                                               uint32_t lane) {
    constexpr uint32_t kVec = sizeof(NamTab) / 16;
    const uint32_t sid = live ? cls_key[c] >> 1 : 0u;
    const uint4 *src = reinterpret_cast<const uint4 *>(sets + (sid ? sid - 1u : 0u));
    uint4 v[kVec];
#pragma unroll
    for (uint32_t k = 0; k < kVec; ++k) v[k] = sid ? src[k] : make_uint4(0, 0, 0, 0);
    uint32_t *dst = reinterpret_cast<uint32_t *>(tabs + lane * kNamTabStride);
#pragma unroll
    for (uint32_t k = 0; k < kVec; ++k) {
        dst[4 * k] = v[k].x;
        dst[4 * k + 1] = v[k].y;
        dst[4 * k + 2] = v[k].z;
        dst[4 * k + 3] = v[k].w;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// grid (class blocks of 64, segments): the segment's composed rescale table per
// class, out[seg * stride + c].
__global__ __launch_bounds__(64) void k_nam_seg(NodeTable t, uint32_t n_rows, uint32_t seg_rows,
                                                const NamTab *__restrict__ sets, uint32_t n_sets,
                                                const uint32_t *__restrict__ ctl, const uint32_t *__restrict__ cls_key,
                                                uint32_t stride, NamSeg *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t tile[kNamTile];
    __shared__ __attribute__((aligned(16))) uint8_t tabs[64 * kNamStride];
    __shared__ __attribute__((aligned(16))) uint8_t terms[64 * kNamTabStride];
    const uint32_t lane = threadIdx.x, n_cls = ctl[0], c0 = blockIdx.x * 64u;
    if (c0 >= n_cls) return;  // (workgroup-uniform)
    const uint32_t c = c0 + lane;
    const bool live = c < n_cls;
    load_class_tab(terms, sets, cls_key, c, live, lane);
    const uint8_t *tb = terms + lane * kNamTabStride;
    const uint32_t tol = live ? (cls_key[c] & 1u) : 0u;
    const uint32_t r0 = blockIdx.y * seg_rows, r1 = min(n_rows, r0 + seg_rows);
    uint8_t *mine = tabs + lane * kNamStride;
    table_identity(mine);
    uint32_t any = 0, top = 100;  // top = T(100): 0 once the table is all 0
    for (uint32_t base = r0; base < r1; base += kNamTile) {
        const uint32_t nt = min(kNamTile, r1 - base);
        // a lane is done once its table is all 0 and it has seen a non-zero node
        const bool done = !live || (top == 0u && any);
        if (__ballot(!done) == 0) break;  // (one wave: wave-uniform)
        const uint32_t nt4 = (nt + 3u) & ~3u;  // (rows past nt: absent, never feasible)
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i = lane; i < nt4; i += 64u) tile[i] = i < nt ? nam_row_word(t, base + i) : 1u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // four rows per step: when no lane rescales at any of them (one ballot)
        // their only effect is `any`; else they go one by one
        for (uint32_t i = 0; i < nt4; i += 4) {
            const uint4 w4 = *reinterpret_cast<const uint4 *>(tile + i);
            const uint32_t wv[4] = {w4.x, w4.y, w4.z, w4.w};
            uint32_t rv[4];
            bool fv[4], resc = false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                fv[k] = live && nam_feasible(wv[k], tol);
                rv[k] = nam_raw(wv[k], tb);
                any |= (fv[k] && rv[k] > 0u) ? 1u : 0u;
                resc = resc || (fv[k] && rv[k] > 100u);
            }
            if (__ballot(resc && top != 0u) == 0) continue;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t r = rv[k];
                uint64_t b = __ballot(fv[k] && r > 100u && top != 0u);
                while (b) {  // (wave-uniform) the lanes with a rescale here, one table at a time
                    const uint32_t L = (uint32_t)__builtin_ctzll(b);
                    b &= b - 1u;
                    const uint32_t rl = (uint32_t)__builtin_amdgcn_readlane((int)r, (int)L);
                    table_post(tabs + L * kNamStride, rl, lane);
                    __builtin_amdgcn_wave_barrier();
                    if (lane == L) top = mine[100];
                }
            }
        }
    }
    if (!live) return;
    mine[101] = (uint8_t)any;
    mine[102] = mine[103] = 0;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(mine);
    uint32_t *dst = reinterpret_cast<uint32_t *>(out + (size_t)blockIdx.y * stride + c);
#pragma unroll
    for (int k = 0; k < (int)(MS_NAM_SEG_BYTES / 4); ++k) dst[k] = src[k];
}

// Per lane p < n_lanes: out = the composition of n records in order (in[s * stride + p], s
// ascending: out.T = T_{n-1} o .. o T_0) and the OR of their "any". With skip_to:
// only the records s > skip_to (a shard's suffix), and m_in gets the OR of the
// records s < skip_to. n_live (optional): lanes past *n_live skip.
__global__ void k_nam_compose(const NamSeg *__restrict__ in, uint32_t stride, uint32_t n, uint32_t n_lanes,
                              int32_t skip_to, NamSeg *__restrict__ out, uint8_t *__restrict__ m_in,
                              const uint32_t *__restrict__ n_live) {
    __shared__ __attribute__((aligned(16))) uint8_t tabs[kNamComposeThreads * kNamStride];
    __shared__ __attribute__((aligned(16))) uint8_t stg[kNamComposeThreads * kNamStride];
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_lanes || (n_live && p >= *n_live)) return;
    uint8_t *U = tabs + threadIdx.x * kNamStride;  // (LDS, not a dynamically indexed private array)
    uint8_t *st = stg + threadIdx.x * kNamStride;  // the record being composed, staged as words
    table_identity(U);
    uint32_t any = 0, before = 0;
    for (uint32_t s = 0; s < n; ++s) {
        const NamSeg *x = in + (size_t)s * stride + p;
        if (skip_to >= 0 && (int32_t)s < skip_to) {
            before |= x->any;
            continue;
        }
        if (skip_to >= 0 && (int32_t)s == skip_to) continue;
        any |= x->any;
        if (U[100] == 0) continue;  // (all 0 stays all 0)
        uint32_t w[MS_NAM_SEG_BYTES / 4];
#pragma unroll
        for (uint32_t k = 0; k < MS_NAM_SEG_BYTES / 4; ++k) w[k] = reinterpret_cast<const uint32_t *>(x)[k];
#pragma unroll
        for (uint32_t k = 0; k < MS_NAM_SEG_BYTES / 4; ++k) reinterpret_cast<uint32_t *>(st)[k] = w[k];
        for (uint32_t v = 0; v <= 100u; ++v) U[v] = st[U[v]];
    }
    U[101] = (uint8_t)any;
    U[102] = U[103] = 0;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(U);
    uint32_t *dst = reinterpret_cast<uint32_t *>(out + p);
#pragma unroll
    for (int k = 0; k < (int)(MS_NAM_SEG_BYTES / 4); ++k) dst[k] = src[k];
    if (m_in) m_in[p] = (uint8_t)before;
}

// Identity records (a shard without rows: no rescale, no non-zero node).
__global__ void k_nam_identity(NamSeg *__restrict__ out, uint32_t n) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    uint8_t *o = out[p].T;
    for (uint32_t v = 0; v <= 100u; ++v) o[v] = (uint8_t)v;
    o[101] = o[102] = o[103] = 0;
}

// Per pod: out[p] = cls_rec[pcls[p]] (a shard's per-class records as the ABI's per-pod ones).
__global__ void k_nam_expand(const NamSeg *__restrict__ cls_rec, const uint32_t *__restrict__ pcls, uint32_t n,
                             NamSeg *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;  // (one thread per 4-B word)
    constexpr uint32_t kW = MS_NAM_SEG_BYTES / 4;
    if (i >= n * kW) return;
    const uint32_t p = i / kW, w = i % kW;
    reinterpret_cast<uint32_t *>(out + p)[w] = reinterpret_cast<const uint32_t *>(cls_rec + pcls[p])[w];
}

// Node name digit of a row word (0..9; 10 = none).
__device__ __forceinline__ uint32_t word_digit(uint32_t w) {
    const uint32_t d = w >> 24;
    return d <= 9u ? d : 10u;
}

// grid (class blocks of 64, segments): every row's normalised NodeAffinity
// score F[c * fpitch + row] for this class (0xFF: infeasible) and, per node
// digit class, the class's maximum of F + 1 (fmax[c * 11 + d], atomicMax; 0:
// no feasible row). local: k_nam_seg's records [seg][stride]; after / m_in
// (node shards): the later shards' composed table and "an earlier shard has a
// non-zero node", read at the class's representative pod, or null.
__global__ __launch_bounds__(64) void k_nam_fscore(NodeTable t, uint32_t n_rows, uint32_t seg_rows,
                                                   const NamTab *__restrict__ sets, uint32_t n_sets,
                                                   const uint32_t *__restrict__ ctl,
                                                   const uint32_t *__restrict__ cls_key,
                                                   const uint32_t *__restrict__ rep, const NamSeg *__restrict__ local,
                                                   uint32_t stride, uint32_t n_segs, const NamSeg *__restrict__ after,
                                                   const uint8_t *__restrict__ m_in, uint8_t *__restrict__ F,
                                                   uint32_t fpitch, uint32_t *__restrict__ fmax) {
    __shared__ __attribute__((aligned(16))) uint32_t tile[kNamTile];
    __shared__ __attribute__((aligned(16))) uint8_t tabs[64 * kNamStride];
    __shared__ __attribute__((aligned(16))) uint8_t terms[64 * kNamTabStride];
    __shared__ uint32_t fm[64][12];
    __shared__ __attribute__((aligned(16))) uint8_t stg[64 * kNamStride];  // a later segment's table, staged
    const uint32_t lane = threadIdx.x, n_cls = ctl[0], c0 = blockIdx.x * 64u, seg = blockIdx.y;
    if (c0 >= n_cls) return;  // (workgroup-uniform)
    const uint32_t c = c0 + lane;
    const bool live = c < n_cls;
    load_class_tab(terms, sets, cls_key, c, live, lane);
    const uint8_t *tb = terms + lane * kNamTabStride;
    const uint32_t tol = live ? (cls_key[c] & 1u) : 0u;
    for (uint32_t d = 0; d < 12u; ++d) fm[lane][d] = 0u;
    // T_{>segment}: the later segments' tables, then the later shards'
    uint8_t *mine = tabs + lane * kNamStride;
    table_identity(mine);
    const uint32_t rp = live ? rep[c] : 0u;
    uint32_t before = (live && m_in) ? m_in[rp] : 0u;
    if (live) {
        for (uint32_t s = 0; s < seg; ++s) before |= local[(size_t)s * stride + c].any;
        // T <- T_s o T for the later segments, then the later shards: each record's
        // 104 B loaded as words into the lane's LDS row, then 101 lookups there
        uint8_t *st = stg + lane * kNamStride;
        auto compose = [&](const NamSeg *x) {
            const uint32_t *src = reinterpret_cast<const uint32_t *>(x);
            uint32_t w[MS_NAM_SEG_BYTES / 4];
#pragma unroll
            for (uint32_t k = 0; k < MS_NAM_SEG_BYTES / 4; ++k) w[k] = src[k];
#pragma unroll
            for (uint32_t k = 0; k < MS_NAM_SEG_BYTES / 4; ++k) reinterpret_cast<uint32_t *>(st)[k] = w[k];
            for (uint32_t v = 0; v <= 100u; ++v) mine[v] = st[mine[v]];
        };
        for (uint32_t s = seg + 1; s < n_segs && mine[100] != 0; ++s) compose(local + (size_t)s * stride + c);
        if (after && mine[100] != 0) compose(static_cast<const NamSeg *>(after) + rp);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    uint32_t top = mine[100];
    // the latest non-zero row seen (in reverse: the earliest so far) is the anchor
    // candidate: its T_{>j}(100) and row are kept; if it stays the first non-zero
    // row of the cluster its F becomes that value
    bool cand = false;
    uint32_t cand_row = 0, cand_top = 0, cand_dig = 0;
    uint8_t *Fc = F + (size_t)c * fpitch;
    const uint32_t r0 = seg * seg_rows, r1 = min(n_rows, r0 + seg_rows);
    const uint32_t n_tiles = r1 > r0 ? (r1 - r0 + kNamTile - 1u) / kNamTile : 0u;
    for (uint32_t ti = n_tiles; ti-- > 0;) {  // tiles and rows in reverse LIST order
        const uint32_t base = r0 + ti * kNamTile, nt = min(kNamTile, r1 - base);
        const uint32_t nt4 = (nt + 3u) & ~3u;  // (rows past nt: absent, never feasible)
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i = lane; i < nt4; i += 64u) tile[i] = i < nt ? nam_row_word(t, base + i) : 1u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i4 = nt4; i4 > 0; i4 -= 4) {
            const uint4 w4 = *reinterpret_cast<const uint4 *>(tile + i4 - 4);
            const uint32_t wv[4] = {w4.x, w4.y, w4.z, w4.w};
            uint32_t rv[4];
            bool fv[4], resc = false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                fv[k] = live && nam_feasible(wv[k], tol);
                rv[k] = nam_raw(wv[k], tb);
                resc = resc || (fv[k] && rv[k] > 100u);
            }
            const bool fix = __ballot(resc && top != 0u) == 0;  // (wave-uniform) the table is fixed across the four
            uint32_t packed = 0;
#pragma unroll
            for (int k = 3; k >= 0; --k) {
                const uint32_t r = rv[k];
                uint32_t f = 0xFFu;
                if (fv[k]) {
                    f = mine[min(r, 100u)];
                    if (r != 0u) {
                        cand = true;
                        cand_row = base + i4 - 4 + (uint32_t)k;
                        cand_top = top;
                        cand_dig = word_digit(wv[k]);
                    }
                    atomicMax(&fm[lane][word_digit(wv[k])], f + 1u);
                }
                packed |= f << (8 * k);
                if (!fix) {
                    uint64_t b = __ballot(fv[k] && r > 100u && top != 0u);
                    while (b) {  // (wave-uniform) this row's rescale applies to the earlier rows
                        const uint32_t L = (uint32_t)__builtin_ctzll(b);
                        b &= b - 1u;
                        const uint32_t rl = (uint32_t)__builtin_amdgcn_readlane((int)r, (int)L);
                        table_pre(tabs + L * kNamStride, rl, lane);
                        if (lane == L) top = mine[100];
                    }
                }
            }
            if (live) *reinterpret_cast<uint32_t *>(Fc + base + i4 - 4) = packed;
        }
    }
    if (!live) return;
    // the segment's first non-zero row is the anchor unless an earlier segment or shard has one
    if (cand && !before) {
        Fc[cand_row] = (uint8_t)cand_top;
        atomicMax(&fm[lane][cand_dig], cand_top + 1u);
    }
    for (uint32_t d = 0; d < kNamDigits; ++d)
        if (fm[lane][d]) atomicMax(&fmax[(size_t)c * kNamDigits + d], fm[lane][d]);
}

// Bytes of a word that are zero: 0x80 in each (exact: no carries across bytes).
__device__ __forceinline__ uint32_t zero_bytes(uint32_t y) {
    const uint32_t t = (y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    return ~(t | y) & 0x80808080u;
}

// Per pod (lane = pod, pods in class-digit order, so a wave's pods mostly share
// one class and digit): the packed key of the best total over this context's
// rows. Row j's total is w_na F_j + w_nn 10 [digit_j = the pod's]; the best S*
// follows from the class's maxima per digit, and the rows reaching S* are the
// ones whose F equals t_nn (digit = the pod's) or t_plain (else): compared four
// rows per word against a per-byte target chosen by the digit mask dmask[d][row]
// (0xFF where the row's name digit is d), then only those rows are hashed.
// Workgroup = 64 pods x kNamPickParts waves (wave w: row part w of the
// workgroup's grid.y slice), combined in LDS, then one atomicMax per pod into
// keys[p] (filled before with kKeyListed / 0: this context lists rows but none is
// feasible / lists none). grid.y x kNamPickParts parts keep many waves in flight
// over the row stream (lane = pod alone gives one wave per 64 pods).
__global__ __launch_bounds__(64 * kNamPickParts) void k_nam_pick(
    const ms_pod_rec *__restrict__ pods, uint32_t n_pods, const uint32_t *__restrict__ perm,
    const uint32_t *__restrict__ pcls, const uint8_t *__restrict__ F, uint32_t fpitch,
    const uint32_t *__restrict__ fmax, const uint8_t *__restrict__ dmask, uint32_t n_rows, uint32_t rows_per_part,
    uint32_t base, uint32_t seed32, uint32_t w_nn, uint32_t w_na, u64 *__restrict__ keys) {
    __shared__ u64 part_best[kNamPickParts][64];
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * 64u + lane;
    const bool live = i < n_pods;
    const uint32_t p = live ? perm[i] : 0u;
    const ms_pod_rec pod = pods[p];
    const uint32_t c = pcls[p], pd = nam_pod_digit(pod);
    uint32_t fall = 0, fpd = 0;
#pragma unroll
    for (uint32_t d = 0; d < kNamDigits; ++d) {
        const uint32_t v = fmax[(size_t)c * kNamDigits + d];
        fall = max(fall, v);
        fpd = d == pd ? v : fpd;  // (pd 10: non-digit pod, never matches)
    }
    if (pd > 9u) fpd = 0u;
    const uint32_t nn = 10u * w_nn;
    const uint32_t s_plain = fall ? w_na * (fall - 1u) : 0u, s_nn = fpd ? w_na * (fpd - 1u) + nn : 0u;
    const uint32_t S = max(s_plain, s_nn);
    // the F a row needs to reach S without / with the NodeNumber match (0xFE: none;
    // 0xFF, infeasible, never equals either)
    const uint32_t t_plain = (S % w_na == 0u && S / w_na <= 100u) ? S / w_na : 0xFEu;
    const uint32_t t_nn = (pd <= 9u && S >= nn && (S - nn) % w_na == 0u && (S - nn) / w_na <= 100u)
                              ? (S - nn) / w_na : 0xFEu;
    const uint32_t tp4 = t_plain * 0x01010101u, tn4 = t_nn * 0x01010101u;
    const uint32_t A = tb_pod(seed32, pod.ordinal);
    const uint8_t *Fc = F + (size_t)c * fpitch;
    const uint8_t *Dd = dmask + (size_t)pd * fpitch;  // (row 10: all zero)
    const uint32_t part = blockIdx.y * kNamPickParts + wave;
    const uint32_t j0 = part * rows_per_part, j1 = min(n_rows, j0 + rows_per_part);
    u64 top = 0;
    if (live && fall)
        for (uint32_t j = j0; j < j1; j += kNamPickRows) {
            const uint4 f0 = *reinterpret_cast<const uint4 *>(Fc + j), f1 = *reinterpret_cast<const uint4 *>(Fc + j + 16);
            const uint4 m0 = *reinterpret_cast<const uint4 *>(Dd + j), m1 = *reinterpret_cast<const uint4 *>(Dd + j + 16);
            const uint32_t fw[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
            const uint32_t mw[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
            uint32_t z[8], any = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                z[k] = zero_bytes(fw[k] ^ ((tn4 & mw[k]) | (tp4 & ~mw[k])));
                any |= z[k];
            }
            if (any) {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    uint32_t b = z[k];
                    while (b) {
                        const uint32_t bit = (uint32_t)__builtin_ctz(b);
                        b &= b - 1u;
                        const uint32_t ord = base + j + 4u * (uint32_t)k + (bit >> 3);
                        top = umax64(top, make_key(S, tb_hash(A, ord), ord));
                    }
                }
            }
        }
    part_best[wave][lane] = top;
    __syncthreads();
    if (wave == 0 && live) {
        u64 b = top;
#pragma unroll
        for (uint32_t w = 1; w < kNamPickParts; ++w) b = umax64(b, part_best[w][lane]);
        if (b) atomicMax(reinterpret_cast<unsigned long long *>(keys + p), (unsigned long long)b);
    }
}

__global__ void k_nam_fill(u64 *__restrict__ keys, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keys[i] = kKeyListed;
}

// dmask[d * fpitch + row] = 0xFF where row's name digit is d (d < 10), rows
// past n_rows and row 10 all zero.
__global__ void k_nam_dmask(NodeTable t, uint32_t n_rows, uint32_t fpitch, uint8_t *__restrict__ dmask) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= fpitch) return;
    const uint32_t d = j < n_rows ? (uint32_t)t.digit[j] : 0xFFu;
#pragma unroll
    for (uint32_t k = 0; k < kNamDigits; ++k) dmask[(size_t)k * fpitch + j] = (k < 10u && d == k) ? 0xFFu : 0u;
}

inline uint32_t cdiv(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

}  // namespace

// Row segments for the per-class passes: enough (segment, class-block) waves to
// spread over the chip, 64-row multiples (F is written four rows per word and
// read sixteen per load; a segment never writes its neighbour's rows).
NamLayout nam_layout(uint32_t n_rows, uint32_t cls_max) {
    NamLayout L;
    const uint32_t blocks = std::max(1u, cdiv(cls_max, 64u));
    // (per class and segment: rows / segs row steps, and up to segs compositions of
    // the later segments' 101-entry tables, so a few tens of segments)
    uint32_t segs = std::min(32u, std::max(8u, cdiv(128u, blocks)));
    L.seg_rows = std::max(64u, cdiv(cdiv(std::max(n_rows, 1u), segs), 64u) * 64u);
    L.segs = std::max(1u, cdiv(std::max(n_rows, 1u), L.seg_rows));
    L.fpitch = cdiv(std::max(n_rows, 1u), 64u) * 64u;
    L.cls_max = cls_max;
    return L;
}

namespace {
struct NamScratch {
    NamSeg *local, *comp;
    uint8_t *F, *dmask;
    uint32_t *fmax, *used, *ctl, *cls_key, *rep, *pcls, *perm, *bcnt, *bstart;
};
NamScratch nam_carve(void *scratch, const NamLayout &L, uint32_t n_pods, uint32_t n_sets, size_t *bytes = nullptr) {
    char *b = static_cast<char *>(scratch);
    NamScratch x;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        char *p = b + o;
        o += (bytes + 255u) & ~size_t(255);
        return p;
    };
    x.local = reinterpret_cast<NamSeg *>(take((size_t)L.segs * L.cls_max * sizeof(NamSeg)));
    x.comp = reinterpret_cast<NamSeg *>(take((size_t)L.cls_max * sizeof(NamSeg)));
    x.F = reinterpret_cast<uint8_t *>(take((size_t)L.cls_max * L.fpitch));
    x.dmask = reinterpret_cast<uint8_t *>(take((size_t)kNamDigits * L.fpitch));
    x.fmax = reinterpret_cast<uint32_t *>(take((size_t)L.cls_max * kNamDigits * 4));
    x.used = reinterpret_cast<uint32_t *>(take(2ull * (n_sets + 1u) * 4));
    x.ctl = reinterpret_cast<uint32_t *>(take(16 * 4));
    x.cls_key = reinterpret_cast<uint32_t *>(take((size_t)L.cls_max * 4));
    x.rep = reinterpret_cast<uint32_t *>(take((size_t)L.cls_max * 4));
    x.pcls = reinterpret_cast<uint32_t *>(take((size_t)n_pods * 4));
    x.perm = reinterpret_cast<uint32_t *>(take((size_t)n_pods * 4));
    const size_t nb = std::min<size_t>((size_t)L.cls_max * kNamDigits, kNamSortCap);
    x.bcnt = reinterpret_cast<uint32_t *>(take(nb * 4));
    x.bstart = reinterpret_cast<uint32_t *>(take(nb * 4));
    if (bytes) *bytes = o;
    return x;
}

}  // namespace

size_t nam_scratch_bytes(const NamLayout &L, uint32_t n_pods, uint32_t n_sets) {
    size_t o = 0;
    (void)nam_carve(nullptr, L, n_pods, n_sets, &o);
    return o;
}

namespace {
hipError_t nam_classes_and_segs(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                                const void *sets, uint32_t n_sets, const NamLayout &L, const NamScratch &x,
                                hipStream_t s) {
    hipError_t e = hipMemsetAsync(x.used, 0, 2ull * (n_sets + 1u) * 4, s);
    if (e != hipSuccess) return e;
    const dim3 pg(cdiv(n_pods, 256u));
    hipLaunchKernelGGL(k_nam_mark, pg, dim3(256), 0, s, pods, n_pods, n_sets, x.used);
    hipLaunchKernelGGL(k_nam_index, dim3(1), dim3(kNamClsThreads), 0, s, n_sets, x.used, x.ctl, x.cls_key, x.rep,
                       x.bcnt);
    hipLaunchKernelGGL(k_nam_count, pg, dim3(256), 0, s, pods, n_pods, n_sets, (const uint32_t *)x.used,
                       (const uint32_t *)x.ctl, x.pcls, x.rep, x.bcnt);
    hipLaunchKernelGGL(k_nam_offsets, dim3(1), dim3(kNamClsThreads), 0, s, (const uint32_t *)x.ctl, x.bcnt, x.bstart);
    hipLaunchKernelGGL(k_nam_scatter, pg, dim3(256), 0, s, pods, n_pods, (const uint32_t *)x.ctl,
                       (const uint32_t *)x.pcls, x.bcnt, x.perm);
    hipLaunchKernelGGL(k_nam_rep, dim3(cdiv(L.cls_max, 256u)), dim3(256), 0, s, (const uint32_t *)x.ctl,
                       (const uint32_t *)x.bstart, (const uint32_t *)x.perm, x.rep);
    hipLaunchKernelGGL(k_nam_seg, dim3(cdiv(L.cls_max, 64u), L.segs), dim3(64), 0, s, t, n_rows, L.seg_rows,
                       static_cast<const NamTab *>(sets), n_sets, (const uint32_t *)x.ctl,
                       (const uint32_t *)x.cls_key, L.cls_max, x.local);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_nam_segment(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                              const void *sets, uint32_t n_sets, const NamLayout &L, void *scratch, void *out,
                              hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    if (n_pods > L.cls_max && L.cls_max < 2u * (n_sets + 1u)) return hipErrorInvalidValue;
    const NamScratch x = nam_carve(scratch, L, n_pods, n_sets);
    hipError_t e = nam_classes_and_segs(t, n_rows, pods, n_pods, sets, n_sets, L, x, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_nam_compose, dim3(cdiv(L.cls_max, kNamComposeThreads)), dim3(kNamComposeThreads), 0, s,
                       (const NamSeg *)x.local, L.cls_max, L.segs, L.cls_max, -1, x.comp, (uint8_t *)nullptr,
                       (const uint32_t *)x.ctl);
    const uint32_t words = n_pods * (MS_NAM_SEG_BYTES / 4);
    hipLaunchKernelGGL(k_nam_expand, dim3(cdiv(words, 256u)), dim3(256), 0, s, (const NamSeg *)x.comp,
                       (const uint32_t *)x.pcls, n_pods, static_cast<NamSeg *>(out));
    return hipGetLastError();
}

hipError_t launch_nam_identity(void *out, uint32_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_nam_identity, dim3(cdiv(n, 256u)), dim3(256), 0, s, static_cast<NamSeg *>(out), n);
    return hipGetLastError();
}

hipError_t launch_nam_compose(const void *in, uint32_t stride, uint32_t n, uint32_t n_pods, int32_t skip_to,
                              void *out, uint8_t *m_in, hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    hipLaunchKernelGGL(k_nam_compose, dim3(cdiv(n_pods, kNamComposeThreads)), dim3(kNamComposeThreads), 0, s,
                       static_cast<const NamSeg *>(in), stride, n, n_pods, skip_to, static_cast<NamSeg *>(out), m_in,
                       (const uint32_t *)nullptr);
    return hipGetLastError();
}

hipError_t launch_nam_keys(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                           const void *sets, uint32_t n_sets, uint32_t seed32, uint32_t w_nn, uint32_t w_na,
                           const void *after, const uint8_t *m_in, uint32_t listed, const NamLayout &L,
                           void *scratch, unsigned long long *keys, hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    if (n_pods > L.cls_max && L.cls_max < 2u * (n_sets + 1u)) return hipErrorInvalidValue;
    const NamScratch x = nam_carve(scratch, L, n_pods, n_sets);
    hipError_t e = nam_classes_and_segs(t, n_rows, pods, n_pods, sets, n_sets, L, x, s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(x.fmax, 0, (size_t)L.cls_max * kNamDigits * 4, s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(x.F, 0xFF, (size_t)L.cls_max * L.fpitch, s);  // (rows past n_rows: never tied)
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_nam_dmask, dim3(cdiv(L.fpitch, 256u)), dim3(256), 0, s, t, n_rows, L.fpitch, x.dmask);
    hipLaunchKernelGGL(k_nam_fscore, dim3(cdiv(L.cls_max, 64u), L.segs), dim3(64), 0, s, t, n_rows, L.seg_rows,
                       static_cast<const NamTab *>(sets), n_sets, (const uint32_t *)x.ctl, (const uint32_t *)x.cls_key,
                       (const uint32_t *)x.rep, (const NamSeg *)x.local, L.cls_max, L.segs,
                       static_cast<const NamSeg *>(after), m_in, x.F, L.fpitch, x.fmax);
    // row parts: enough waves to keep the row stream busy (~16 per SIMD at 50k pods),
    // each part a multiple of kNamPickRows rows
    const uint32_t pod_blocks = cdiv(n_pods, 64u);
    uint32_t gy = std::max(1u, std::min(cdiv(16384u, pod_blocks * kNamPickParts), cdiv(n_rows, 256u * kNamPickParts)));
    const uint32_t parts = gy * kNamPickParts;
    const uint32_t rows_per_part = cdiv(cdiv(n_rows, parts), kNamPickRows) * kNamPickRows;
    gy = cdiv(cdiv(n_rows, rows_per_part), kNamPickParts);
    e = hipMemsetAsync(keys, 0, sizeof(u64) * n_pods, s);
    if (e != hipSuccess) return e;
    if (listed) hipLaunchKernelGGL(k_nam_fill, dim3(cdiv(n_pods, 256u)), dim3(256), 0, s, reinterpret_cast<u64 *>(keys), n_pods);
    hipLaunchKernelGGL(k_nam_pick, dim3(pod_blocks, gy), dim3(64 * kNamPickParts), 0, s, pods, n_pods,
                       (const uint32_t *)x.perm, (const uint32_t *)x.pcls, (const uint8_t *)x.F, L.fpitch,
                       (const uint32_t *)x.fmax, (const uint8_t *)x.dmask, n_rows, rows_per_part, t.base, seed32, w_nn,
                       w_na, reinterpret_cast<u64 *>(keys));
    return hipGetLastError();
}

}  // namespace msgpu
