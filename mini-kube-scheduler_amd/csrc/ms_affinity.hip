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
// as ONE table (its rescales composed) plus "has a non-zero node":
//   k_nam_seg   per (segment, pod): that table, forward over the segment's rows
//               (T <- f_r o T at each rescale);
//   k_nam_keys  per (segment, pod): the suffix table of the later segments (and
//               of the later node shards) composed, then the segment's rows in
//               REVERSE order keeping T_{>j} (T <- T o f_r after each rescale)
//               and the best packed key; the anchor decided by whether an
//               earlier segment or shard has a non-zero node. atomicMax over the
//               segments; node shards combine by uint64 MAX like NU+NN.
// Lane = pod, rows streamed through LDS. A lane's table lives in LDS (a 108-B
// row per lane); a rescale updates one table with all 64 lanes of the wave
// (one lane per table entry, 2 passes), the lanes with a rescale on the same row
// taken in turn by a ballot loop. Every f_r maps 1..100 below itself, so a table
// is all 0 after at most 100 rescales; a lane whose T(100) is 0 stops updating.
#include <algorithm>

#include "ms_device.h"

namespace msgpu {

namespace {

constexpr uint32_t kNamThreads = 256;  // pods per workgroup (one per lane)
constexpr uint32_t kNamTile = 1024;    // rows staged in LDS per pass
constexpr uint32_t kNamSegRows = 2048, kNamMaxSegs = 16;
constexpr uint32_t kNamStride = 108;   // bytes per lane table in LDS: 27 words (odd: per-lane gathers spread banks)

constexpr uint32_t kNamComposeThreads = 128;

struct NamSeg {
    uint8_t T[101];  // the composed rescale map on 0..100
    uint8_t any;     // a feasible node of the segment has a non-zero raw score
    uint8_t _pad[2];
};
static_assert(sizeof(NamSeg) == MS_NAM_SEG_BYTES, "NamSeg layout");

// Row word staged in LDS: bit 0 absent, bit 1 unschedulable, zone << 8,
// label2 << 16, digit << 24 (15 = none).
__device__ __forceinline__ uint32_t nam_row_word(const NodeTable &t, uint32_t r) {
    const uint8_t f = t.flags[r];
    const uint32_t d = t.digit[r];
    return ((f & kNodeAbsent) ? 1u : 0u) | ((f & kNodeUnschedulable) ? 2u : 0u) | ((uint32_t)t.zone[r] << 8) |
           ((uint32_t)t.label2[r] << 16) | ((d <= 9u ? d : 15u) << 24);
}

// A pod's terms: term k matches a row whose label byte (zone: byte 1 of the
// row word, label2: byte 2) lies in [lo, lo + span] (In: value, span 0;
// Exists: 1..255, every labelled row) and adds weight (0: unused slot, or value 0 = "unlabelled",
// which never matches).
#ifndef MS_NAM_PACKED  // terms two per register in 16-bit halves (v_perm + v_pk_*_u16; 0: one at a time, A/B)
#define MS_NAM_PACKED 1
#endif
#if MS_NAM_PACKED
typedef unsigned short nam_u16x2 __attribute__((ext_vector_type(2)));
// Terms (0, 1) and (2, 3) in the halves of one register each: sel picks the
// terms' label bytes out of the row word into the low byte of each half
// (v_perm_b32, 0x0C = a zero byte), lo / span + 1 / weight per half.
struct NamTerms {
    uint32_t sel[2];
    nam_u16x2 lo[2], sp1[2], w[2];
};
#else
struct NamTerms {
    uint32_t sh[MS_NAM_TERMS], lo[MS_NAM_TERMS], span[MS_NAM_TERMS], w[MS_NAM_TERMS];
};
#endif

__device__ __forceinline__ NamTerms load_terms(const ms_pod_rec &pod, const ms_nam_term_set *sets, uint32_t n_sets) {
    NamTerms m;
    const uint32_t sid = (uint32_t)pod.pref_zone | (uint32_t)pod.pref_weight << 8;
    ms_nam_term_set st = {};
    if (sid != 0u && sid <= n_sets) st = sets[sid - 1u];
#pragma unroll
    for (int k = 0; k < MS_NAM_TERMS; ++k) {
        const ms_pref_term x = st.term[k];
        const uint32_t lo = x.value == 0xFFu ? 1u : x.value, span = x.value == 0xFFu ? 254u : 0u;
        const uint32_t w = x.value == 0u ? 0u : x.weight;
#if MS_NAM_PACKED
        const int h = k >> 1, half = k & 1;
        const uint32_t b = x.key ? 2u : 1u;
        if (half == 0) {
            m.sel[h] = b | 0x0C0C0C00u;  // (bytes 1-3 zero until term k+1 fills byte 2)
            m.lo[h].x = (unsigned short)lo;
            m.sp1[h].x = (unsigned short)(span + 1u);
            m.w[h].x = (unsigned short)w;
        } else {
            m.sel[h] = (m.sel[h] & 0xFF00FFFFu) | b << 16;
            m.lo[h].y = (unsigned short)lo;
            m.sp1[h].y = (unsigned short)(span + 1u);
            m.w[h].y = (unsigned short)w;
        }
#else
        m.sh[k] = x.key ? 16u : 8u;
        m.lo[k] = lo;
        m.span[k] = span;
        m.w[k] = w;
#endif
    }
    return m;
}

// NodeAffinity.Score: the sum of the weights of the matching terms.
__device__ __forceinline__ uint32_t nam_raw(uint32_t w, const NamTerms &m) {
#if MS_NAM_PACKED
    // per half: d = label - lo (wrapping: a label below lo lands above 65280),
    // s = sat(span + 1 - d) > 0 exactly when lo <= label <= lo + span, and
    // min(s * weight, weight) (s * weight <= 255 * 100 < 2^16) the term's share
    nam_u16x2 t = {0, 0};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t lab = __builtin_amdgcn_perm(0u, w, m.sel[h]);
        const nam_u16x2 d = __builtin_bit_cast(nam_u16x2, lab) - m.lo[h];
        const nam_u16x2 s = __builtin_elementwise_sub_sat(m.sp1[h], d);
        t += __builtin_elementwise_min(s * m.w[h], m.w[h]);
    }
    return (uint32_t)t.x + (uint32_t)t.y;
#else
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < MS_NAM_TERMS; ++k) {
        const uint32_t lab = (w >> m.sh[k]) & 0xFFu;
        r += (lab - m.lo[k] <= m.span[k]) ? m.w[k] : 0u;
    }
    return r;
#endif
}

__device__ __forceinline__ bool nam_feasible(uint32_t w, uint32_t tol) { return (w & (tol ? 1u : 3u)) == 0u; }

// The identity map in a lane's LDS table.
__device__ __forceinline__ void table_identity(uint8_t *row) {
    for (uint32_t v = 0; v <= 100u; v += 4u) {
        const uint32_t x = v | (v + 1u) << 8 | (v + 2u) << 16 | (v + 3u) << 24;
        *reinterpret_cast<uint32_t *>(row + v) = x;
    }
}

// f_r o T on table `row` (every lane of the wave: entries lane, lane + 64).
__device__ __forceinline__ void table_post(uint8_t *row, uint32_t r, uint32_t lane) {
    for (uint32_t v = lane; v <= 100u; v += 64u) row[v] = (uint8_t)((100u * row[v]) / r);
}

// T o f_r on table `row` (reads of both passes before the writes).
__device__ __forceinline__ void table_pre(uint8_t *row, uint32_t r, uint32_t lane) {
    const uint32_t v0 = lane, v1 = lane + 64u;
    const uint8_t a = row[(100u * v0) / r];
    const uint8_t b = v1 <= 100u ? row[(100u * v1) / r] : 0;
    __builtin_amdgcn_wave_barrier();
    row[v0] = a;
    if (v1 <= 100u) row[v1] = b;
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void seg_bounds(uint32_t n_rows, uint32_t seg_rows, uint32_t seg, uint32_t &r0,
                                           uint32_t &r1) {
    r0 = seg * seg_rows;
    r1 = min(n_rows, r0 + seg_rows);
}

// grid (pod blocks, segments): the segment's composed rescale table per pod.
__global__ __launch_bounds__(kNamThreads) void k_nam_seg(NodeTable t, uint32_t n_rows, uint32_t seg_rows,
                                                         const ms_pod_rec *__restrict__ pods, uint32_t n_pods,
                                                         const ms_nam_term_set *__restrict__ sets, uint32_t n_sets,
                                                         NamSeg *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t tile[kNamTile];
    __shared__ __attribute__((aligned(16))) uint8_t tabs[kNamThreads * kNamStride];
    const uint32_t tid = threadIdx.x, lane = lane_id(), wbase = tid & ~63u;
    const uint32_t p = blockIdx.x * kNamThreads + tid;
    uint32_t r0, r1;
    seg_bounds(n_rows, seg_rows, blockIdx.y, r0, r1);
    ms_pod_rec pod = {};
    if (p < n_pods) pod = pods[p];
    const NamTerms m = load_terms(pod, sets, n_sets);
    const uint32_t tol = pod.tolerates_unschedulable ? 1u : 0u;
    uint8_t *mine = tabs + tid * kNamStride;
    table_identity(mine);
    uint32_t any = 0, top = 100;  // top = T(100): 0 once the table is all 0
    for (uint32_t base = r0; base < r1; base += kNamTile) {
        const uint32_t nt = min(kNamTile, r1 - base);
        // a lane is done once its table is all 0 and it has seen a non-zero node:
        // nothing later in the segment changes its record (the workgroup stops
        // when all its lanes are, a wave skips the tile's rows)
        const bool done = p >= n_pods || (top == 0u && any);
        if (__syncthreads_and(done)) break;
        // (rows past nt up to a multiple of 4: absent, never feasible)
        const uint32_t nt4 = (nt + 3u) & ~3u;
        for (uint32_t i = tid; i < nt4; i += kNamThreads) tile[i] = i < nt ? nam_row_word(t, base + i) : 1u;
        __syncthreads();
        if (__ballot(!done) == 0) continue;  // (wave-uniform)
        // four rows per step (one 16-B LDS broadcast): when no lane rescales at any
        // of them (one ballot), their only effect is `any`; else they go one by one
        for (uint32_t i = 0; i < nt4; i += 4) {
            const uint4 w4 = *reinterpret_cast<const uint4 *>(tile + i);
            const uint32_t wv[4] = {w4.x, w4.y, w4.z, w4.w};
            uint32_t rv[4];
            bool fv[4], resc = false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                fv[k] = nam_feasible(wv[k], tol);
                rv[k] = nam_raw(wv[k], m);
                any |= (fv[k] && rv[k] > 0u) ? 1u : 0u;
                resc = resc || (fv[k] && rv[k] > 100u);
            }
            if (__ballot(resc && top != 0u) == 0) continue;  // (wave-uniform)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t r = rv[k];
                uint64_t b = __ballot(fv[k] && r > 100u && top != 0u);
                while (b) {  // (wave-uniform) the lanes with a rescale here, one table at a time
                    const uint32_t L = (uint32_t)__builtin_ctzll(b);
                    b &= b - 1u;
                    const uint32_t rl = (uint32_t)__builtin_amdgcn_readlane((int)r, (int)L);
                    table_post(tabs + (wbase + L) * kNamStride, rl, lane);
                    __builtin_amdgcn_wave_barrier();
                    if (lane == L) top = mine[100];
                }
            }
        }
    }
    if (p >= n_pods) return;
    mine[101] = (uint8_t)any;
    mine[102] = mine[103] = 0;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(mine);
    uint32_t *dst = reinterpret_cast<uint32_t *>(out + (size_t)blockIdx.y * n_pods + p);
#pragma unroll
    for (int k = 0; k < (int)(MS_NAM_SEG_BYTES / 4); ++k) dst[k] = src[k];
}

// Per pod: out = the composition of n segment records in order (in[s * stride + p], s
// ascending: out.T = T_{n-1} o .. o T_0) and the OR of their "any". With skip_to:
// only the records s > skip_to (a shard's suffix), and m_in gets the OR of the
// records s < skip_to.
__global__ void k_nam_compose(const NamSeg *__restrict__ in, uint32_t stride, uint32_t n, uint32_t n_pods,
                              int32_t skip_to, NamSeg *__restrict__ out, uint8_t *__restrict__ m_in) {
    __shared__ __attribute__((aligned(16))) uint8_t tabs[kNamComposeThreads * kNamStride];
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pods) return;
    uint8_t *U = tabs + threadIdx.x * kNamStride;  // (LDS, not a dynamically indexed private array)
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
        for (uint32_t v = 0; v <= 100u; ++v) U[v] = x->T[U[v]];
    }
    U[101] = (uint8_t)any;
    U[102] = U[103] = 0;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(U);
    uint32_t *dst = reinterpret_cast<uint32_t *>(out + p);
#pragma unroll
    for (int k = 0; k < (int)(MS_NAM_SEG_BYTES / 4); ++k) dst[k] = src[k];
    if (m_in) m_in[p] = (uint8_t)before;
}

// grid (pod blocks, segments): the segment's best packed key per pod (atomicMax
// into keys). local: this context's segment records [n_segs][n_pods]; after /
// m_in (node shards): the later shards' composed table and "an earlier shard has
// a non-zero node" per pod, or null (single shard).
__global__ __launch_bounds__(kNamThreads) void k_nam_keys(NodeTable t, uint32_t n_rows, uint32_t seg_rows,
                                                          const ms_pod_rec *__restrict__ pods, uint32_t n_pods,
                                                          const ms_nam_term_set *__restrict__ sets, uint32_t n_sets,
                                                          uint32_t seed32, uint32_t w_nn, uint32_t w_na,
                                                          const NamSeg *__restrict__ local, uint32_t n_segs,
                                                          const NamSeg *__restrict__ after,
                                                          const uint8_t *__restrict__ m_in, u64 *__restrict__ keys,
                                                          const uint32_t *__restrict__ perm) {
    __shared__ __attribute__((aligned(16))) uint32_t tile[kNamTile];
    __shared__ __attribute__((aligned(16))) uint8_t tabs[kNamThreads * kNamStride];
    const uint32_t tid = threadIdx.x, lane = lane_id(), wbase = tid & ~63u;
    const uint32_t pi = blockIdx.x * kNamThreads + tid;
    const bool live = pi < n_pods;
    // lanes take the pods in name-digit order (perm, k_nam_perm): a wave's pods then
    // mostly share the rows that can score NodeNumber's 10
    const uint32_t p = live ? (perm ? perm[pi] : pi) : pi;
    const uint32_t seg = blockIdx.y;
    uint32_t r0, r1;
    seg_bounds(n_rows, seg_rows, seg, r0, r1);
    ms_pod_rec pod = {};
    if (live) pod = pods[p];
    const NamTerms m = load_terms(pod, sets, n_sets);
    const uint32_t tol = pod.tolerates_unschedulable ? 1u : 0u;
    const uint32_t pd = pod.name_digit >= 0 && pod.name_digit <= 9 ? (uint32_t)pod.name_digit : 14u;
    const uint32_t A = tb_pod(seed32, pod.ordinal);
    // T_{>segment}: the later segments' tables, then the later shards'
    uint8_t *mine = tabs + tid * kNamStride;
    table_identity(mine);
    uint32_t before = (live && m_in) ? m_in[p] : 0u;
    if (live) {
        for (uint32_t s = 0; s < seg; ++s) before |= local[(size_t)s * n_pods + p].any;
        for (uint32_t s = seg + 1; s < n_segs && mine[100] != 0; ++s) {
            const uint8_t *T = local[(size_t)s * n_pods + p].T;
            for (uint32_t v = 0; v <= 100u; ++v) mine[v] = T[mine[v]];
        }
        if (after && mine[100] != 0) {
            const uint8_t *T = after[p].T;
            for (uint32_t v = 0; v <= 100u; ++v) mine[v] = T[mine[v]];
        }
    }
    uint32_t top = mine[100];
    // A row's key is hashed only when its score can reach the best so far (a lower
    // score cannot win; an equal one needs its hash). The latest non-zero row
    // (the anchor candidate) keeps its two scores and ordinal; it is hashed when
    // committed.
    u64 best = 0;
    uint32_t cand_sreg = 0, cand_sanc = 0, cand_ord = 0;
    bool cand = false;
    const uint32_t n_tiles = r1 > r0 ? (r1 - r0 + kNamTile - 1u) / kNamTile : 0u;
    // one row's candidate update (before its own rescale, which applies to earlier rows)
    // Branch-light: at most one key is hashed per row (the row's own with a
    // zero raw score, T(0) = 0, or -- a later non-zero node is not the anchor --
    // the previous candidate's regular key), the candidate update is selects.
    auto row_key = [&](uint32_t w, bool f, uint32_t r, uint32_t ord) {
        const uint32_t sn = ((w >> 24) == pd) ? 10u * w_nn : 0u;
        const uint32_t bs = (uint32_t)(best >> 52);
        const bool nz = f && r != 0u;
        const bool h0 = f && r == 0u && sn >= bs, h1 = nz && cand && cand_sreg >= bs;
        if (h0 || h1) {
            const uint32_t o = h0 ? ord : cand_ord, sc = h0 ? sn : cand_sreg;
            best = umax64(best, make_key(sc, tb_hash(A, o), o));
        }
        const uint32_t mv = mine[min(r, 100u)];
        cand = cand || nz;
        cand_sreg = nz ? sn + w_na * mv : cand_sreg;
        cand_sanc = nz ? sn + w_na * top : cand_sanc;
        cand_ord = nz ? ord : cand_ord;
    };
    for (uint32_t ti = n_tiles; ti-- > 0;) {  // tiles and rows in reverse LIST order
        const uint32_t base = r0 + ti * kNamTile, nt = min(kNamTile, r1 - base);
        const uint32_t nt4 = (nt + 3u) & ~3u;  // (rows past nt: absent, never feasible)
        __syncthreads();
        for (uint32_t i = tid; i < nt4; i += kNamThreads) tile[i] = i < nt ? nam_row_word(t, base + i) : 1u;
        __syncthreads();
        // four rows per step (one 16-B LDS broadcast, one ballot): while no lane
        // rescales at any of them the table is fixed across the four
        for (uint32_t i4 = nt4; i4 > 0; i4 -= 4) {
            const uint4 w4 = *reinterpret_cast<const uint4 *>(tile + i4 - 4);
            const uint32_t wv[4] = {w4.x, w4.y, w4.z, w4.w};
            uint32_t rv[4];
            bool fv[4], resc = false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                fv[k] = nam_feasible(wv[k], tol);
                rv[k] = nam_raw(wv[k], m);
                resc = resc || (fv[k] && rv[k] > 100u);
            }
            const uint32_t ord0 = t.base + base + i4 - 4;
            if (__ballot(resc && top != 0u) == 0) {  // (wave-uniform)
#pragma unroll
                for (int k = 3; k >= 0; --k) row_key(wv[k], fv[k], rv[k], ord0 + k);
                continue;
            }
#pragma unroll
            for (int k = 3; k >= 0; --k) {
                row_key(wv[k], fv[k], rv[k], ord0 + k);
                const uint32_t r = rv[k];
                uint64_t b = __ballot(fv[k] && r > 100u && top != 0u);
                while (b) {  // (wave-uniform) this row's rescale applies to the earlier rows
                    const uint32_t L = (uint32_t)__builtin_ctzll(b);
                    b &= b - 1u;
                    const uint32_t rl = (uint32_t)__builtin_amdgcn_readlane((int)r, (int)L);
                    table_pre(tabs + (wbase + L) * kNamStride, rl, lane);
                    if (lane == L) top = mine[100];
                }
            }
        }
    }
    if (!live) return;
    // the segment's first non-zero node is the anchor unless an earlier segment or shard has one
    if (cand) {
        const uint32_t sc = before ? cand_sreg : cand_sanc;
        best = umax64(best, make_key(sc, tb_hash(A, cand_ord), cand_ord));
    }
    if (best) atomicMax(keys + p, best);
}

// The pods of a chunk in name-digit order (digits 0..9, then the rest): perm[i]
// = the pod index lane i of k_nam_keys takes. One workgroup, LDS counting sort.
__global__ __launch_bounds__(1024) void k_nam_perm(const ms_pod_rec *__restrict__ pods, uint32_t n,
                                                   uint32_t *__restrict__ perm) {
    __shared__ uint32_t cnt[11], off[11];
    const uint32_t tid = threadIdx.x;
    if (tid < 11u) cnt[tid] = 0u;
    __syncthreads();
    auto cls = [&](uint32_t i) {
        const int d = pods[i].name_digit;
        return d >= 0 && d <= 9 ? (uint32_t)d : 10u;
    };
    for (uint32_t i = tid; i < n; i += 1024u) atomicAdd(&cnt[cls(i)], 1u);
    __syncthreads();
    if (tid == 0) {
        uint32_t a = 0;
        for (int k = 0; k < 11; ++k) {
            off[k] = a;
            a += cnt[k];
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < n; i += 1024u) perm[atomicAdd(&off[cls(i)], 1u)] = i;
}

inline uint32_t cdiv(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

}  // namespace

uint32_t nam_segments(uint32_t n_rows, uint32_t *seg_rows) {
    uint32_t sr = std::max(kNamSegRows, cdiv(std::max(n_rows, 1u), kNamMaxSegs));
    sr = cdiv(sr, kNamTile) * kNamTile;
    if (seg_rows) *seg_rows = sr;
    return std::max(1u, cdiv(n_rows, sr));
}

hipError_t launch_nam_seg(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                          const void *sets, uint32_t n_sets, void *segs, hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    uint32_t sr = 0;
    const uint32_t ns = nam_segments(n_rows, &sr);
    hipLaunchKernelGGL(k_nam_seg, dim3(cdiv(n_pods, kNamThreads), ns), dim3(kNamThreads), 0, s, t, n_rows, sr, pods,
                       n_pods, static_cast<const ms_nam_term_set *>(sets), n_sets, static_cast<NamSeg *>(segs));
    return hipGetLastError();
}

hipError_t launch_nam_compose(const void *in, uint32_t stride, uint32_t n, uint32_t n_pods, int32_t skip_to,
                              void *out, uint8_t *m_in, hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    hipLaunchKernelGGL(k_nam_compose, dim3(cdiv(n_pods, kNamComposeThreads)), dim3(kNamComposeThreads), 0, s, static_cast<const NamSeg *>(in),
                       stride, n, n_pods, skip_to, static_cast<NamSeg *>(out), m_in);
    return hipGetLastError();
}

hipError_t launch_nam_keys(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                           const void *sets, uint32_t n_sets, uint32_t seed32, uint32_t w_nn, uint32_t w_na,
                           const void *local, const void *after, const uint8_t *m_in, unsigned long long *keys,
                           uint32_t *perm, hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    uint32_t sr = 0;
    const uint32_t ns = nam_segments(n_rows, &sr);
    if (perm) hipLaunchKernelGGL(k_nam_perm, dim3(1), dim3(1024), 0, s, pods, n_pods, perm);
    hipLaunchKernelGGL(k_nam_keys, dim3(cdiv(n_pods, kNamThreads), ns), dim3(kNamThreads), 0, s, t, n_rows, sr, pods,
                       n_pods, static_cast<const ms_nam_term_set *>(sets), n_sets, seed32, w_nn, w_na,
                       static_cast<const NamSeg *>(local), ns, static_cast<const NamSeg *>(after), m_in, keys,
                       static_cast<const uint32_t *>(perm));
    return hipGetLastError();
}

}  // namespace msgpu
