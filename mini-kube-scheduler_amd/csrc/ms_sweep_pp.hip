// ms_sweep_pp.hip — K1 "pp", the production NU+NN sweep: for every (pod, node)
// pair it evaluates NodeUnschedulable and NodeNumber, and selectHost's argmax
// with the deterministic tie-break.
//
// Reference path (/root/reference/minisched/minisched.go):
//   RunFilterPlugins :115-151 -> NodeUnschedulable.Filter (k8s@v1.22.0, restated)
//   RunScorePlugins  :164-199 -> NodeNumber.Score (plugins/score/nodenumber/nodenumber.go:73-95)
//   unweighted sum   :187-196
//   selectHost       :304-325 (rand.Intn tie-break -> rule r3, minisched_gpu.h)
//
// Bit-sliced evaluation. The node table keeps, per group of 30 consecutive
// rows, bit planes (ms_internal.h kPlane*): the four bits of each row's
// name digit (15 = no digit), "present and schedulable" and "present" (and
// both restricted to digit names, plus a per-group flag word). A lane
// holds up to kPpWords groups in registers. For one pod and one group:
//   F = tolerates ? present : schedulable                     (NodeUnschedulable, 30 rows)
//   m = F & XNOR(d0, pod bit 0) & .. & XNOR(d3, pod bit 3)    (NodeNumber's 10, 30 rows)
// five v_bitop3 in all, each computing one boolean term for each of the 30
// (pod, row) pairs of the group: every pair's filter and score comes from its
// own row's bits and the pod's own bits. The rows set in m are the pairs that
// pass the filter with score 10; their tie-break hashes (mix32 of A + ordinal *
// kG24, rule r3) are the candidates of selectHost's max. A group of 30
// consecutive names holds at most 3 rows of one digit when the digits cycle, so
// three v_ffbl slots cover it with no lane-divergent loop; a tile where some
// lane has more (the wave-uniform `gen` flag, computed when the tile is
// loaded) takes a bit-scan loop instead. Rows scoring 0 matter only when no
// feasible row of the wave scores 10: the wave's maximum is then 0 and the pod
// is redone by the exact slow path (every feasible row hashed, explicit
// found flags), which also covers non-digit pods.
// Fixed-slot form (word_fix): where every present digit-named row of a
// wave's groups has digit == ordinal mod 10 (the digit-aligned allocator's
// layout, and the synthetic clusters'), the pod's digit can only sit at three
// known slots, so the per-pod mask is one v_bitop3 and the slots need no
// search: 24 VALU per pod and group instead of 31, same keys bit for bit.
//
// Grid: a workgroup holds ALL of the context's rows (up to 16 waves x 64 lanes
// x kPpWords groups = 122,880 rows; more rows split over grid.y and combine
// with atomicMax) and sweeps a chunk of pods through them, 8 pods at a time.
// The 8 lane maxima are reduced by one transposed butterfly (reduce8), the
// waves combine in LDS (ds_max_u64 of level<<32 | hash), and after one barrier
// the workgroup unhashes each pod's winner (tb_unhash) and writes either the
// packed key (ms_sweep_device: one plain store per pod, no zeroing, no
// atomics) or the decoded ms_result directly (the fused single-shard cycle).
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>

#include "ms_device.h"

namespace msgpu {

namespace {

template <typename F>
constexpr uint32_t truth3(F f) {  // v_bitop3 table, S0 the most significant index bit
    uint32_t t = 0;
    for (int i = 0; i < 8; ++i)
        if (f((i >> 2) & 1, (i >> 1) & 1, i & 1)) t |= 1u << i;
    return t;
}
constexpr uint32_t kXnorAnd = truth3([](int a, int b, int c) { return c && a == b; });  // c & ~(a ^ b)
constexpr uint32_t kSelect = truth3([](int a, int b, int c) { return c ? a : b; });     // c ? a : b

#ifndef MS_TAIL_PACK
#define MS_TAIL_PACK 1  // (0: the last partial word as a full one, A/B)
#endif
#ifndef MS_TAIL_SHARE
#define MS_TAIL_SHARE 4  // waves sharing the packed last word (A/B)
#endif

constexpr int kPpWords = 4;      // 30-row groups per lane (KW, shards above kPpSmallGroups)
constexpr int kPpWordsSmall = 8; // KW for small shards: one wave holds every row
constexpr int kPpMaxWaves = 16;  // 1024-thread workgroups
constexpr uint32_t kPpSmallGroups = 64u * kPpWordsSmall;  // 15,360 rows

struct Word {
    uint32_t d0, d1, d2, d3;  // digit bit planes
    uint32_t sched, pres;     // present & schedulable, present
    uint32_t dsched, dpres;   // the same restricted to rows whose name ends in a digit
    uint32_t hb;              // (ordinal of the group's row 0) * kG24
};

// One pod as the wave sees it (all wave-uniform, SGPRs).
struct Pod {
    uint32_t A;               // tb_pod(seed32, ordinal)
    uint32_t s0, s1, s2, s3;  // digit bit i as 0 / ~0 (non-digit pods: 14, which no node has)
    uint32_t tol;             // tolerates node.kubernetes.io/unschedulable: 0 / ~0
    // fixed-slot form (groups whose rows' digits equal their ordinals mod 10):
    // the three slots of the pod's digit, p0 = (digit - node_base) mod 10, p0 + 10,
    // p0 + 20 (non-digit pods: 30, a bit no group sets), and A + p_j * kG24
    uint32_t p0, p1, p2;
    uint32_t A0, A1, A2;
};

#define MS_BITOP3(a, b, c, imm) __builtin_amdgcn_bitop3_b32((a), (b), (c), (imm))

__device__ __forceinline__ uint32_t feasible(const Word &w, const Pod &q) {
    return MS_BITOP3(w.pres, w.sched, q.tol, kSelect);
}

// Rows of the group that pass NodeUnschedulable and score NodeNumber's 10.
__device__ __forceinline__ uint32_t match10(const Word &w, const Pod &q) {
    uint32_t m = MS_BITOP3(w.d0, q.s0, feasible(w, q), kXnorAnd);
    m = MS_BITOP3(w.d1, q.s1, m, kXnorAnd);
    m = MS_BITOP3(w.d2, q.s2, m, kXnorAnd);
    return MS_BITOP3(w.d3, q.s3, m, kXnorAnd);
}

// Leading zeros (v_ffbh_u32; 0xFFFFFFFF for an empty mask).
__device__ __forceinline__ uint32_t last_lz(uint32_t m) {
    uint32_t s;
    asm("v_ffbh_u32 %0, %1" : "=v"(s) : "v"(m));
    return s;
}

__device__ __forceinline__ uint32_t hash_slot(uint32_t slot, uint32_t hbA) {
    return mix32(__umul24(slot, kG24) + hbA);  // A + (row0 + slot) * kG24, rule r3
}

// Lane maximum hash over the group's score-10 rows, at most 3 of them (the
// tile's `gen` flag is clear): the lowest (v_ffbl), the highest (v_ffbh) and
// the lowest of the rest, which falls back to the lowest when fewer than 3
// (a duplicate leaves the max unchanged); an empty mask gives 0.
__device__ __forceinline__ uint32_t word_fast(const Word &w, const Pod &q) {
    const uint32_t m = match10(w, q);
    const uint32_t hbA = w.hb + q.A;
    const int i0 = (int)first_slot(m);
    const int i2 = 31 - (int)last_lz(m);
    const int i1 = max((int)first_slot(m & (m - 1u)), i0);
    const uint32_t h = max(max(hash_slot((uint32_t)i0, hbA), hash_slot((uint32_t)i1, hbA)),
                           hash_slot((uint32_t)i2, hbA));
    return m ? h : 0u;
}

// Any number of score-10 rows per lane: a bit-scan loop (lane-divergent trip count).
__device__ __forceinline__ uint32_t word_scan(uint32_t m, uint32_t hbA) {
    uint32_t h = 0;
    while (m) {
        const uint32_t s = first_slot(m);
        m &= m - 1u;
        h = max(h, hash_slot(s, hbA));
    }
    return h;
}

// info: the pod entry's class bits (pod_entry), the fixed slot p0 in bits 16-20.
__device__ __forceinline__ Pod pod_bits(uint32_t A, uint32_t info) {
    Pod q;
    q.A = A;
    q.s0 = (info & 1u) ? ~0u : 0u;
    q.s1 = (info & 2u) ? ~0u : 0u;
    q.s2 = (info & 4u) ? ~0u : 0u;
    q.s3 = (info & 8u) ? ~0u : 0u;
    q.tol = (info & 16u) ? ~0u : 0u;
    q.p0 = (info >> 16) & 31u;  // (30 for a non-digit pod: p1 = p2 = 30 too)
    const uint32_t step = q.p0 < 10u ? 10u : 0u;
    q.p1 = q.p0 + step;
    q.p2 = q.p1 + step;
    q.A0 = A + q.p0 * kG24;
    q.A1 = q.A0 + 10u * kG24;
    q.A2 = q.A0 + 20u * kG24;
    return q;
}

// Fixed-slot form: in a group where every present row's name digit is its
// ordinal mod 10 (the digit-aligned allocator's layout, ms_nodes_upsert docs),
// the rows of the pod's digit can only sit at slots p0, p0 + 10, p0 + 20, and
// such a row scores NodeNumber's 10 exactly when its name ends in a digit. So
// the filter-and-score mask of the group is ONE v_bitop3 over the digit-name
// planes (NodeUnschedulable with the toleration, as feasible()), and the
// three candidates need no slot search: each hash input is hb + A_j, zeroed by
// its slot's bit (v_bfe_i32 gives 0 / ~0; mix32(0) = 0, the empty value).
__device__ __forceinline__ uint32_t match_fix(const Word &w, const Pod &q) {
    return MS_BITOP3(w.dpres, w.dsched, q.tol, kSelect);
}

__device__ __forceinline__ uint32_t word_fix(const Word &w, const Pod &q) {
    const uint32_t m = match_fix(w, q);
    const uint32_t k0 = (uint32_t)__builtin_amdgcn_sbfe((int)m, (int)q.p0, 1);
    const uint32_t k1 = (uint32_t)__builtin_amdgcn_sbfe((int)m, (int)q.p1, 1);
    const uint32_t k2 = (uint32_t)__builtin_amdgcn_sbfe((int)m, (int)q.p2, 1);
    uint32_t x0 = (w.hb + q.A0) & k0, x1 = (w.hb + q.A1) & k1, x2 = (w.hb + q.A2) & k2;
    // (opaque: left visible, the compiler folds the AND into a v_bitop3 with the
    // first xor-shift and pays a separate shift for it, one VALU more per slot)
    asm("" : "+v"(x0), "+v"(x1), "+v"(x2));
    return max(max(mix32(x0), mix32(x1)), mix32(x2));
}

// Exact evaluation of one pod over the wave's NW groups, with explicit found
// flags: level 11 (score 10 + 1) over the score-10 rows, else level 1 over
// every feasible row (all score 0). Returns level<<32 | max hash (wave-uniform),
// 0 when no row of the wave is feasible.
// tail: the wave's packed last word (below) is evaluated here like a full one:
// its groups repeat in every lane segment, and repeats leave the max unchanged.
// FIX: the wave's words are digit-aligned (word_fix): the score-10 rows are
// the fixed slots' digit-name rows.
template <int KW, int NW, bool FIX>
__device__ __forceinline__ u64 pod_slow(const Word (&W)[KW], const Word &Wt, bool tail, const Pod &q) {
    uint32_t h = 0;
    bool found = false;
    const uint32_t cmask = (1u << q.p0) | (1u << q.p1) | (1u << q.p2);  // (non-digit pods: bit 30, never set)
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint32_t m = FIX ? match_fix(W[k], q) & cmask : match10(W[k], q);
        found = found || m != 0;
        h = max(h, word_scan(m, W[k].hb + q.A));
    }
    if (tail) {
        const uint32_t m = match10(Wt, q);
        found = found || m != 0;
        h = max(h, word_scan(m, Wt.hb + q.A));
    }
    if (__ballot(found) != 0) return (11ull << 32) | wave_max_u32_dpp(h);
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint32_t m = feasible(W[k], q);
        found = found || m != 0;
        h = max(h, word_scan(m, W[k].hb + q.A));
    }
    if (tail) {
        const uint32_t m = feasible(Wt, q);
        found = found || m != 0;
        h = max(h, word_scan(m, Wt.hb + q.A));
    }
    if (__ballot(found) != 0) return (1ull << 32) | wave_max_u32_dpp(h);
    return 0;
}

// Pod p of a workgroup's chunk as the prologue leaves it in LDS: x = A =
// tb_pod(seed32, ordinal), y = class bits (digit, 14 for a non-digit name, |
// tolerates << 4) | name digit byte << 8 | the fixed slot p0 << 16 ((digit -
// node_base) mod 10, 30 for a non-digit name: word_fix).
// pstride: bytes per pod record (sizeof(ms_pod_rec), or 8 for ms_pod_compact,
// its first 8 bytes).
__device__ __forceinline__ uint2 pod_entry(const ms_pod_rec *__restrict__ pods, uint32_t p, uint32_t seed32,
                                           uint32_t pstride, uint32_t base10) {
    const uint2 pr = *reinterpret_cast<const uint2 *>(reinterpret_cast<const char *>(pods) + (size_t)p * pstride);
    const int dig = (int)(int8_t)(pr.y & 0xFFu);
    const bool isd = (uint32_t)dig <= 9u;
    const uint32_t info = (isd ? (uint32_t)dig : 14u) | (((pr.y >> 8) & 0xFFu) ? 16u : 0u);
    const uint32_t p0 = isd ? ((uint32_t)dig + 10u - base10) % 10u : 30u;
    return make_uint2(tb_pod(seed32, pr.x), info | ((pr.y & 0xFFu) << 8) | (p0 << 16));
}

// One wave sweeps the chunk's pods [0, np) through its NW words into lds[p].
// tpt != 0: the wave also holds the workgroup's packed last word Wt, whose
// T <= 64 / tpt groups repeat in tpt lane segments of 64 / tpt lanes: segment
// i evaluates pod i of a group of tpt pods (its bits from the lanes' block
// entries by ds_bpermute), so a partial word costs 8 / tpt evaluations per 8
// pods instead of 8; and up to 4 waves (on different SIMDs) hold it, wave
// tidx of tshare taking the 8-pod blocks b with b mod tshare == tidx. (A
// partial word holding the full cost on one SIMD was 6 % of config C:
// 100,000 rows 323 us, 99,840 rows 303 us, profiles/r03zd_tail.json.)
// MODE: kModeFast (three slots found by bit scans, word_fast), kModeGen (some
// group of the wave holds more than 3 rows of a digit: the bit-scan loop),
// kModeFix (every group of the wave is digit-aligned: word_fix).
constexpr int kModeFast = 0, kModeGen = 1, kModeFix = 2;

template <int KW, int NW, int MODE, bool TAIL>
__device__ __forceinline__ void sweep_range(const Word (&W)[KW], const Word &Wt, uint32_t tpt, uint32_t tshare,
                                            uint32_t tidx, const uint2 *pinfo, uint32_t np, uint32_t lane, u64 *lds) {
    constexpr bool GEN = MODE == kModeGen;
    const uint32_t seg_shift = tpt == 8u ? 3u : tpt == 4u ? 4u : 5u;  // log2(64 / tpt)
    for (uint32_t pb = 0; pb < np; pb += 64) {
        const uint32_t nblk = min(64u, np - pb);
        // the block's pods, one per lane: A and digit | tolerates << 4
        uint32_t a_l = 0, info_l = 14u | (30u << 16);  // (lanes past the block: no row matches)
        if (lane < nblk) {
            const uint2 e = pinfo[pb + lane];
            a_l = e.x;
            info_l = e.y;
        }
        for (uint32_t j = 0; j < nblk; j += 8) {
            Pod q[8];
#pragma unroll
            for (int t = 0; t < 8; ++t)
                q[t] = pod_bits((uint32_t)__builtin_amdgcn_readlane((int)a_l, (int)(j + t)),
                                (uint32_t)__builtin_amdgcn_readlane((int)info_l, (int)(j + t)));
            uint32_t r[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                uint32_t h = 0;
#pragma unroll
                for (int k = 0; k < NW; ++k)
                    h = max(h, MODE == kModeGen ? word_scan(match10(W[k], q[t]), W[k].hb + q[t].A)
                               : MODE == kModeFix ? word_fix(W[k], q[t])
                                                  : word_fast(W[k], q[t]));
                r[t] = h;
            }
            if (TAIL && ((pb + j) >> 3) % tshare == tidx) {  // wave-uniform
                const uint32_t seg = lane >> seg_shift;
                for (uint32_t e = 0; e < 8u; e += tpt) {
                    // lanes of segment seg: pod j + e + seg of the block (past nblk: A 0 and
                    // class 14, which no row matches, so h stays 0)
                    const int src = (int)(j + e + seg) << 2;
                    const Pod qt = pod_bits((uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)a_l),
                                            (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)info_l));
                    const uint32_t h = GEN ? word_scan(match10(Wt, qt), Wt.hb + qt.A) : word_fast(Wt, qt);
#pragma unroll
                    for (int t = 0; t < 8; ++t)
                        if ((uint32_t)t >= e && (uint32_t)t < e + tpt) r[t] = max(r[t], seg == (uint32_t)t - e ? h : 0u);
                }
            }
            const uint32_t u = reduce8(r, lane);
            const uint32_t pi = j + rev3(lane >> 3);  // lanes 8k: pod pi of the block
            const bool mine = (lane & 7u) == 0u && pi < nblk;
            if (mine && u != 0u) atomicMax(&lds[pb + pi], (11ull << 32) | u);
            // a zero maximum: no score-10 row in this wave (or one whose hash is 0);
            // redo those pods exactly
            u64 redo = __ballot(mine && u == 0u);
            while (redo) {
                const uint32_t l = (uint32_t)__builtin_ctzll(redo);
                redo &= redo - 1ull;
                const uint32_t t = rev3(l >> 3);
                const Pod qs = pod_bits((uint32_t)__builtin_amdgcn_readlane((int)a_l, (int)(j + t)),
                                        (uint32_t)__builtin_amdgcn_readlane((int)info_l, (int)(j + t)));
                const u64 v = pod_slow<KW, NW, MODE == kModeFix>(W, Wt, TAIL && ((pb + j) >> 3) % tshare == tidx, qs);
                if (lane == 0 && v) atomicMax(&lds[pb + j + t], v);
            }
        }
    }
}

// KW words per lane: 4 (workgroups of up to 16 waves split the rows) or 8 for
// shards of at most kPpSmallGroups groups, where ONE wave holds every row: then
// every wave does the same work whatever SIMD it lands on (with 4 words a
// 12.5k-row shard dealt over 4 waves gave them 2, 2, 2 and 1 words, and the
// SIMD that hosts the short waves idled), and the per-pod reduction is paid
// once per 7 words instead of once per 2.
// Pods per evaluation of a workgroup's packed last word (sweep_range): 8 for a
// last word of <= 8 groups, 0 when it stays a full word (sweep_range also
// takes 4 and 2: 16 and 32 groups). ng
// groups over `waves` waves. Packed only where that lowers the busiest SIMD's
// load (waves w and w + 4 of a workgroup share a SIMD): words per SIMD, in
// sixteenths, with and without it (100,000 rows over 16 waves: 14 -> 13.06;
// 50,010 over 8: 7 either way, and packing cost 1 %).
__host__ __device__ inline uint32_t tail_pods(uint32_t ng, uint32_t waves) {
    if (!MS_TAIL_PACK || ng == 0) return 0u;
    const uint32_t wlast = (ng + 63u) / 64u - 1u, tail_n = ng - wlast * 64u;
    // (8 pods per evaluation only: 2 per evaluation, 17 groups left over a
    // 6,250-row wave, cost more than the full word, profiles/r03zk_tail_pack_ab.txt)
    const uint32_t tpt = tail_n <= 8u ? 8u : 0u;
    if (!tpt) return 0u;
    // up to 4 waves: several workgroups share a CU and the hardware rotates
    // their waves over the SIMDs (profiles/r03z_hwid_placement.txt), so every
    // word saved is saved on every SIMD
    if (waves <= 4u) return tpt;
    const uint32_t wv_t = wlast % waves;
    const uint32_t tshare = (uint32_t)MS_TAIL_SHARE < waves - wv_t ? (uint32_t)MS_TAIL_SHARE : waves - wv_t;
    uint32_t L[4] = {0, 0, 0, 0};
    for (uint32_t w = 0; w < waves && w <= wlast; ++w) L[w & 3u] += 16u * ((wlast - w) / waves + 1u);
    auto mx = [&] {
        const uint32_t a = L[0] > L[1] ? L[0] : L[1], b = L[2] > L[3] ? L[2] : L[3];
        return a > b ? a : b;
    };
    const uint32_t m0 = mx();
    L[wv_t & 3u] -= 16u;
    const uint32_t eps = ((tpt == 8u ? 4u : tpt == 4u ? 8u : 12u) + tshare - 1u) / tshare;
    for (uint32_t i = 0; i < tshare; ++i) L[(wv_t + i) & 3u] += eps;
    return mx() < m0 ? tpt : 0u;
}

// A second batch swept by the same launch (shard sweeps with key output only:
// ms_sharded_submit coalesces two consecutive submits into one launch, paying
// the per-launch ramp and drain once). Workgroups nblk1.. take its chunks.
struct PpJob2 {
    const ms_pod_rec *pods;  // nullptr: one batch
    u64 *keys;
    uint32_t n_pods, nblk1;
};

// TP: the packed-last-word path is compiled in (launch_sweep_pp picks it only
// for shapes tail_pods packs; the others run the plain form).
template <int KW, bool TP>
__global__ __launch_bounds__(64 * kPpMaxWaves) void k_sweep_nunn_pp(
    const uint32_t *__restrict__ planes, uint32_t gstride, uint32_t n_groups, uint32_t node_base,
    const ms_pod_rec *__restrict__ pods1, uint32_t n_pods1, uint32_t chunk, uint32_t seed32, u64 *__restrict__ keys1,
    int atomic_keys, ms_result *__restrict__ results, uint32_t present, NodeTable tab, int commit,
    uint32_t pstride, ms_result_compact *__restrict__ resc, PpJob2 j2, int fix_ok, uint32_t xtra) {
    // LDS: one combine slot per pod of the chunk, then the chunk's pod entries
    // (xtra: workgroups 0 .. xtra-1 take chunk + 8 pods, the balanced split)
    extern __shared__ u64 lds[];
    uint2 *pinfo = reinterpret_cast<uint2 *>(lds + chunk + (xtra ? 8u : 0u));
    const uint32_t lane = lane_id();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const bool second = j2.pods && blockIdx.x >= j2.nblk1;  // (workgroup-uniform)
    const ms_pod_rec *__restrict__ pods = second ? j2.pods : pods1;
    const uint32_t n_pods = second ? j2.n_pods : n_pods1;
    u64 *__restrict__ keys = second ? j2.keys : keys1;
    const uint32_t bi = second ? blockIdx.x - j2.nblk1 : blockIdx.x;
    const uint32_t pbeg = bi * chunk + min(bi, xtra) * 8u;
    const uint32_t pend = min(n_pods, pbeg + chunk + (bi < xtra ? 8u : 0u));
    const uint32_t np = pend > pbeg ? pend - pbeg : 0u;
    for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) {
        lds[i] = 0;
        pinfo[i] = pod_entry(pods, pbeg + i, seed32, pstride, node_base % 10u);
    }

    // the wave's groups, dealt round-robin over the workgroup's waves so their
    // word counts differ by at most one: word k of lane l is group
    // g0 + (k * waves + wv) * 64 + l. The workgroup's last word, when it holds
    // T <= 32 groups, is packed instead (sweep_range): its wave loads group
    // (lane mod 64/tpt) of it into Wt.
    const uint32_t waves = blockDim.x >> 6;
    const uint32_t g0 = blockIdx.y * waves * 64u * KW;
    const uint32_t ng = min(n_groups - g0, waves * 64u * KW);  // (blockIdx.y < gy: g0 < n_groups)
    const uint32_t wlast = (ng + 63u) / 64u - 1u, tail_n = ng - wlast * 64u;
    uint32_t tpt = TP ? tail_pods(ng, waves) : 0u;
    const uint32_t wv_t = wlast % waves, tshare = min((uint32_t)MS_TAIL_SHARE, waves - wv_t);  // its waves
    const bool owner = wv == wv_t;     // it is this wave's last word in the dealing
    if (wv < wv_t || wv >= wv_t + tshare) tpt = 0u;  // wave-uniform
    Word W[KW], Wt;
    int nw = 0;
    bool over = false, misaligned = false;
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        const uint32_t wi = k * waves + wv;
        const uint32_t gw = g0 + wi * 64u;
        const uint32_t g = gw + lane;
        const bool in = g < n_groups && !(tpt && owner && wi == wlast);
        if (gw < n_groups && !(tpt && owner && wi == wlast)) nw = k + 1;  // wave-uniform
        W[k].d0 = in ? planes[kPlaneD0 * gstride + g] : 0u;
        W[k].d1 = in ? planes[kPlaneD1 * gstride + g] : 0u;
        W[k].d2 = in ? planes[kPlaneD2 * gstride + g] : 0u;
        W[k].d3 = in ? planes[kPlaneD3 * gstride + g] : 0u;
        W[k].sched = in ? planes[kPlaneSched * gstride + g] : 0u;
        W[k].pres = in ? planes[kPlanePresent * gstride + g] : 0u;
        W[k].dsched = in ? planes[kPlaneDigitSched * gstride + g] : 0u;
        W[k].dpres = in ? planes[kPlaneDigitPres * gstride + g] : 0u;
        W[k].hb = (node_base + g * kGroupRows) * kG24;
        const uint32_t ov = in ? planes[kPlaneOver * gstride + g] : 0u;
        // more than 3 present rows of one digit in a group: the fast slots cannot hold them
        over = over || (ov & 1u) != 0u;
        misaligned = misaligned || (ov & 2u) != 0u;
    }
    {
        const uint32_t gi = tpt ? lane & ((64u / tpt) - 1u) : 0u;
        const uint32_t g = g0 + wlast * 64u + gi;
        const bool in = tpt && gi < tail_n;
        Wt.d0 = in ? planes[kPlaneD0 * gstride + g] : 0u;
        Wt.d1 = in ? planes[kPlaneD1 * gstride + g] : 0u;
        Wt.d2 = in ? planes[kPlaneD2 * gstride + g] : 0u;
        Wt.d3 = in ? planes[kPlaneD3 * gstride + g] : 0u;
        Wt.sched = in ? planes[kPlaneSched * gstride + g] : 0u;
        Wt.pres = in ? planes[kPlanePresent * gstride + g] : 0u;
        Wt.hb = (node_base + g * kGroupRows) * kG24;
        Wt.dsched = Wt.dpres = 0u;  // (the packed word always takes word_fast / word_scan)
        over = over || (in && (planes[kPlaneOver * gstride + g] & 1u) != 0u);
    }
    const bool gen = __ballot(over) != 0;
    // every word of the wave digit-aligned (MINISCHED_PP_FIX=0 at launch: never)
    const int mode = gen ? kModeGen : (fix_ok && __ballot(misaligned) == 0) ? kModeFix : kModeFast;
    __syncthreads();
    if (np && (nw || tpt)) {
        switch (nw * 6 + mode * 2 + (tpt ? 1 : 0)) {  // wave-uniform
#define MS_PP_CASE1(N, M, T)                                                                                     \
    case 6 * N + 2 * M + T:                                                                                      \
        if constexpr (N <= KW && (N > 0 || T))                                                                   \
            sweep_range<KW, (N <= KW ? N : KW), M, T>(W, Wt, tpt, tshare, wv - wv_t, pinfo, np, lane, lds);         \
        break;
#define MS_PP_CASE(N)        \
    MS_PP_CASE1(N, 0, false) \
    MS_PP_CASE1(N, 0, true)  \
    MS_PP_CASE1(N, 1, false) \
    MS_PP_CASE1(N, 1, true)  \
    MS_PP_CASE1(N, 2, false) \
    MS_PP_CASE1(N, 2, true)
            MS_PP_CASE(0)
            MS_PP_CASE(1)
            MS_PP_CASE(2)
            MS_PP_CASE(3)
            MS_PP_CASE(4)
            MS_PP_CASE(5)
            MS_PP_CASE(6)
            MS_PP_CASE(7)
            MS_PP_CASE(8)
#undef MS_PP_CASE
#undef MS_PP_CASE1
            default:
                break;  // no groups in this wave
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) {
        const u64 v = lds[i];
        const uint2 pe = pinfo[i];
        u64 key = present ? kKeyListed : 0ull;  // no feasible row: listed or not (decode_key)
        if (v) {
            const uint32_t h = (uint32_t)v;
            key = make_key((uint32_t)(v >> 32) - 1u, h, tb_unhash(pe.x, h));
        }
        if (keys) {
            if (!atomic_keys) keys[pbeg + i] = key;
            else if (key) atomicMax(&keys[pbeg + i], key);
        }
        if (results || resc) {
            const ms_result r = decode_key(key, (int8_t)(pe.y >> 8), nullptr, 0, present);
            if (results) {
                results[pbeg + i] = r;
            } else {  // the compact record, straight into the caller's (pinned host) array
                ms_result_compact rc;
                rc.node = r.node;
                rc.score = (uint16_t)r.score;
                rc.code = (uint8_t)r.code;
                rc.plugin_mask = (uint8_t)r.plugin_mask;
                resc[pbeg + i] = rc;
            }
            // assume-on-select in the same launch (ms_schedule_batch / the sequential
            // NU+NN cycle): NodeInfo.AddPod on the winner, which this context owns
            // (one workgroup holds all its rows); a compact pod requests nothing
            if (commit && r.code == MS_CODE_SUCCESS) {
                if (resc) {
                    const ms_pod_rec z = {};
                    add_pod(tab, (uint32_t)r.node - tab.base, z, +1);
                } else {
                    add_pod(tab, (uint32_t)r.node - tab.base, pods[pbeg + i], +1);
                }
            }
        }
    }
}

// Bit planes of one 30-row group from the SoA columns (flags, digit).
__device__ __forceinline__ void build_group(const NodeTable &t, uint32_t g) {
    uint32_t d[4] = {0, 0, 0, 0}, sched = 0, pres = 0, isdig = 0, misal = 0;
    for (uint32_t s = 0; s < kGroupRows; ++s) {
        const uint32_t r = g * kGroupRows + s;
        if (r >= t.cap) break;
        const uint32_t f = t.flags[r], dg = t.digit[r];
        const uint32_t v = dg <= 9u ? dg : 15u;
#pragma unroll
        for (int b = 0; b < 4; ++b) d[b] |= ((v >> b) & 1u) << s;
        if (!(f & kNodeAbsent)) {
            pres |= 1u << s;
            if (!(f & kNodeUnschedulable)) sched |= 1u << s;
            if (v <= 9u) {
                isdig |= 1u << s;
                if (v != (t.base + r) % 10u) misal = 2u;  // digit != ordinal mod 10
            }
        }
    }
    uint32_t over = misal;
#pragma unroll
    for (int v = 0; v < 10; ++v) {
        const uint32_t m = pres & ((v & 1) ? d[0] : ~d[0]) & ((v & 2) ? d[1] : ~d[1]) & ((v & 4) ? d[2] : ~d[2]) &
                           ((v & 8) ? d[3] : ~d[3]);
        over |= __popc(m) > 3 ? 1u : 0u;
    }
    const uint32_t st = t.gcap;
    t.planes[kPlaneDigitPres * st + g] = pres & isdig;
    t.planes[kPlaneDigitSched * st + g] = sched & isdig;
    t.planes[kPlaneOver * st + g] = over;
    t.planes[kPlaneD0 * st + g] = d[0];
    t.planes[kPlaneD1 * st + g] = d[1];
    t.planes[kPlaneD2 * st + g] = d[2];
    t.planes[kPlaneD3 * st + g] = d[3];
    t.planes[kPlaneSched * st + g] = sched;
    t.planes[kPlanePresent * st + g] = pres;
}

// deltas != nullptr: the groups of the applied deltas (a group rebuilt twice gets the
// same bits: the deltas' column writes finished in the previous launch); else all groups.
__global__ void k_build_planes(NodeTable t, const NodeDelta *__restrict__ deltas, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t g = deltas ? deltas[i].local / kGroupRows : i;
    if (g < t.gcap) build_group(t, g);
}

inline uint32_t cdiv(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

}  // namespace

hipError_t launch_build_planes(const NodeTable &t, const NodeDelta *d_deltas, uint32_t n, hipStream_t s) {
    if (!t.planes) return hipSuccess;
    if (!d_deltas) n = t.gcap;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_build_planes, dim3(cdiv(n, 256)), dim3(256), 0, s, t, d_deltas, n);
    return hipGetLastError();
}

// Geometry: W waves (<= 16) of up to 256 groups each hold the rows (more
// rows: grid.y workgroups per chunk); pods per workgroup sized for one
// round of resident workgroups (16 waves per CU while chunks stay <= 1024
// pods, else 32) in multiples of 8, at most kPpMaxChunk (LDS).
// MINISCHED_PP_CHUNK overrides the chunk (tuning).
constexpr uint32_t kPpMaxChunk = 2048;

namespace {
hipError_t sweep_pp_impl(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                         uint32_t seed32, unsigned long long *keys, ms_result *results, uint32_t present, int num_cus,
                         hipStream_t s, int commit, hipEvent_t done, uint32_t pstride, ms_result_compact *resc,
                         const ms_pod_rec *pods2 = nullptr, uint32_t n_pods2 = 0, unsigned long long *keys2 = nullptr) {
    if (n_pods == 0 && n_pods2 == 0) return done ? hipEventRecord(done, s) : hipSuccess;
    // (two batches: shard sweeps into keys, one workgroup holding every row)
    const uint32_t n_all = n_pods + (pods2 ? n_pods2 : 0u);
    if (!t.planes) return hipErrorInvalidValue;
    const uint32_t n_groups = cdiv(n_rows, kGroupRows);
    // small shards with many pods: KW = 8, one single-wave workgroup per pod
    // chunk holds every row. It needs enough pods per wave to balance whole
    // waves over the SIMDs: 12.5k rows x 800k pods 347 vs 412 us, but x 100k
    // pods 58.8 vs 52.7 us (profiles/r03_pp_words_ab.txt): a line through the
    // two crosses near 160k pods, and a coalesced pair of 100k-pod batches
    // (200k) still ran faster at KW = 4 (53.5 vs 54.5 us per batch,
    // profiles/r04f_coalesce_probe.txt), so the form switches at 1024 pods per
    // CU. MINISCHED_PP_WORDS = 4 / 8 forces a form (A/B).
    const char *wenv = getenv("MINISCHED_PP_WORDS");
    const uint32_t cus_ = (uint32_t)(num_cus > 0 ? num_cus : 256);
    bool small = n_groups <= kPpSmallGroups && n_all >= 1024u * cus_ && !getenv("MINISCHED_PP_WAVES");
    if (wenv) small = n_groups <= kPpSmallGroups && atoi(wenv) == 8;
    const uint32_t KW = small ? (uint32_t)kPpWordsSmall : (uint32_t)kPpWords;
    const uint32_t waves_needed = std::max(1u, cdiv(n_groups, 64u * KW));
    // W a power of two (32 / W workgroups per CU fill all 8 wave slots per
    // SIMD; W = 7 leaves one idle and was 9% slower at 50k rows): large shards
    // 16-wave workgroups (the groups are dealt round-robin, so every wave holds
    // 3 or 4 words), shards of 257..2048 groups at least 4 waves
    // (profiles/r02c_ab.json, r02j_ab_shard_waves.jsonl)
    // Shards needing exactly 2 waves (257..512 groups) keep 2: with the fixed-slot
    // form's shorter words the 4-wave split (2, 2, 2, 1 words at 12.5k rows) paid the
    // per-8-pod reduction twice as often; the pipelined G = 8 step went 46.1 -> 43.9 us
    // (profiles/r04t_g8_w2.txt; the slot-search form was 53.7 -> 53.0, r04f).
    uint32_t W = 1;
    if (waves_needed == 2) W = 2;
    else if (waves_needed > 1)
        while (W < std::max(4u, waves_needed) && W < (uint32_t)kPpMaxWaves) W *= 2;
    if (const char *w = getenv("MINISCHED_PP_WAVES")) W = (uint32_t)std::min(16, std::max(1, atoi(w)));
    if (!keys) W = std::max(W, std::min<uint32_t>(kPpMaxWaves, waves_needed));  // no scratch: one workgroup per chunk
    const uint32_t gy = std::max(1u, cdiv(n_groups, W * 64u * KW));
    const uint32_t cus = (uint32_t)(num_cus > 0 ? num_cus : 256);
    // (multiples of 8: a wave takes pods 8 at a time, and a part-filled 8 costs
    // a full one -- exact chunks ran 11% slower at 25k rows, r02k_ab_chunk.txt)
    auto chunk_for = [&](uint32_t per_cu) {
        const uint32_t resident = std::max(1u, per_cu * cus / gy);
        return cdiv(cdiv(n_all, resident), 8) * 8;
    };
    uint32_t chunk = chunk_for(std::max(1u, 32u / W));  // one round at 32 waves per CU
    // Half as many workgroups (16 waves per CU, 4 per SIMD still saturate VALU
    // issue) while chunks stay modest: each workgroup's fixed costs (plane
    // loads, pod prologue, two barriers, epilogue) are paid half as often.
    // Config C 334 -> 324 us and 350 -> 341 us on two boxes; at 1M pods (chunks
    // near 2k) it was 1.3% slower, at 12.5k rows x 800k pods (784) 1.6% faster
    // (profiles/r02zb_ab_chunk_half.jsonl).
    if (32u / W > 1u && chunk_for(std::max(1u, 16u / W)) <= 1024u) chunk = chunk_for(std::max(1u, 16u / W));
    // (Chunks of <= 56 pods for <= 8-wave workgroups sped the shard sweep alone up,
    // 12.5k rows 44.3 -> 43.7 us, 25k 73.3 -> 71.0, 50k 133.0 -> 127.0, but slowed the
    // pipelined sharded step, whose collective and decode kernels then interleave with
    // a multi-round sweep: 74.6 -> 77.7 us at 25k, 136.3 -> 140 at 50k;
    // profiles/r04n_shard_shapes.txt, r04p_chunk56_probe.json. Not kept.)
    chunk = std::min(std::max(chunk, 8u), kPpMaxChunk);
    uint32_t nblk1 = cdiv(n_pods, chunk), xtra = 0;
    // Balanced split of a one-batch shard sweep (2- and 4-wave workgroups, one
    // round of 16 waves per CU): chunks rounded up to 8 leave some SIMDs a wave
    // short of others (12.5k rows x 100k pods: 1,786 workgroups of 56 pods over
    // 2,048 slots, 3.5 waves per SIMD, the busiest 4 x 56 pods). Instead every
    // slot gets a workgroup: `chunk` pods each, 8 more for the first `xtra`
    // (4 x 48.8 pods on the busiest SIMD): the shard sweep alone 42.0 -> 38.7 us
    // at G = 8, 71.5 -> 67.5 at G = 4 (profiles/r05r_balance_ab.txt).
    // A coalesced pair of equal batches splits the slots in halves, each balanced alike.
    if ((!pods2 || n_pods2 == n_pods) && gy == 1 && W <= 4u) {
        const uint32_t slots = (16u / W) * cus / (pods2 ? 2u : 1u);
        const uint32_t cb = (n_pods / slots) / 8u * 8u;
        if (cb >= 8u && cb + 8u <= kPpMaxChunk && n_pods > cb * slots) {
            const uint32_t nx = cdiv(n_pods - cb * slots, 8u);
            if (nx <= slots) {
                chunk = cb;
                xtra = nx;
                nblk1 = slots;
            }
        }
    }
    const dim3 grid(nblk1 + (pods2 ? (xtra ? nblk1 : cdiv(n_pods2, chunk)) : 0u), gy);
    // the fixed-slot form for digit-aligned waves (profiles/r04j_fix_ab.txt)
    constexpr int fix_ok = 1;
    const PpJob2 j2 = {pods2, reinterpret_cast<u64 *>(keys2), n_pods2, nblk1};
    if (pods2 && (gy > 1 || results || resc || !keys || !keys2)) return hipErrorInvalidValue;
    if (gy > 1) {
        // several workgroups per chunk: combine keys with atomicMax, then decode
        // (done: an event record after the last of these launches)
        if (!keys || resc) return hipErrorInvalidValue;
        hipError_t e = hipMemsetAsync(keys, 0, sizeof(unsigned long long) * n_pods, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((k_sweep_nunn_pp<kPpWords, false>), grid, dim3(64 * W), chunk * (sizeof(u64) + sizeof(uint2)), s, t.planes,
                           t.gcap, n_groups, t.base, pods, n_pods, chunk, seed32, keys, 1, (ms_result *)nullptr, present,
                           t, 0, (uint32_t)sizeof(ms_pod_rec), (ms_result_compact *)nullptr, PpJob2{}, fix_ok, 0u);
        e = hipGetLastError();
        if (e == hipSuccess && results) e = launch_decode(pods, n_pods, keys, nullptr, present, results, s);
        if (e == hipSuccess && results && commit) e = launch_apply_binds(t, pods, n_pods, results, s);
        if (e == hipSuccess && done) e = hipEventRecord(done, s);
        return e;
    }
    // done: recorded by the dispatch itself (hipExtLaunchKernel's stop event: no
    // separate event packet between this sweep and the next launch on s)
    const uint32_t lds = (chunk + (xtra ? 8u : 0u)) * (sizeof(u64) + sizeof(uint2));
    unsigned long long *kk = (results || resc) ? nullptr : keys;
    const int cm = (results || resc) ? commit : 0;
    // (gy == 1: the workgroup holds every group; the 8-word form stays unpacked: its
    // packed instantiation needs 117 VGPRs, half the waves per SIMD it sizes for)
    const bool tp = KW == (uint32_t)kPpWords && tail_pods(n_groups, W) != 0u;
#define MS_PP_LAUNCH(KWV, TPV)                                                                                     \
    hipExtLaunchKernelGGL((k_sweep_nunn_pp<KWV, TPV>), grid, dim3(64 * W), lds, s, nullptr, done, 0, t.planes, t.gcap, \
                          n_groups, t.base, pods, n_pods, chunk, seed32, kk, 0, results, present, t, cm, pstride, resc, j2, \
                          fix_ok, xtra)
    if (KW == (uint32_t)kPpWordsSmall) {
        MS_PP_LAUNCH(kPpWordsSmall, false);
    } else {
        if (tp) MS_PP_LAUNCH(kPpWords, true);
        else MS_PP_LAUNCH(kPpWords, false);
    }
#undef MS_PP_LAUNCH
    return hipGetLastError();
}
}  // namespace

hipError_t launch_sweep_pp(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                           uint32_t seed32, unsigned long long *keys, ms_result *results, uint32_t present,
                           int num_cus, hipStream_t s, int commit, hipEvent_t done) {
    return sweep_pp_impl(t, n_rows, pods, n_pods, seed32, keys, results, present, num_cus, s, commit, done,
                         (uint32_t)sizeof(ms_pod_rec), nullptr);
}

hipError_t launch_sweep_pp2(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods1, uint32_t n1,
                            unsigned long long *keys1, const ms_pod_rec *pods2, uint32_t n2, unsigned long long *keys2,
                            uint32_t seed32, uint32_t present, int num_cus, hipStream_t s, hipEvent_t done) {
    if (n_rows > kPpMaxFusedRows) return hipErrorInvalidValue;
    return sweep_pp_impl(t, n_rows, pods1, n1, seed32, keys1, nullptr, present, num_cus, s, 0, done,
                         (uint32_t)sizeof(ms_pod_rec), nullptr, pods2, n2, keys2);
}

hipError_t launch_sweep_pp_compact(const NodeTable &t, uint32_t n_rows, const ms_pod_compact *pods, uint32_t n_pods,
                                   uint32_t seed32, ms_result_compact *results, uint32_t present, int num_cus,
                                   hipStream_t s) {
    static_assert(sizeof(ms_pod_compact) == 8 && sizeof(ms_result_compact) == 8, "compact records");
    if (n_rows > kPpMaxFusedRows || !results) return hipErrorInvalidValue;
    return sweep_pp_impl(t, n_rows, reinterpret_cast<const ms_pod_rec *>(pods), n_pods, seed32, nullptr, nullptr,
                         present, num_cus, s, 1, nullptr, (uint32_t)sizeof(ms_pod_compact), results);
}

}  // namespace msgpu
