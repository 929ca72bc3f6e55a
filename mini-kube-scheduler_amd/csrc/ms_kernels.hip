// ms_kernels.hip — gfx950 kernels for minisched's scheduling cycle.
//
// Reference path (all in /root/reference/minisched/minisched.go):
//   RunFilterPlugins :115-151 -> NodeUnschedulable.Filter (k8s@v1.22.0, restated)
//   RunScorePlugins  :164-199 -> NodeNumber.Score (plugins/score/nodenumber/nodenumber.go:73-95)
//   unweighted sum   :187-196
//   selectHost       :304-325 (tie-break replaced by the packed key, see minisched_gpu.h)
//
// The per-(pod,node) work is integer-only and tiny, so the kernels keep a
// tile of node columns in registers and stream pods through it: one node per
// lane-slot, pods wave-uniform (scalar loads), a 64-bit wave max per pod and
// one coalesced atomicMax wave-instruction per 64 pods.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "ms_device.h"

namespace msgpu {

namespace {

__device__ __forceinline__ u64 wave_max_u64(u64 v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = umax64(v, __shfl_xor(v, off, 64));
    return v;
}

__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v |= __shfl_xor(v, off, 64);
    return v;
}

// ----------------------------------------------------------------------------
// K3: NodeUnschedulable + NodeResourcesFit filters, NodeNumber + LeastAllocated
// scores (upstream v1.22 semantics restated in oracle/ms_oracle.c).
// ----------------------------------------------------------------------------
// LeastAllocated (k8s@v1.22.0 least_allocated.go leastRequestedScore) per
// resource: capacity 0 or requested > capacity -> 0, else
// floor((capacity - requested) * 100 / capacity), requested = NonZeroRequested
// + the pod's non-zero request n. With av = capacity - NonZeroRequested and
// d = av - n, the f32 estimate x = (f32(av) - f32(n)) * f32(100/capacity) is
// within 4e-5 of q = 100 d / capacity whenever 0 <= d (then n <= av <= capacity:
// every operand's rounding is relative to at most capacity). So with
// m = round(x), floor(q) is m or m - 1, and ONE exact int64 comparison
// 100 d >= m * capacity decides it. 100 d = a100 - n100 with a100 = 100 av per
// node and n100 = 100 min(n, 2^55) per pod; valid (d >= 0) <=> 100 d >= 0.
// Rows with capacity >= 2^53 (beyond any real allocatable) hold av in the a100
// field and take plain int64 arithmetic (kHuge, chosen per wave).
constexpr int64_t kHugeCap = 1ll << 53;

struct FullRow {
    int64_t fr_cpu, fr_mem;      // Allocatable - Requested          (NodeResourcesFit)
    int64_t a100_cpu, a100_mem;  // 100 (Allocatable - NonZeroRequested); av itself when huge
    int64_t cap_cpu, cap_mem;    // Allocatable
    float avf_cpu, avf_mem;      // f32(Allocatable - NonZeroRequested)
    float r_cpu, r_mem;          // f32(100 / Allocatable), 0 when Allocatable == 0
    int32_t room;                // AllowedPodNumber - len(Pods)
    uint32_t fd;                 // flags | digit << 8
};

__device__ __forceinline__ float r100(int64_t cap) { return cap > 0 ? 100.0f / (float)cap : 0.0f; }

__device__ __forceinline__ FullRow make_row(int64_t alloc_cpu, int64_t alloc_mem, int64_t req_cpu, int64_t req_mem,
                                            int64_t nz_cpu, int64_t nz_mem, int32_t room, uint32_t fd) {
    FullRow x;
    x.cap_cpu = alloc_cpu;
    x.cap_mem = alloc_mem;
    x.fr_cpu = alloc_cpu - req_cpu;
    x.fr_mem = alloc_mem - req_mem;
    const int64_t av_cpu = alloc_cpu - nz_cpu, av_mem = alloc_mem - nz_mem;
    x.a100_cpu = alloc_cpu >= kHugeCap ? av_cpu : av_cpu * 100;
    x.a100_mem = alloc_mem >= kHugeCap ? av_mem : av_mem * 100;
    x.avf_cpu = (float)av_cpu;
    x.avf_mem = (float)av_mem;
    x.r_cpu = r100(alloc_cpu);
    x.r_mem = r100(alloc_mem);
    x.room = room;
    x.fd = fd;
    return x;
}

__device__ __forceinline__ FullRow load_row(const NodeTable &t, uint32_t r, uint32_t n_rows) {
    if (r >= n_rows) return make_row(0, 0, 0, 0, 0, 0, 0, kNodeAbsent | (0xFFu << 8));
    return make_row(t.alloc_cpu[r], t.alloc_mem[r], t.req_cpu[r], t.req_mem[r], t.nz_cpu[r], t.nz_mem[r],
                    t.allowed_pods[r] - t.pod_count[r], (uint32_t)t.flags[r] | ((uint32_t)t.digit[r] << 8));
}

template <bool kHuge = true>
__device__ __forceinline__ int64_t least_requested(int64_t a100, float avf, int64_t cap, float r, int64_t n,
                                                   int64_t n100, float nf) {
    if (kHuge && cap >= kHugeCap) {  // a100 holds av
        const int64_t d = a100 - n;
        return (a100 < n) ? 0 : (int64_t)((uint64_t)d * 100u) / cap;
    }
    const uint32_t m = (uint32_t)__builtin_fmaf(avf - nf, r, 0.5f);  // round(x); x < 0 -> 0
    const int64_t d100 = a100 - n100;
    const uint32_t lo = (uint32_t)cap, hi = (uint32_t)((uint64_t)cap >> 32);
    const uint64_t mc = (uint64_t)m * lo + ((uint64_t)(m * hi) << 32);  // m * capacity (< 2^60)
    const uint32_t q = m - (d100 < (int64_t)mc ? 1u : 0u);
    return d100 >= 0 ? (int64_t)q : 0;
}

struct PodFull {
    int64_t rc, rm, nc, nm;   // requests (Fit) and non-zero requests (LeastAllocated)
    int64_t n100c, n100m;     // 100 min(nonzero, 2^55)
    float nfc, nfm;           // f32(nonzero)
    int dig;
    bool tol;
    bool zero_req;
    uint32_t A;
};

__device__ __forceinline__ PodFull load_pod(const ms_pod_rec &pr, uint32_t seed32) {
    PodFull q;
    q.rc = pr.req_milli_cpu;
    q.rm = pr.req_memory;
    q.nc = pr.nonzero_milli_cpu;
    q.nm = pr.nonzero_memory;
    q.n100c = min(q.nc, 1ll << 55) * 100;
    q.n100m = min(q.nm, 1ll << 55) * 100;
    q.nfc = (float)q.nc;
    q.nfm = (float)q.nm;
    q.dig = pr.name_digit;
    q.tol = pr.tolerates_unschedulable != 0;
    q.zero_req = (q.rc == 0 && q.rm == 0);
    q.A = tb_pod(seed32, pr.ordinal);
    return q;
}

__device__ __forceinline__ int64_t readlane_i64(int64_t v, uint32_t l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), (int)l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Sweeps hold up to 64 pods lane-resident (one parallel load, no per-pod
// memory round trip) and broadcast pod i with readlanes.
struct PodLanes {
    PodFull q;
};

__device__ __forceinline__ PodLanes stage_pods(const ms_pod_rec *__restrict__ pods, uint32_t g, uint32_t cnt,
                                               uint32_t lane, uint32_t seed32) {
    PodLanes m;
    ms_pod_rec z = {};
    m.q = load_pod(lane < cnt ? pods[g + lane] : z, seed32);
    return m;
}

__device__ __forceinline__ PodFull pod_of_lane(const PodLanes &m, uint32_t i) {
    PodFull q;
    q.rc = readlane_i64(m.q.rc, i);
    q.rm = readlane_i64(m.q.rm, i);
    q.nc = readlane_i64(m.q.nc, i);
    q.nm = readlane_i64(m.q.nm, i);
    q.n100c = readlane_i64(m.q.n100c, i);
    q.n100m = readlane_i64(m.q.n100m, i);
    q.nfc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m.q.nfc), (int)i));
    q.nfm = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m.q.nfm), (int)i));
    q.A = (uint32_t)__builtin_amdgcn_readlane((int)m.q.A, (int)i);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane(
        (int)(((uint32_t)m.q.dig & 0xFFu) | (m.q.tol ? 0x100u : 0u) | (m.q.zero_req ? 0x200u : 0u)), (int)i);
    q.dig = (int)(int8_t)(b & 0xFFu);
    q.tol = (b & 0x100u) != 0;
    q.zero_req = (b & 0x200u) != 0;
    return q;
}

// Evaluates one (pod,node) pair: returns the packed key (0 when filtered out)
// and sets the first-failing filter plugin (minisched.go:130-137 breaks on
// the first failure, so a node rejected by NU is never charged to NRF).
template <bool kHuge = true>
__device__ __forceinline__ u64 eval_full(const FullRow &x, uint32_t ord, const PodFull &q,
                                         uint32_t &nu, uint32_t &nrf) {
    const uint32_t fl = x.fd & 0xFFu;
    const bool absent = (fl & kNodeAbsent) != 0;
    const bool f_nu = !absent && (fl & kNodeUnschedulable) != 0 && !q.tol;
    bool bad = x.room < 1;  // len(Pods)+1 > AllowedPodNumber
    if (!q.zero_req) bad = bad || (q.rc > x.fr_cpu) || (q.rm > x.fr_mem);
    const bool f_nrf = !absent && !f_nu && bad;
    nu = f_nu ? 1u : 0u;
    nrf = f_nrf ? 1u : 0u;
    const int64_t s_cpu = least_requested<kHuge>(x.a100_cpu, x.avf_cpu, x.cap_cpu, x.r_cpu, q.nc, q.n100c, q.nfc);
    const int64_t s_mem = least_requested<kHuge>(x.a100_mem, x.avf_mem, x.cap_mem, x.r_mem, q.nm, q.n100m, q.nfm);
    const uint32_t nn = ((int)(x.fd >> 8) == q.dig) ? 10u : 0u;
    const uint32_t la = (uint32_t)((s_cpu + s_mem) / 2);
    const u64 key = make_key(nn + la, tb_hash(q.A, ord), ord);
    return (absent || f_nu || bad) ? 0ull : key;
}

// Whether any of the wave's rows needs the int64 LeastAllocated path.
__device__ __forceinline__ bool rows_huge(const FullRow *x) {
    bool h = false;
#pragma unroll
    for (int s = 0; s < kFullSlots; ++s) h = h || x[s].cap_cpu >= kHugeCap || x[s].cap_mem >= kHugeCap;
    return __ballot(h) != 0;
}

// ---- binary64 LeastAllocated (the config-E sweep's fast form) --------------
// floor(100 (av - n) / cap) as ONE fma + a saturating conversion per resource:
//   r = RN(100 / cap), a = RN(RN(av * r) + 2^-43), x = RN(-n * r + a) (fma),
//   score = x <= 0 ? 0 : trunc(x)                               (v_cvt_u32_f64)
// |x - (X + 2^-43)| <= 402 u (u = 2^-53) for X = 100 (av - n) / cap <= 100, so
// trunc(x) = floor(X) whenever 2^-43 > 402 u and 2^-43 + 402 u < 1 / cap, i.e.
// for 0 < cap < 2^41 (cap <= 0: r = 0, score 0 as leastRequestedScore gives);
// negative X (requested > capacity) lands below 0 and saturates to 0.
// Exact by the bound and by tests/c/la_f64_exact.c (boundary cases around every
// k * cap / 100; the window of working epsilons is 2^-46 .. 2^-42). Needs
// NonZeroRequested >= 0 (av <= cap) and 0 <= pod non-zero request < 2^53; a
// wave whose rows or pods fall outside takes the general path (eval_full).
constexpr int64_t kFastCap = 1ll << 41;
constexpr int64_t kFastReq = 1ll << 53;
constexpr double kLaEps = 0x1p-43;

typedef DRow FastRow;  // (ms_internal.h)

__device__ __forceinline__ double la_r(int64_t cap) { return cap > 0 ? __ddiv_rn(100.0, (double)cap) : 0.0; }

__device__ __forceinline__ double la_a(int64_t cap, int64_t nz, double r) {
    const int64_t av = (int64_t)((uint64_t)cap - (uint64_t)nz);  // (wraps only where r == 0 or av < 0 anyway)
    return __dadd_rn(__dmul_rn((double)av, r), kLaEps);
}

__device__ __forceinline__ DRow make_drow(int64_t ac, int64_t am, int64_t rqc, int64_t rqm, int64_t zc, int64_t zm,
                                          int32_t room, uint32_t fd) {
    DRow x;
    x.fr_cpu = (int64_t)((uint64_t)ac - (uint64_t)rqc);
    x.fr_mem = (int64_t)((uint64_t)am - (uint64_t)rqm);
    x.r_cpu = la_r(ac);
    x.r_mem = la_r(am);
    x.a_cpu = la_a(ac, zc, x.r_cpu);
    x.a_mem = la_a(am, zm, x.r_mem);
    x.room = room;
    x.fd = fd;
    x.digit = fd >> 8;
    const bool absent = (fd & kNodeAbsent) != 0;
    const bool unsched = !absent && (fd & kNodeUnschedulable);
    x.rbits = (absent ? kRbAbsent : 0u) | (unsched ? kRbUnsched : 0u) | (absent || unsched ? kRbBlocked : 0u) |
              (!absent && room < 1 ? kRbNoRoom : 0u) |
              ((ac < kFastCap && am < kFastCap && zc >= 0 && zm >= 0) ? 0u : kRbSlow);
    return x;
}

__device__ __forceinline__ DRow absent_drow() {
    DRow x;
    x.fr_cpu = x.fr_mem = 0;
    x.r_cpu = x.r_mem = x.a_cpu = x.a_mem = 0.0;
    x.room = 0;
    x.fd = kNodeAbsent | (0xFFu << 8);
    x.digit = 0xFFu;
    x.rbits = kRbAbsent | kRbBlocked;
    return x;
}

__device__ __forceinline__ FastRow load_fast_row(const NodeTable &t, uint32_t r, uint32_t n_rows) {
    if (r >= n_rows) return absent_drow();
    return make_drow(t.alloc_cpu[r], t.alloc_mem[r], t.req_cpu[r], t.req_mem[r], t.nz_cpu[r], t.nz_mem[r],
                     t.allowed_pods[r] - t.pod_count[r], (uint32_t)t.flags[r] | ((uint32_t)t.digit[r] << 8));
}

__global__ void k_build_drows(NodeTable t, uint32_t n_rows, uint32_t n_total) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n_total) t.drow[r] = load_fast_row(t, r, n_rows);
}

struct PodFast {
    int64_t rc, rm;    // requests (Fit)
    double nnc, nnm;   // -(double) non-zero requests (LeastAllocated)
    uint32_t A;
    uint32_t bits;     // digit (9 bits, sign-extended) | kPfTol | kPfZero | kPfOk
    uint32_t rej;      // DRow::rbits that reject the pod statically: absent, no room, unschedulable unless tolerated
    uint32_t cand;     // DRow::rbits that exclude a rejection from NodeResourcesFit: absent, NU-rejected
};
constexpr uint32_t kPfTol = 0x200u, kPfZero = 0x400u, kPfOk = 0x800u;

__device__ __forceinline__ PodFast load_pod_fast(const ms_pod_rec &pr, uint32_t seed32) {
    PodFast q;
    q.rc = pr.req_milli_cpu;
    q.rm = pr.req_memory;
    q.nnc = -(double)pr.nonzero_milli_cpu;
    q.nnm = -(double)pr.nonzero_memory;
    q.A = tb_pod(seed32, pr.ordinal);
    const bool ok = pr.nonzero_milli_cpu >= 0 && pr.nonzero_milli_cpu < kFastReq && pr.nonzero_memory >= 0 &&
                    pr.nonzero_memory < kFastReq;
    // the digit as 9 bits: a negative (non-digit) name never equals a node's digit byte
    q.bits = ((uint32_t)(int32_t)pr.name_digit & 0x1FFu) | (pr.tolerates_unschedulable ? kPfTol : 0u) |
             ((pr.req_milli_cpu == 0 && pr.req_memory == 0) ? kPfZero : 0u) | (ok ? kPfOk : 0u);
    q.cand = kRbAbsent | (pr.tolerates_unschedulable ? 0u : kRbUnsched);
    q.rej = q.cand | kRbNoRoom;
    return q;
}

__device__ __forceinline__ double readlane_f64(double v, uint32_t l) {
    return __longlong_as_double(readlane_i64(__double_as_longlong(v), l));
}

__device__ __forceinline__ PodFast pod_fast_of_lane(const PodFast &m, uint32_t i) {
    PodFast q;
    q.rc = readlane_i64(m.rc, i);
    q.rm = readlane_i64(m.rm, i);
    q.nnc = readlane_f64(m.nnc, i);
    q.nnm = readlane_f64(m.nnm, i);
    q.A = (uint32_t)__builtin_amdgcn_readlane((int)m.A, (int)i);
    q.bits = (uint32_t)__builtin_amdgcn_readlane((int)m.bits, (int)i);
    q.rej = (uint32_t)__builtin_amdgcn_readlane((int)m.rej, (int)i);
    q.cand = (uint32_t)__builtin_amdgcn_readlane((int)m.cand, (int)i);
    return q;
}

__device__ __forceinline__ uint32_t cvt_u32_sat(double x) {  // negatives -> 0
    uint32_t q;
    asm("v_cvt_u32_f64 %0, %1" : "=v"(q) : "v"(x));
    return q;
}

// eval_full's key and first-failure flags through the binary64 LeastAllocated.
__device__ __forceinline__ u64 eval_fast(const FastRow &x, uint32_t ord, const PodFast &q, uint32_t &nu,
                                         uint32_t &nrf) {
    const uint32_t rb = x.rbits;
    const bool absent = (rb & kRbAbsent) != 0;
    const bool f_nu = (rb & kRbUnsched) != 0 && !(q.bits & kPfTol);
    bool bad = (rb & kRbNoRoom) != 0;
    if (!(q.bits & kPfZero)) bad = bad || (q.rc > x.fr_cpu) || (q.rm > x.fr_mem);
    const bool f_nrf = !absent && !f_nu && bad;
    nu = f_nu ? 1u : 0u;
    nrf = f_nrf ? 1u : 0u;
    const uint32_t s_cpu = cvt_u32_sat(__builtin_fma(q.nnc, x.r_cpu, x.a_cpu));
    const uint32_t s_mem = cvt_u32_sat(__builtin_fma(q.nnm, x.r_mem, x.a_mem));
    const uint32_t nn = (x.digit == (q.bits & 0x1FFu)) ? 10u : 0u;
    const u64 key = make_key(nn + ((s_cpu + s_mem) >> 1), tb_hash(q.A, ord), ord);
    return (absent || f_nu || bad) ? 0ull : key;
}

// Batched resource-aware sweep: atomicMax into keys[P] / atomicOr into flags[P].
__global__ __launch_bounds__(kFullThreads) void k_sweep_full(NodeTable t, uint32_t n_rows,
                                                             const ms_pod_rec *__restrict__ pods, uint32_t n_pods,
                                                             uint32_t chunk, uint32_t seed32, u64 *__restrict__ keys,
                                                             uint32_t *__restrict__ pflags) {
    const uint32_t lane = lane_id();
    const uint32_t row0 = blockIdx.x * kFullTile + threadIdx.x * kFullSlots;
    FullRow x[kFullSlots];
#pragma unroll
    for (int s = 0; s < kFullSlots; ++s) x[s] = load_row(t, row0 + s, n_rows);
    const uint32_t ord0 = t.base + row0;
    const bool huge = rows_huge(x);
    const uint32_t pbeg = blockIdx.y * chunk;
    const uint32_t pend = min(n_pods, pbeg + chunk);
    for (uint32_t g = pbeg; g < pend; g += 64) {
        const uint32_t cnt = min(64u, pend - g);
        const PodLanes m = stage_pods(pods, g, cnt, lane, seed32);
        u64 mine = 0;
        uint32_t myflag = 0;
        for (uint32_t i = 0; i < cnt; ++i) {
            const PodFull q = pod_of_lane(m, i);
            u64 best = 0;
            uint32_t nu_any = 0, nrf_any = 0;
#pragma unroll
            for (int s = 0; s < kFullSlots; ++s) {
                uint32_t nu, nrf;
                best = umax64(best, huge ? eval_full<true>(x[s], ord0 + s, q, nu, nrf)
                                         : eval_full<false>(x[s], ord0 + s, q, nu, nrf));
                nu_any |= nu;
                nrf_any |= nrf;
            }
            best = wave_max_u64(best);
            const uint32_t f = (__ballot(nu_any != 0) ? 1u : 0u) | (__ballot(nrf_any != 0) ? 0x100u : 0u);
            if (lane == i) {
                mine = best;
                myflag = f;
            }
        }
        if (lane < cnt) {
            if (mine) atomicMax(&keys[g + lane], mine);
            if (myflag) atomicOr(&pflags[g + lane], myflag);
        }
    }
}

// 64-bit unsigned wave max from two DPP u32 reductions; wave-uniform result.
__device__ __forceinline__ u64 wave_max_u64_dpp(u64 v) {
    const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    const uint32_t hmax = wave_max_u32_dpp(hi);
    const uint32_t lmax = wave_max_u32_dpp(hi == hmax ? lo : 0u);
    return ((u64)hmax << 32) | lmax;
}

// Max over each quad of lanes (4i .. 4i+3), every lane of the quad gets it.
// wave_max_u64_dpp where one lane usually holds the high-word maximum (the
// sweep's packed keys): that lane supplies the low word by one readlane
// instead of a second reduction.
__device__ __forceinline__ u64 wave_max_u64_unique(u64 v) {
    const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    const uint32_t hmax = wave_max_u32_dpp(hi);
    const u64 tie = __ballot(hi == hmax);
    if ((tie & (tie - 1ull)) == 0ull)
        return ((u64)hmax << 32) | (uint32_t)__builtin_amdgcn_readlane((int)lo, (int)__builtin_ctzll(tie));
    return ((u64)hmax << 32) | wave_max_u32_dpp(hi == hmax ? lo : 0u);
}

template <int CTRL>
__device__ __forceinline__ u64 dpp_u64(u64 v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, false);
    return ((u64)hi << 32) | lo;
}

__device__ __forceinline__ u64 quad_max_u64(u64 v) {
    v = umax64(v, dpp_u64<0xB1>(v));     // quad_perm [1,0,3,2]
    return umax64(v, dpp_u64<0x4E>(v));  // quad_perm [2,3,0,1]
}

__device__ __forceinline__ void cswap_desc(u64 &a, u64 &b) {
    // one 64-bit compare, four 32-bit selects (selecting whole u64s lets the
    // compiler re-derive min with a second compare)
    const bool c = a > b;
    const uint32_t al = (uint32_t)a, ah = (uint32_t)(a >> 32), bl = (uint32_t)b, bh = (uint32_t)(b >> 32);
    const uint32_t hl = c ? al : bl, hh = c ? ah : bh, ll = c ? bl : al, lh = c ? bh : ah;
    a = ((u64)hh << 32) | hl;
    b = ((u64)lh << 32) | ll;
}

// ----------------------------------------------------------------------------
// Exact sequential engine, speculative half (config E).
// For each pod of a batch and each 256-row wave tile: the tile's top-K packed
// keys against the batch-start state (0-terminated when the tile has fewer
// than K feasible rows) and the tile's filter flags.
// ----------------------------------------------------------------------------
// Tile-list stores and loads coherent across the XCDs within one launch
// (agent-scope relaxed atomics: the store writes through, the load bypasses a
// possibly stale L2 line). The in-step merge (k_seq_step, SeqMergeIO) reads the
// lists of sweep workgroups that ran on other XCDs in the same launch.
// In-step merge synchronisation (round 5). MS_MERGE_TAGS 1 (default): the
// sweep stamps every list of the step with a 2-bit tag (bits 61-62 of each key,
// bits 16-17 of the flags word; 1..3, cycling over the steps; a buffer set is
// rewritten every second step and zeroed at the start of each run) and a merge
// worker polls the lists themselves until every one it reads carries the tag:
// no counter, no barrier, and the lists arrive with the check. MS_MERGE_TAGS 0:
// the sweep workgroups count themselves done on one counter after their stores
// landed and the workers poll it, then load the lists (A/B). Measured and
// dropped: system-scope counter, spin without s_sleep, fine-grained counter
// memory (all 40.5-40.6 ms), per-workgroup slots instead of the counter (41.7),
// release/acquire fences with plain list stores (85 ms: the fences write back
// and invalidate whole L2s) (profiles/r05f_e_sync_ab.txt, r05j_e_slots_ab.txt).
#ifndef MS_MERGE_TAGS
#define MS_MERGE_TAGS 1
#endif
constexpr int kListTagShift = 61;  // (config E scores stay below 512: bits 61-62 of a key are 0)
constexpr u64 kListTagMask = 3ull << kListTagShift;
__device__ __forceinline__ u64 untag_key(u64 k) { return k & ~kListTagMask; }
__device__ __forceinline__ uint32_t untag_flags(uint32_t f) { return f & 0xFFFFu; }
// Diagnostic timeline fields per workgroup (MS_VSTAMPS / MS_TIMELINE_ONLY builds,
// s_memrealtime): 0 start, 1 swept (counted), 2 worker's wait done, 3 worker's
// merges done, 4 validator done (workgroup 0), 5 first tile staged in LDS,
// 6 wave 0's sweep tasks done, 7 every wave's tasks done (barrier)
enum { kTlBegin = 0, kTlSwept, kTlWaited, kTlMerged, kTlValidated, kTlStaged, kTlWave0, kTlTasks };
typedef __attribute__((address_space(1))) u64 gu64_t;
typedef __attribute__((address_space(1))) uint32_t gu32_t;
__device__ __forceinline__ void st_coh(u64 *p, u64 v) {
    __hip_atomic_store(((gu64_t *)(p)), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coh(uint32_t *p, uint32_t v) {
    __hip_atomic_store(((gu32_t *)(p)), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 ld_coh(const u64 *p) {
    return __hip_atomic_load(((const gu64_t *)(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_coh(const uint32_t *p) {
    return __hip_atomic_load(((const gu32_t *)(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kTopK = 4;
constexpr int kTopExt = 8;  // ranks the merge lists for the validator's slow pods (4 beyond the top-4)
static_assert(kFullSlots == kTopK, "one key per row slot feeds the per-lane sort");

#ifndef MS_MERGE_WMAX
#define MS_MERGE_WMAX wave_max_u64_dpp
#endif
#ifndef MS_SWEEP_WMAX
#define MS_SWEEP_WMAX wave_max_u64_unique
#endif
// Row forms of the sweep (F): 0 general int64/f32 LeastAllocated, 1 rows with
// capacities >= 2^53, 2 the binary64 fast form.
template <int F, typename Pod>
__device__ __forceinline__ u64 sweep_eval(const FullRow &x, uint32_t ord, const Pod &q, uint32_t &nu, uint32_t &nrf) {
    return eval_full<F == 1>(x, ord, q, nu, nrf);
}
template <int F, typename Pod>
__device__ __forceinline__ u64 sweep_eval(const FastRow &x, uint32_t ord, const Pod &q, uint32_t &nu, uint32_t &nrf) {
    return eval_fast(x, ord, q, nu, nrf);
}

__device__ __forceinline__ PodFull lane_pod(const PodLanes &m, uint32_t i) { return pod_of_lane(m, i); }
__device__ __forceinline__ PodFast lane_pod(const PodFast &m, uint32_t i) { return pod_fast_of_lane(m, i); }

// NP pods at a time: their evaluations, sorts and wave reductions are
// independent, so the DPP chains of one hide the latency of the other's (3
// waves per SIMD leave little else to hide it). F: 0 general, 1 huge rows, 2
// binary64 fast form (Row FastRow, Lanes PodFast).
template <int F, int NP, typename Row, typename Lanes>
__device__ __forceinline__ void sweep_topk_group(const Row *x, uint32_t ord0, const Lanes &m, uint32_t pbeg,
                                                 uint32_t i, uint32_t lane, uint32_t tile, uint32_t n_tiles,
                                                 u64 *__restrict__ tile_keys, uint32_t *__restrict__ tile_flags,
                                                 uint32_t tag) {
    u64 k[NP][kFullSlots], out[NP];
    uint32_t nu_any[NP], nrf_any[NP];
#pragma unroll
    for (int n = 0; n < NP; ++n) {
        const auto q = lane_pod(m, i + n);
        nu_any[n] = nrf_any[n] = 0;
#pragma unroll
        for (int s = 0; s < kFullSlots; ++s) {
            uint32_t nu, nrf;
            k[n][s] = sweep_eval<F>(x[s], ord0 + s, q, nu, nrf);
            nu_any[n] |= nu;
            nrf_any[n] |= nrf;
        }
        // descending sort of the lane's 4 keys (keys are unique unless 0)
        cswap_desc(k[n][0], k[n][1]);
        cswap_desc(k[n][2], k[n][3]);
        cswap_desc(k[n][0], k[n][2]);
        cswap_desc(k[n][1], k[n][3]);
        cswap_desc(k[n][1], k[n][2]);
        out[n] = 0;
    }
#pragma unroll
    for (int j = 0; j < kTopK; ++j) {
#pragma unroll
        for (int n = 0; n < NP; ++n) {
            const u64 mx = MS_SWEEP_WMAX(k[n][0]);
            if (lane == (uint32_t)j) out[n] = mx;
            if (mx != 0 && k[n][0] == mx) {  // the owning lane pops its head
                k[n][0] = k[n][1];
                k[n][1] = k[n][2];
                k[n][2] = k[n][3];
                k[n][3] = 0;
            }
        }
    }
#pragma unroll
    for (int n = 0; n < NP; ++n) {
        const uint32_t f = (__ballot(nu_any[n] != 0) ? 1u : 0u) | (__ballot(nrf_any[n] != 0) ? 0x100u : 0u);
        const size_t cell = (size_t)(pbeg + i + n) * n_tiles + tile;
        if (tag) {  // (launch-uniform) an in-step merge reads these lists in this launch
            if (lane < (uint32_t)kTopK) st_coh(tile_keys + cell * kTopK + lane, out[n] | (u64)tag << kListTagShift);
            if (lane == 0) st_coh(tile_flags + cell, f | tag << 16);
        } else {
            if (lane < (uint32_t)kTopK) tile_keys[cell * kTopK + lane] = out[n];
            if (lane == 0) tile_flags[cell] = f;
        }
    }
}

template <int F, typename Row, typename Lanes, int NPMAX = 2>
__device__ __forceinline__ void sweep_topk_pods(const Row *x, uint32_t ord0, const Lanes &m, uint32_t pbeg,
                                                uint32_t cnt, uint32_t lane, uint32_t tile, uint32_t n_tiles,
                                                u64 *__restrict__ tile_keys, uint32_t *__restrict__ tile_flags,
                                                uint32_t tag) {
    uint32_t i = 0;
    if (NPMAX >= 2)
        for (; i + 2 <= cnt; i += 2)
            sweep_topk_group<F, 2>(x, ord0, m, pbeg, i, lane, tile, n_tiles, tile_keys, tile_flags, tag);
    for (; i < cnt; ++i)
        sweep_topk_group<F, 1>(x, ord0, m, pbeg, i, lane, tile, n_tiles, tile_keys, tile_flags, tag);
}

struct SweepArgs {
    NodeTable t;
    uint32_t n_rows;
    const ms_pod_rec *pods;
    uint32_t n_pods;
    uint32_t chunk;  // pods per task, <= 64
    uint32_t seed32;
    u64 *tile_keys;
    uint32_t *tile_flags;
    uint32_t n_tiles;
    uint32_t fast;  // binary64 LeastAllocated where exact (default 1)
    uint32_t coh;   // 1..3: an in-step merge reads the lists in this launch: stores write through (st_coh),
                    // tagged with this value (MS_MERGE_TAGS); 0: plain stores
};

// One wave, lane = row: tile `tile`'s top-4 lists and filter flags for pods
// [pbeg, pbeg + cnt), cnt <= 64. The binary64 fast form unless a row or pod of
// the task is outside its exact range (MINISCHED_SEQ_FAST=0: a.fast == 0).
// Row `slot` (lane * kFullSlots + s) of tile `tile`, or an absent row (~0u) past
// the tile's height (t.tile_rows < kFullWaveTile: the next tile's rows).
__device__ __forceinline__ uint32_t tile_slot_row(const NodeTable &t, uint32_t tile, uint32_t slot) {
    const uint32_t tr = tile_rows_of(t);
    return slot < tr ? tile * tr + slot : ~0u;
}

__device__ __forceinline__ void sweep_rows_task(const SweepArgs &a, uint32_t tile, uint32_t pbeg, uint32_t cnt,
                                                uint32_t lane) {
    const uint32_t row0 = tile * tile_rows_of(a.t) + lane * kFullSlots;
    const uint32_t ord0 = a.t.base + row0;
    if (a.fast) {
        FastRow x[kFullSlots];
        bool ok = true;
#pragma unroll
        for (int s = 0; s < kFullSlots; ++s) {
            x[s] = load_fast_row(a.t, tile_slot_row(a.t, tile, lane * kFullSlots + s), a.n_rows);
            ok = ok && !(x[s].rbits & kRbSlow);
        }
        ms_pod_rec z = {};
        const PodFast m = load_pod_fast(lane < cnt ? a.pods[pbeg + lane] : z, a.seed32);
        ok = ok && (lane >= cnt || (m.bits & kPfOk));
        if (__ballot(!ok) == 0) {
            sweep_topk_pods<2>(x, ord0, m, pbeg, cnt, lane, tile, a.n_tiles, a.tile_keys, a.tile_flags, a.coh);
            return;
        }
    }
    FullRow x[kFullSlots];
#pragma unroll
    for (int s = 0; s < kFullSlots; ++s) x[s] = load_row(a.t, tile_slot_row(a.t, tile, lane * kFullSlots + s), a.n_rows);
    const PodLanes m = stage_pods(a.pods, pbeg, cnt, lane, a.seed32);
    if (rows_huge(x)) sweep_topk_pods<1>(x, ord0, m, pbeg, cnt, lane, tile, a.n_tiles, a.tile_keys, a.tile_flags, a.coh);
    else sweep_topk_pods<0>(x, ord0, m, pbeg, cnt, lane, tile, a.n_tiles, a.tile_keys, a.tile_flags, a.coh);
}

// The transposed form's fallback (a row or pod outside the binary64 range,
// rare): the general int64 form one pod at a time, lean on registers.
__device__ __forceinline__ void sweep_rows_task_lean(const SweepArgs &a, uint32_t tile, uint32_t pbeg, uint32_t cnt,
                                                     uint32_t lane) {
    const uint32_t row0 = tile * tile_rows_of(a.t) + lane * kFullSlots;
    const uint32_t ord0 = a.t.base + row0;
    FullRow x[kFullSlots];
#pragma unroll
    for (int s = 0; s < kFullSlots; ++s) x[s] = load_row(a.t, tile_slot_row(a.t, tile, lane * kFullSlots + s), a.n_rows);
    const PodLanes m = stage_pods(a.pods, pbeg, cnt, lane, a.seed32);
    if (rows_huge(x))
        sweep_topk_pods<1, FullRow, PodLanes, 1>(x, ord0, m, pbeg, cnt, lane, tile, a.n_tiles, a.tile_keys,
                                                 a.tile_flags, a.coh);
    else
        sweep_topk_pods<0, FullRow, PodLanes, 1>(x, ord0, m, pbeg, cnt, lane, tile, a.n_tiles, a.tile_keys,
                                                 a.tile_flags, a.coh);
}

// ---- transposed sweep: lane = (pod, row part) ------------------------------
// A workgroup stages one tile's 256 derived rows (t.drow, 16 KB) in LDS; each
// wave then takes kTpPods pods of the batch: lane 4p + j evaluates pod p
// against rows j, j+4, .., j+252 (the four lanes of a pod read 4 consecutive
// rows, the 16 pods' lanes the same ones: LDS broadcasts), keeping its own
// sorted top-4 (each 4 rows: a sorting network, then a bitonic merge), and
// the pod's four lanes merge their lists over DPP quad permutations. No
// cross-lane reduction per (pod, row): ~52 VALU per pair in the inner loop,
// where the lane = row form paid a sort plus four wave-wide max extractions
// per (pod, tile) on top of its evaluations.
constexpr uint32_t kTpPods = 16;
#define MS_PRAGMA(x) _Pragma(#x)
#define MS_UNROLL(n) MS_PRAGMA(unroll n)

__device__ __forceinline__ void tile_keys_store(u64 *dst, uint32_t j, const u64 (&k)[4], uint32_t tag) {
    const u64 v = j == 0 ? k[0] : j == 1 ? k[1] : j == 2 ? k[2] : k[3];
    if (tag) st_coh(dst, v | (u64)tag << kListTagShift);
    else *dst = v;
}

__device__ __forceinline__ void sort4_desc(u64 (&x)[4]) {
    cswap_desc(x[0], x[1]);
    cswap_desc(x[2], x[3]);
    cswap_desc(x[0], x[2]);
    cswap_desc(x[1], x[3]);
    cswap_desc(x[1], x[2]);
}

// k <- top 4 of k u s, both sorted descending (bitonic half-cleaner).
__device__ __forceinline__ void merge4_desc(u64 (&k)[4], const u64 (&s)[4]) {
    u64 c0 = umax64(k[0], s[3]), c1 = umax64(k[1], s[2]), c2 = umax64(k[2], s[1]), c3 = umax64(k[3], s[0]);
    cswap_desc(c0, c2);
    cswap_desc(c1, c3);
    cswap_desc(c0, c1);
    cswap_desc(c2, c3);
    k[0] = c0;
    k[1] = c1;
    k[2] = c2;
    k[3] = c3;
}

template <int CTRL>
__device__ __forceinline__ void quad_merge4(u64 (&k)[4], uint32_t &f) {
    u64 o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = dpp_u64<CTRL>(k[j]);
    merge4_desc(k, o);
    f |= (uint32_t)__builtin_amdgcn_mov_dpp((int)f, CTRL, 0xF, 0xF, false);
}

// ---- tile-local keys as binary64 (round 5) ---------------------------------
// Inside one 256-row tile a packed key needs score (11 bits), the 32-bit hash
// and the row's place in the tile (8 bits): 51 bits. Placed in the mantissa of
// a double with the exponent of 2^52 (bits 0x433 << 52), every such key is an
// exactly represented normal number 2^52 + K, ordered like K; an infeasible
// row is +0.0, below every key. A compare-exchange of the per-lane top-4 sort
// network is then v_max_f64 + v_min_f64 (2 VALU) instead of a 64-bit compare
// and four selects (5), and a running max is one v_max_f64 instead of three.
// Issued as inline asm: in IEEE mode the compiler would quiet (canonicalise)
// operands it cannot prove canonical before llvm.maxnum, one more v_max_f64
// per operand; every operand here is +0.0 or a normal number.
#ifndef MS_TP_LDROW  // staged rows read as 16-B vectors (ld_drow; 0: field by field, A/B)
#define MS_TP_LDROW 1
#endif
#ifndef MS_TP_F64KEYS
#define MS_TP_F64KEYS 1
#endif
constexpr uint32_t kTkExpHi = 0x43300000u;  // high word of 2^52

__device__ __forceinline__ double fmax64(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double fmin64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// K = score << 40 | h << 8 | (255 - place), place = the row's index in its tile.
// se = score + (kTkExpHi >> 8): the exponent rides in the score word, so the
// high word is one v_alignbit. reject: the high word is 0 instead, a value
// (+0.0 or a subnormal) below every key; global_key maps any high word below
// the exponent's to "no feasible row".
__device__ __forceinline__ double tile_key(uint32_t se, uint32_t h, uint32_t place, bool reject) {
    const uint32_t hi = reject ? 0u : __builtin_amdgcn_alignbit(se, h, 24);
    const uint32_t lo = (h << 8) | (255u - place);
    return __hiloint2double((int)hi, (int)lo);
}
// The global packed key (make_key) of a tile key of tile `tile` (0 stays 0).
__device__ __forceinline__ u64 global_key(double k, uint32_t tile_ord0) {
    const uint64_t b = (uint64_t)__double_as_longlong(k);
    if ((uint32_t)(b >> 32) < kTkExpHi) return 0ull;
    const uint32_t hi = (uint32_t)(b >> 32), lo = (uint32_t)b;
    const uint32_t score = (hi >> 8) & 0x7FFu, h = (hi << 24) | (lo >> 8), place = 255u - (lo & 0xFFu);
    return make_key(score, h, tile_ord0 + place);
}
__device__ __forceinline__ void cswap_desc(double &a, double &b) {
    const double hi = fmax64(a, b), lo = fmin64(a, b);
    a = hi;
    b = lo;
}
__device__ __forceinline__ void sort4_desc(double (&x)[4]) {
    cswap_desc(x[0], x[1]);
    cswap_desc(x[2], x[3]);
    cswap_desc(x[0], x[2]);
    cswap_desc(x[1], x[3]);
    cswap_desc(x[1], x[2]);
}
__device__ __forceinline__ void merge4_desc(double (&k)[4], const double (&s)[4]) {
    double c0 = fmax64(k[0], s[3]), c1 = fmax64(k[1], s[2]), c2 = fmax64(k[2], s[1]), c3 = fmax64(k[3], s[0]);
    cswap_desc(c0, c2);
    cswap_desc(c1, c3);
    cswap_desc(c0, c1);
    cswap_desc(c2, c3);
    k[0] = c0;
    k[1] = c1;
    k[2] = c2;
    k[3] = c3;
}
template <int CTRL>
__device__ __forceinline__ void quad_merge4(double (&k)[4], uint32_t &f) {
    double o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = __longlong_as_double((long long)dpp_u64<CTRL>((u64)__double_as_longlong(k[j])));
    merge4_desc(k, o);
    f |= (uint32_t)__builtin_amdgcn_mov_dpp((int)f, CTRL, 0xF, 0xF, false);
}

// The fields eval_tp64 reads of a staged row, as three 16-B and one 8-B LDS
// reads (4 + 4 + 4 + 2 LDS cycles per wave; the compiler's own split of the
// middle 32 B into two ds_read2_b64 took 8 + 8, MICROARCH §LDS).
__device__ __forceinline__ DRow ld_drow(const DRow *p) {
    const longlong2 a = reinterpret_cast<const longlong2 *>(p)[0];
    const double2 b = reinterpret_cast<const double2 *>(p)[1], c = reinterpret_cast<const double2 *>(p)[2];
    const uint2 e = reinterpret_cast<const uint2 *>(p)[7];
    DRow x;
    x.fr_cpu = a.x;
    x.fr_mem = a.y;
    x.r_cpu = b.x;
    x.r_mem = b.y;
    x.a_cpu = c.x;
    x.a_mem = c.y;
    x.room = 0;
    x.fd = 0;
    x.digit = e.x;
    x.rbits = e.y;
    return x;
}

// eval_tp with the tile-local binary64 key (place: the row's index in its tile).
__device__ __forceinline__ double eval_tp64(const DRow &x, uint32_t ord, uint32_t place, const PodFast &q) {
    const bool fit_fail = (q.rc > x.fr_cpu) | (q.rm > x.fr_mem);
    const bool reject = ((x.rbits & q.rej) != 0) | (fit_fail & !(q.bits & kPfZero));
    const uint32_t s_cpu = cvt_u32_sat(__builtin_fma(q.nnc, x.r_cpu, x.a_cpu));
    const uint32_t s_mem = cvt_u32_sat(__builtin_fma(q.nnm, x.r_mem, x.a_mem));
    // nn + floor(s / 2) = floor((s + 2 nn) / 2); the exponent word added twice before the halving
    constexpr uint32_t kE2 = kTkExpHi >> 7;
    const uint32_t nn2 = x.digit == (q.bits & 0x1FFu) ? 20u + kE2 : kE2;
    return tile_key((s_cpu + s_mem + nn2) >> 1, tb_hash(q.A, ord), place, reject);
}

// eval_fast for the transposed form, where the pod differs per lane: the
// static filters from the row's precomputed rbits (one AND + compare), Fit's
// two compares; the filter flags come from the tile's rbits (TileBits).
__device__ __forceinline__ u64 eval_tp(const DRow &x, uint32_t ord, const PodFast &q) {
    const bool fit_fail = (q.rc > x.fr_cpu) | (q.rm > x.fr_mem);
    const bool reject = ((x.rbits & q.rej) != 0) | (fit_fail & !(q.bits & kPfZero));
    const uint32_t s_cpu = cvt_u32_sat(__builtin_fma(q.nnc, x.r_cpu, x.a_cpu));
    const uint32_t s_mem = cvt_u32_sat(__builtin_fma(q.nnm, x.r_mem, x.a_mem));
    const uint32_t nn2 = x.digit == (q.bits & 0x1FFu) ? 20u : 0u;  // nn + floor(s / 2) = floor((s + 2 nn) / 2)
    const u64 key = make_key((s_cpu + s_mem + nn2) >> 1, tb_hash(q.A, ord), ord);
    return reject ? 0ull : key;
}

// OR (any) and AND (all) of a staged tile's rbits, wave-uniform.
struct TileBits {
    uint32_t any, all;
};

__device__ __forceinline__ TileBits tile_bits(const DRow *rows, uint32_t lane, uint32_t tr) {
    uint32_t o = 0, a = ~0u;
#pragma unroll
    for (int k = 0; k < (int)kFullWaveTile / 64; ++k) {
        if (lane + 64u * k >= tr) continue;  // (a tile of tr < kFullWaveTile rows)
        const uint32_t r = rows[lane + 64u * k].rbits;
        o |= r;
        a &= r;
    }
    TileBits b = {0u, 0u};
#pragma unroll
    for (uint32_t bit = 1; bit <= kRbBlocked; bit <<= 1) {
        if (__ballot((o & bit) != 0)) b.any |= bit;
        if (!__ballot((a & bit) == 0)) b.all |= bit;
    }
    return b;
}

// false: a row or pod of the task is outside the binary64 form's exact range
// and nothing was written (the caller runs the lane = row form instead).
// Tile flags: NodeUnschedulable if a present unschedulable row exists and the
// pod does not tolerate it; NodeResourcesFit if a row is neither absent nor
// NodeUnschedulable-rejected. For a tile with no feasible row that is exactly
// "a row NodeResourcesFit rejected"; for a tile with a feasible row every
// consumer (merge_pod_lists, the validator) sets NodeResourcesFit anyway.
__device__ __forceinline__ bool sweep_tp_task(const SweepArgs &a, uint32_t tile, uint32_t grp, uint32_t lane,
                                              const DRow *rows, TileBits tb) {
    const uint32_t pbeg = grp * kTpPods;
    if (pbeg >= a.n_pods) return true;  // wave-uniform
    const uint32_t cnt = min(kTpPods, a.n_pods - pbeg);
    const uint32_t pi = lane >> 2, part = lane & 3u;
    ms_pod_rec z = {};
    const PodFast q = load_pod_fast(pi < cnt ? a.pods[pbeg + pi] : z, a.seed32);
    if ((tb.any & kRbSlow) || __ballot(pi < cnt && !(q.bits & kPfOk))) return false;
    // (tr: a multiple of 16, so every part's rows come in whole 4-row blocks; a
    // runtime trip count, not unrolled: unroll 2 gained 0.6 % at a fixed 256 rows,
    // profiles/r05ay_e_unroll_ab.txt, but written out by hand, or left to the
    // compiler's runtime unrolling, it made k_seq_step spill 121 VGPRs)
    const uint32_t tr = tile_rows_of(a.t);
    const uint32_t row0 = tile * tr + part;
    const uint32_t ord0 = a.t.base + row0;
    const DRow *d = rows + part;  // the tile's rows, staged in LDS
#if MS_TP_F64KEYS
    double k[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 1
    for (uint32_t i = 0; i < tr / 4u; i += 4) {
        double x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            x[u] = eval_tp64(MS_TP_LDROW ? ld_drow(d + 4 * (i + u)) : d[4 * (i + u)], ord0 + 4 * (i + u), part + 4 * (i + u), q);
        sort4_desc(x);
        merge4_desc(k, x);
    }
    const bool tol = (q.bits & kPfTol) != 0;
    uint32_t f = ((tb.any & kRbUnsched) && !tol ? 1u : 0u) | (tb.all & (tol ? kRbAbsent : kRbBlocked) ? 0u : 0x100u);
    quad_merge4<0xB1>(k, f);  // quad_perm [1,0,3,2]
    quad_merge4<0x4E>(k, f);  // quad_perm [2,3,0,1]
    if (pi < cnt) {
        const size_t cell = (size_t)(pbeg + pi) * a.n_tiles + tile;
        const double mine = part == 0 ? k[0] : part == 1 ? k[1] : part == 2 ? k[2] : k[3];
        const u64 g = global_key(mine, a.t.base + tile * tr);
        if (a.coh) {  // (launch-uniform)
            st_coh(a.tile_keys + cell * kTopK + part, g | (u64)a.coh << kListTagShift);
            if (part == 0) st_coh(a.tile_flags + cell, f | a.coh << 16);
        } else {
            a.tile_keys[cell * kTopK + part] = g;
            if (part == 0) a.tile_flags[cell] = f;
        }
    }
    return true;
#else
    u64 k[4] = {0ull, 0ull, 0ull, 0ull};
    // rows 4 at a time (LDS reads issued together at the top of each block)
#pragma unroll 1
    for (uint32_t i = 0; i < tr / 4u; i += 4) {
        u64 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = eval_tp(d[4 * (i + u)], ord0 + 4 * (i + u), q);
        sort4_desc(x);
        merge4_desc(k, x);
    }
    const bool tol = (q.bits & kPfTol) != 0;
    uint32_t f = ((tb.any & kRbUnsched) && !tol ? 1u : 0u) | (tb.all & (tol ? kRbAbsent : kRbBlocked) ? 0u : 0x100u);
    quad_merge4<0xB1>(k, f);  // quad_perm [1,0,3,2]
    quad_merge4<0x4E>(k, f);  // quad_perm [2,3,0,1]
    if (pi < cnt) {
        const size_t cell = (size_t)(pbeg + pi) * a.n_tiles + tile;
        tile_keys_store(a.tile_keys + cell * kTopK + part, part, k, a.coh);
        if (part == 0) {
            if (a.coh) st_coh(a.tile_flags + cell, f | a.coh << 16);
            else a.tile_flags[cell] = f;
        }
    }
    return true;
#endif
}

// One task of the lane = row sweep: (tile, pod chunk cidx of a.chunk pods).
__device__ __forceinline__ void sweep_topk_task(const SweepArgs &a, uint32_t tile, uint32_t cidx, uint32_t lane) {
    const uint32_t pbeg = cidx * a.chunk;
    if (pbeg >= a.n_pods) return;
    sweep_rows_task(a, tile, pbeg, min(min(a.chunk, 64u), a.n_pods - pbeg), lane);
}

// The transposed sweep of one tile by a workgroup of W waves: every thread
// stages the tile's rows, then wave w takes pod groups w, w + W, ..
// (block-uniform control flow: every wave reaches both barriers). Returns the
// wave's groups (bit i: its i-th group) outside the binary64 form's range,
// which sweep_tp_redo then takes in the lane = row form.
template <int W>
__device__ __forceinline__ uint32_t sweep_tp_tile(const SweepArgs &a, uint32_t tile, DRow *rows, uint32_t wave,
                                                  uint32_t lane, u64 *tl = nullptr) {
    __syncthreads();  // the previous tile's readers are done
    const uint32_t tr = tile_rows_of(a.t);
    const uint4 *src = reinterpret_cast<const uint4 *>(a.t.drow + (size_t)tile * tr);
    uint4 *dst = reinterpret_cast<uint4 *>(rows);
    const uint32_t n_vec = tr * (uint32_t)(sizeof(DRow) / sizeof(uint4));
    for (uint32_t i = threadIdx.x; i < n_vec; i += 64u * W) dst[i] = src[i];
    __syncthreads();
    if (tl && threadIdx.x == 0) tl[kTlStaged] = __builtin_amdgcn_s_memrealtime();  // (diagnostic builds)
    const TileBits tb = tile_bits(rows, lane, tr);
    // (a batch holds at most kSeqBatch <= 256 pods, i.e. 16 groups)
    uint32_t redo = 0;
    for (uint32_t grp = wave, i = 0; grp * kTpPods < a.n_pods; grp += W, ++i)
        if (!sweep_tp_task(a, tile, grp, lane, rows, tb)) redo |= 1u << i;
    return redo;
}

// The groups sweep_tp_tile left (bit i: the wave's i-th group), lane = row form.
template <int W>
__device__ __forceinline__ void sweep_tp_redo(const SweepArgs &a, uint32_t tile, uint32_t redo, uint32_t wave,
                                              uint32_t lane) {
    for (uint32_t grp = wave, i = 0; redo; grp += W, ++i)
        if (redo & (1u << i)) {
            redo &= ~(1u << i);
            sweep_rows_task_lean(a, tile, grp * kTpPods, min(kTpPods, a.n_pods - grp * kTpPods), lane);
        }
}

constexpr int kTpWaves = 8;  // standalone transposed sweep: 8 waves x 16 pods = a full batch per tile

__global__ __launch_bounds__(64 * kTpWaves) void k_sweep_tp_topk(SweepArgs a) {
    __shared__ DRow rows[kFullWaveTile];
    const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
    sweep_tp_redo<kTpWaves>(a, blockIdx.x, sweep_tp_tile<kTpWaves>(a, blockIdx.x, rows, wave, lane), wave, lane);
}

__global__ __launch_bounds__(kFullThreads) void k_sweep_full_topk(SweepArgs a) {
    const uint32_t tile = blockIdx.x * (kFullThreads / 64) + (threadIdx.x >> 6);
    if (tile >= a.n_tiles) return;  // wave-uniform; no block barriers in this kernel
    sweep_topk_task(a, tile, blockIdx.y, lane_id());
}

// ----------------------------------------------------------------------------
// Global speculative top-4 per pod, merged from the per-tile top-4 lists (one
// wave per pod). Exact: the global rank-r entry (r < 4) is within its tile's
// top r+1, so it is in its tile's list.
// ----------------------------------------------------------------------------
// Record of a touched node in the in-order validator, one i64 per field
// (F_INV_*: f32 bits of 100 / Allocatable); kSpecF fields come from the table.
constexpr int kRecF = 12;
constexpr int kSpecF = 9;
enum RecField { F_REQ_CPU = 0, F_REQ_MEM, F_NZ_CPU, F_NZ_MEM, F_ALLOC_CPU, F_ALLOC_MEM, F_CNT, F_ALLOWED, F_FD,
                F_ROW, F_INV_CPU, F_INV_MEM };

__device__ __forceinline__ uint32_t row_of_key(u64 k, uint32_t base) {
    return (0xFFFFFu - (uint32_t)(k & 0xFFFFFu)) - base;
}

// Field f (< kSpecF) of node row r's current device record.
__device__ __forceinline__ int64_t rec_field(const NodeTable &t, uint32_t r, uint32_t f) {
    switch (f) {
        case F_REQ_CPU: return t.req_cpu[r];
        case F_REQ_MEM: return t.req_mem[r];
        case F_NZ_CPU: return t.nz_cpu[r];
        case F_NZ_MEM: return t.nz_mem[r];
        case F_ALLOC_CPU: return t.alloc_cpu[r];
        case F_ALLOC_MEM: return t.alloc_mem[r];
        case F_CNT: return t.pod_count[r];
        case F_ALLOWED: return t.allowed_pods[r];
        default: return (int64_t)((uint32_t)t.flags[r] | ((uint32_t)t.digit[r] << 8));  // F_FD
    }
}

// The validator's record of key k's node (F_ROW = -1 for an empty entry),
// written with 16-byte stores so the validator copies it as is.
struct MergedRec {
    int64_t v[kSpecF];
    uint32_t row;  // ~0u: an empty entry
};

// The table loads of key k's record, issued (nothing waits for them here).
__device__ __forceinline__ MergedRec load_merged_rec(const NodeTable &t, u64 k) {
    MergedRec m;
    m.row = k ? row_of_key(k, t.base) : ~0u;
    const uint32_t r = k ? m.row : 0u;  // (row 0 is a valid address)
#pragma unroll
    for (uint32_t f = 0; f < (uint32_t)kSpecF; ++f) m.v[f] = rec_field(t, r, f);
    return m;
}

__device__ __forceinline__ void store_rec(const MergedRec &m, int64_t *dst) {
    int64_t v[kRecF];
    const bool e = m.row != ~0u;
#pragma unroll
    for (int f = 0; f < kSpecF; ++f) v[f] = e ? m.v[f] : 0;
    v[F_ROW] = e ? (int64_t)m.row : -1;
    v[F_INV_CPU] = e ? __float_as_uint(r100(m.v[F_ALLOC_CPU])) : 0;
    v[F_INV_MEM] = e ? __float_as_uint(r100(m.v[F_ALLOC_MEM])) : 0;
    longlong2 *d = reinterpret_cast<longlong2 *>(dst);
#pragma unroll
    for (int f = 0; f < kRecF; f += 2) d[f / 2] = make_longlong2(v[f], v[f + 1]);
}

__device__ __forceinline__ void store_merged_rec(const NodeTable &t, u64 k, int64_t *dst) {
    store_rec(load_merged_rec(t, k), dst);
}

struct NoTop4Hook {
    __device__ __forceinline__ void operator()(u64) const {}
};

// One wave merges pod p's tile lists: lane r < R gets the global rank-r key
// (out, 0 past the feasible rows), f the filters of the tiles with no feasible
// row (bit0 NodeUnschedulable, bit8 NodeResourcesFit; wave-uniform) and, in
// bits 16 / 24, those of all tiles with NodeResourcesFit for a tile that had a
// feasible row: the FitError mask once binds have filled every feasible row.
// cert: how many ranks are exact. A rank past 3 may miss a row when a tile's
// full list of four was used up before it (its fifth row is not listed), so
// the ranks after the one that exhausts a full list are not certified.
// COH: the lists are written in the same launch (ld_coh); with tag != 0 the
// lists carry it (MS_MERGE_TAGS) and the loads repeat until every list read
// has it, or until `deadline` (s_memrealtime) passes: then false, nothing out.
// at4(out): called on every lane once ranks 0..3 are final (lane r < 4 holds
// rank r), before the ranks past them are merged: the caller's record loads for
// those entries overlap the later rounds.
template <int J, int R = kTopK, bool COH = false, typename H = NoTop4Hook>
__device__ __forceinline__ bool merge_pod_lists(const u64 *__restrict__ tile_keys,
                                                const uint32_t *__restrict__ tile_flags, uint32_t p, uint32_t n_tiles,
                                                uint32_t lane, u64 &out, uint32_t &f, uint32_t *cert_out = nullptr,
                                                uint32_t tag = 0, uint64_t deadline = 0, const H &at4 = H(),
                                                uint64_t *t_poll = nullptr) {
    u64 e[J][kTopK];
    uint32_t pos[J];
    uint32_t tfs[J];
    uint32_t fl = 0;  // filters of this lane's tiles that have no feasible row
    uint32_t fa = 0;  // filters of all its tiles, + NRF for a tile with feasible rows
#ifndef MS_MERGE_FUSEDPOLL
// 1 (default): one poll loop loads flags and keys together, so the last poll is
// one memory round trip instead of two (E 38.52 -> 38.24 ms, profiles/r05u_e_ab.txt;
// 0: flags until tagged, then keys)
#define MS_MERGE_FUSEDPOLL 1
#endif
    if constexpr (COH) {
        if (tag && !MS_MERGE_FUSEDPOLL) {  // the flag words first (4 B per list), then the keys, each until tagged
            for (;;) {
                bool ok = true;
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    const uint32_t tt = lane + 64u * j;
                    tfs[j] = ld_coh(tile_flags + (size_t)p * n_tiles + min(tt, n_tiles - 1));
                    ok = ok && (tt >= n_tiles || (tfs[j] >> 16 & 3u) == tag);
                }
                if (__ballot(!ok) == 0) break;
                if (__builtin_amdgcn_s_memrealtime() > deadline) return false;
                __builtin_amdgcn_s_sleep(2);
            }
        }
    }
    for (;;) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const uint32_t tt = lane + 64u * j;
            const uint32_t tc = min(tt, n_tiles - 1);
            const size_t cell = (size_t)p * n_tiles + tc;
            if constexpr (COH) {
                if (!tag || MS_MERGE_FUSEDPOLL) {
                    tfs[j] = ld_coh(tile_flags + cell);
                    ok = ok && (!tag || tt >= n_tiles || (tfs[j] >> 16 & 3u) == tag);
                }
#pragma unroll
                for (int k = 0; k < kTopK; ++k) {
                    e[j][k] = ld_coh(tile_keys + cell * kTopK + k);
                    ok = ok && (!tag || tt >= n_tiles || (uint32_t)(e[j][k] >> kListTagShift) == tag);
                }
            } else {
                tfs[j] = tile_flags[cell];
                const uint4 *q = reinterpret_cast<const uint4 *>(tile_keys + cell * kTopK);
                const uint4 a = q[0], b = q[1];
                e[j][0] = ((u64)a.y << 32) | a.x;
                e[j][1] = ((u64)a.w << 32) | a.z;
                e[j][2] = ((u64)b.y << 32) | b.x;
                e[j][3] = ((u64)b.w << 32) | b.z;
            }
        }
        if (!COH || !tag || __ballot(!ok) == 0) break;
        if (__builtin_amdgcn_s_memrealtime() > deadline) return false;
#ifndef MS_MERGE_SLEEP
#define MS_MERGE_SLEEP 2  // s_sleep between a merge worker's list polls (x 64 cycles)
#endif
        __builtin_amdgcn_s_sleep(MS_MERGE_SLEEP);
    }
    if (t_poll) *t_poll = __builtin_amdgcn_s_memrealtime();  // (timeline build: every list arrived)
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const uint32_t tt = lane + 64u * j;
        pos[j] = tt < n_tiles ? 0u : (uint32_t)kTopK;
#pragma unroll
        for (int k = 0; k < kTopK; ++k) e[j][k] = untag_key(e[j][k]);
        const uint32_t tf = untag_flags(tfs[j]);
        if (tt < n_tiles && e[j][0] == 0) fl |= tf;
        if (tt < n_tiles) fa |= tf | (e[j][0] != 0 ? 0x100u : 0u);
    }
    out = 0;
    uint32_t cert = R;
#ifndef MS_MERGE_SORTED
#define MS_MERGE_SORTED 1  // each lane's lists merged into one sorted top-8 first; a round pops by a shift
#endif
    if (MS_MERGE_SORTED) {
        // The lane's own J lists (each sorted, best first) merged into its top
        // 8, best first: list j joins by Batcher's half merge (the elementwise
        // max of L and the list reversed is bitonic and holds the top 8), then a
        // bitonic sort of 8. A round then reads L[0] and the popping lane shifts:
        // a few independent selects instead of J list heads picked by position.
        u64 L[8];
        u64 sp[J];  // the last entry of each full list: popping it ends the certified ranks
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const bool in = lane + 64u * (uint32_t)j < n_tiles;  // (past n_tiles: the clamped tile's copy)
#pragma unroll
            for (int k = 0; k < kTopK; ++k) e[j][k] = in ? e[j][k] : 0ull;
            sp[j] = e[j][kTopK - 1];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) L[k] = k < kTopK ? e[0][k] : 0ull;
        const auto ce = [](u64 &a, u64 &b) {  // max to a
            const u64 x = a > b ? a : b, y = a > b ? b : a;
            a = x;
            b = y;
        };
#pragma unroll
        for (int j = 1; j < J; ++j) {
#pragma unroll
            for (int i = 8 - kTopK; i < 8; ++i) L[i] = L[i] > e[j][7 - i] ? L[i] : e[j][7 - i];
#pragma unroll
            for (int d = 4; d >= 1; d >>= 1)
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if ((i & d) == 0) ce(L[i], L[i + d]);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const u64 head = L[0];
            const u64 m = MS_MERGE_WMAX(head);
            if (lane == (uint32_t)r) out = m;
            const bool pop = m != 0 && head == m;  // keys are unique: exactly one lane pops
            bool used_up = false;
            if (R > kTopK) {
#pragma unroll
                for (int j = 0; j < J; ++j) used_up = used_up || (pop && head == sp[j]);
            }
#pragma unroll
            for (int i = 0; i < 7; ++i) L[i] = pop ? L[i + 1] : L[i];
            L[7] = pop ? 0ull : L[7];
            if (R > kTopK && cert == (uint32_t)R && __ballot(used_up)) cert = (uint32_t)r + 1u;
            if (r == kTopK - 1) at4(out);
        }
    } else
#pragma unroll
    for (int r = 0; r < R; ++r) {
        u64 head = 0;  // this lane's best list head
        int hj = -1;
#pragma unroll
        for (int j = 0; j < J; ++j) {
            u64 h = 0;
#pragma unroll
            for (int k = 0; k < kTopK; ++k) h = pos[j] == (uint32_t)k ? e[j][k] : h;
            if (h > head) {
                head = h;
                hj = j;
            }
        }
        const u64 m = MS_MERGE_WMAX(head);
        if (lane == (uint32_t)r) out = m;
        bool used_up = false;
        if (m != 0 && head == m) {  // keys are unique: exactly one lane pops
#pragma unroll
            for (int j = 0; j < J; ++j)
                if (j == hj) {
                    pos[j] += 1;
                    used_up = pos[j] == (uint32_t)kTopK;
                }
        }
        if (R > kTopK && cert == (uint32_t)R && __ballot(used_up)) cert = (uint32_t)r + 1u;
        if (r == kTopK - 1) at4(out);
    }
    if (cert_out) *cert_out = cert;
    f = (__ballot((fl & 0xFFu) != 0) ? 1u : 0u) | (__ballot((fl & 0xFF00u) != 0) ? 0x100u : 0u) |
        (__ballot((fa & 0xFFu) != 0) ? 0x10000u : 0u) | (__ballot((fa & 0xFF00u) != 0) ? 0x1000000u : 0u);
    return true;
}

// Per pod (one wave): merge the tiles' top-4 lists into the global top-4, the
// speculative winner and the no-feasible-row filter flags; recs (optional)
// gets the batch-start records of the four entries for the in-order validator.
// ext (optional): ranks 4..7 at ext[p * 4 + r - 4] and the number of certified
// ranks (4..8) in bits 28-31 of spec_flags (merge_pod_lists).
// One pod's merge by one wave (k_topk_merge, and k_seq_step's merge workgroups).
// tag / deadline: merge_pod_lists (COH, an in-step worker); false: the lists did
// not all arrive before the deadline and nothing was written.
template <int J, bool COH = false>
__device__ __forceinline__ bool merge_pod(const u64 *__restrict__ tile_keys, const uint32_t *__restrict__ tile_flags,
                                          uint32_t p, uint32_t n_tiles, u64 *__restrict__ top, u64 *__restrict__ spec,
                                          uint32_t *__restrict__ spec_flags, const NodeTable &t,
                                          int64_t *__restrict__ recs, u64 *__restrict__ ext, uint32_t lane,
                                          uint32_t tag = 0, uint64_t deadline = 0, uint64_t *t_poll = nullptr,
                                          uint64_t *t_rank = nullptr) {
    u64 out;
    uint32_t f, cert = 0;
#ifndef MS_MERGE_REC_EARLY
#define MS_MERGE_REC_EARLY 1  // the four records' table loads issued right after rank 3
#endif
    MergedRec mr;  // lanes 0..3: their entry's record
    const auto at4 = [&](u64 o) {
        if (MS_MERGE_REC_EARLY && recs && lane < (uint32_t)kTopK) mr = load_merged_rec(t, o);
    };
    if (ext) {
        if (!merge_pod_lists<J, kTopExt, COH>(tile_keys, tile_flags, p, n_tiles, lane, out, f, &cert, tag, deadline, at4,
                                              t_poll))
            return false;
        if (lane >= (uint32_t)kTopK && lane < (uint32_t)kTopExt) ext[(size_t)p * kTopK + lane - kTopK] = out;
    } else {
        if (!merge_pod_lists<J, kTopK, COH>(tile_keys, tile_flags, p, n_tiles, lane, out, f, nullptr, tag, deadline, at4,
                                            t_poll))
            return false;
    }
    if (t_rank) *t_rank = __builtin_amdgcn_s_memrealtime();  // (timeline build: ranks merged)
    if (lane < (uint32_t)kTopK) top[(size_t)p * kTopK + lane] = out;
    if (recs && lane < (uint32_t)kTopK) {
        if (!MS_MERGE_REC_EARLY) mr = load_merged_rec(t, out);
        store_rec(mr, recs + ((size_t)p * kTopK + lane) * kRecF);
    }
    // the speculative winner (rank 0) and, when no row is feasible, the filters
    if (lane == 0) {
        spec[p] = out;
        spec_flags[p] = f | (cert << 28);
    }
    return true;
}

template <int J>
__global__ __launch_bounds__(64) void k_topk_merge(const u64 *__restrict__ tile_keys,
                                                   const uint32_t *__restrict__ tile_flags, uint32_t n_pods,
                                                   uint32_t n_tiles, u64 *__restrict__ top, u64 *__restrict__ spec,
                                                   uint32_t *__restrict__ spec_flags, NodeTable t,
                                                   int64_t *__restrict__ recs, u64 *__restrict__ ext) {
    const uint32_t p = blockIdx.x;
    if (p >= n_pods) return;
    merge_pod<J>(tile_keys, tile_flags, p, n_tiles, top, spec, spec_flags, t, recs, ext, threadIdx.x);
}

// ----------------------------------------------------------------------------
// Exact sequential engine, in-order half: ONE wave walks the batch in queue
// order, with no barriers. A bind only lowers keys of the node it lands on
// (NRF feasibility and LeastAllocated are monotone in Requested/pod_count; NU,
// NN and the hash do not read them), so for each tile the first top-K entry
// whose node is untouched so far in the batch is still that tile's best among
// untouched nodes; touched entries above it are re-evaluated from the LDS copy
// of their current record. Only a tile whose K entries are all touched (and
// whose list is full) is re-swept against current state.
//
// Latency layout (one wave has nothing to hide latency behind):
//  - prologue: the batch's pod records, speculative winner rows (the sweep's
//    per-pod atomicMax) and those rows' batch-start records go to LDS;
//  - a lane owns tiles lane, lane+64, ...; their lists and flags are loaded
//    two pods ahead into one of two register buffers (the pod loop is
//    unrolled by two, so no buffer rotation forces a vmcnt wait);
//  - every head's touched-map probe is issued before any is tested;
//  - a 64-bit DPP max picks the winner; the lane that produced it knows
//    whether it is a touched node's LDS slot;
//  - the bind (NodeInfo.AddPod) updates that LDS record, one field per lane.
// Results and records stay in LDS until the batch ends.
// ----------------------------------------------------------------------------
#ifndef MS_SEQ_BATCH
#define MS_SEQ_BATCH 128
#endif
constexpr int kSeqBatch = MS_SEQ_BATCH;  // pods per speculative batch (host clamps); a multiple of 64
constexpr int kMapBits = 11;
constexpr int kMapCap = 1 << kMapBits;  // >= 4 x the nodes a batch and its predecessor bind
constexpr int kSeqMaxJ = 16;            // tile lists per lane in registers: n_tiles <= 1024 (262k rows)
constexpr int kClaimBits = 12;          // claim table: 64 lanes in 4096 buckets, ~0.8% false conflicts
constexpr int kClaimCap = 1 << kClaimBits;
constexpr uint32_t kForceSlow = 0xFFFFu;  // spec_slot: speculation could not be re-resolved
constexpr int kPrevCap = 2 * kSeqBatch;              // stale nodes: the two previous batches' binds
constexpr int kPrevSlot0 = kTopK * kSeqBatch;         // first slot of the stale nodes
constexpr int kSeqSlots = kPrevSlot0 + kPrevCap;      // <= 2048 (the map's slot field)
constexpr int kPrevWords = 2 + kPrevCap;              // prev lists: {n_own, n_carried, rows...}
constexpr uint32_t kSlotBits = 11;  // map entry = (row + 1) << kSlotBits | slot (rows < 2^21)
static_assert(kSeqSlots <= (1 << kSlotBits), "map entries hold an 11-bit slot");
static_assert(kSeqBatch % 64 == 0, "the validator takes pods 64 at a time");

// Record slots: rec[4p + r] is the batch-start record of pod p's top-4 entry
// r (k_topk_merge wrote it; it becomes that node's live record when pod p
// binds there first, and is dead otherwise); rec[kPrevSlot0 + i] are the
// stale nodes: those the previous one or two batches bound (pipelined mode:
// this batch's speculation may predate those binds), as the previous batch's
// validator left them. A node has at most one live slot: the map's.
struct WalkResult {
    u64 key;        // winner against the current state (0: none feasible among the listed)
    uint32_t slot;  // its record slot
    uint32_t flags; // bit0: untouched node (first bind inserts the map entry), bit1: needs the tile lists
};

struct SeqShared {
    alignas(16) uint32_t map[kMapCap];  // ((row + 1) << kSlotBits) | slot; 0 = empty
    int64_t rec[kSeqSlots][kRecF];
    alignas(16) uint8_t bound[kSeqSlots];  // binds on the slot in this batch (<= 128: no wrap)
    uint32_t n_out;
    uint32_t n_prorec;  // recomputes of the workgroup prologue (prologue_wg_finish), for the counters
    ms_pod_rec pods[kSeqBatch];
    u64 spec_key[kSeqBatch];     // speculative winner key per pod (0: no feasible row at speculation)
    uint32_t spec_flags[kSeqBatch];  // OR of the tile flags of tiles with no feasible row at speculation
    alignas(16) u64 top4[kSeqBatch][kTopK];  // global speculative top-4 keys per pod (k_topk_merge)
    u64 top_ext[kSeqBatch][kTopK];   // ranks 4..7 (keys only), exact up to cert[]
    uint8_t cert[kSeqBatch];         // certified ranks, 4..8 (4 without the extension)
    alignas(16) uint32_t claim[kClaimCap];  // per round: lowest lane whose speculative winner hashes here
    uint16_t spec_slot[kSeqBatch];   // slot of the speculative winner's record (kForceSlow: unresolved)
    uint32_t walk[16];               // a round's re-resolution pass: lanes whose pod walks its top-4
    uint16_t bl[kSeqBatch];          // write-back: the slots bound in this batch (one per binding pod at most)
    WalkResult walkres[16];          // and each one's winner
};
static_assert(sizeof(SeqShared) <= 160 * 1024, "validator LDS");
constexpr uint32_t kTpDeferCap = 32;  // deferred (tile, groups) entries per sweep wave (k_seq_step)
static_assert(sizeof(SeqShared) >= kFullWaveTile * sizeof(DRow) + 16u * kTpDeferCap * sizeof(uint32_t),  // (W <= 16)
              "a sweep workgroup stages a tile in it, and its waves' deferred lists after it");

__device__ __forceinline__ uint32_t map_hash(uint32_t row) { return (row * kGolden32) >> (32 - kMapBits); }
__device__ __forceinline__ uint32_t claim_hash(uint32_t row) { return (row * 0x85EBCA6Bu) >> (32 - kClaimBits); }

// slot of row in the touched-node map, -1 if untouched, continuing a probe
// whose first read returned v (load factor <= 1/4)
__device__ __forceinline__ int map_resolve(const SeqShared &S, uint32_t row, uint32_t v) {
    uint32_t h = map_hash(row);
    const uint32_t key = row + 1;
    for (;;) {
        if (v == 0) return -1;
        if ((v >> kSlotBits) == key) return (int)(v & ((1u << kSlotBits) - 1u));
        h = (h + 1) & (kMapCap - 1);
        v = S.map[h];
    }
}

__device__ __forceinline__ int map_find(const SeqShared &S, uint32_t row) {
    return map_resolve(S, row, S.map[map_hash(row)]);
}

__device__ __forceinline__ FullRow slot_row(const SeqShared &S, int sl) {
    const int64_t *r = S.rec[sl];
    FullRow x = make_row(r[F_ALLOC_CPU], r[F_ALLOC_MEM], r[F_REQ_CPU], r[F_REQ_MEM], r[F_NZ_CPU], r[F_NZ_MEM],
                         (int32_t)(r[F_ALLOWED] - r[F_CNT]), (uint32_t)r[F_FD]);
    x.r_cpu = __uint_as_float((uint32_t)r[F_INV_CPU]);  // (the division above is dead)
    x.r_mem = __uint_as_float((uint32_t)r[F_INV_MEM]);
    return x;
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void global_void_t;

// n16 16-byte units global src -> LDS dst (contiguous), straight to LDS with
// global_load_lds_dwordx4 (64 lanes x 16 B per instruction, no registers);
// the caller waits (s_waitcnt vmcnt(0)) before reading dst. U = units per
// lane at most; sources clamped to valid units.
template <int U>
__device__ __forceinline__ void lds_dma16(void *dst, const void *src, uint32_t n16, uint32_t lane) {
    if (n16 == 0) return;
    const uint4 *g = reinterpret_cast<const uint4 *>(src);
    uint4 *d = reinterpret_cast<uint4 *>(dst);
#ifdef MS_NO_LDS_DMA
#pragma unroll
    for (int k = 0; k < U; ++k) d[lane + 64 * k] = g[min(lane + 64u * k, n16 - 1)];
#else
#pragma unroll
    for (int k = 0; k < U; ++k)
        __builtin_amdgcn_global_load_lds((global_void_t *)(g + min(lane + 64u * k, n16 - 1)), (lds_void_t *)(d + 64 * k),
                                         16, 0, 0);
#endif
}

// The same copy issued by nthreads threads (tid < nthreads) of a workgroup:
// more loads in flight than one wave can hold (the step's idle validator
// waves help the validating wave's prologue). The caller waits and barriers.
__device__ __forceinline__ void lds_dma16_wg(void *dst, const void *src, uint32_t n16, uint32_t n_units, uint32_t tid,
                                             uint32_t nthreads) {
    if (n16 == 0) return;
    const uint4 *g = reinterpret_cast<const uint4 *>(src);
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    for (uint32_t u = tid; u < n_units; u += nthreads) {
#ifdef MS_NO_LDS_DMA
        d[u] = g[min(u, n16 - 1)];
#else
        // (global_load_lds writes lane i's 16 B at the wave's base + 16 i: the
        // wave-uniform base is d + u - lane)
        __builtin_amdgcn_global_load_lds((global_void_t *)(g + min(u, n16 - 1)), (lds_void_t *)(d + (u - (tid & 63u))),
                                         16, 0, 0);
#endif
    }
}

// Entry k (wave-divergent) of a register-held top-4 list, without the dynamic
// register indexing that would put the list in scratch.
__device__ __forceinline__ u64 pick4(const u64 (&e)[kTopK], int k) {
    return k == 0 ? e[0] : k == 1 ? e[1] : k == 2 ? e[2] : e[3];
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

template <int J>
struct TileLists {
    u64 e[J][kTopK];
    uint32_t f[J];
};

// Pod p's lists and flags for this lane's tiles. The loads are unconditional
// from clamped (always valid) cells: a zero-fill branch for the out-of-range
// lanes would write the load's destination registers and force the wave to
// wait for the loads right here. Consumers skip tiles outside the lane's
// `tiles` mask; lists of pods past the batch are never consumed.
template <int J>
__device__ __forceinline__ void load_lists(TileLists<J> &B, const u64 *__restrict__ tile_keys,
                                           const uint32_t *__restrict__ tile_flags, uint32_t p, uint32_t n_pods,
                                           uint32_t n_tiles, uint32_t lane) {
    const uint32_t pc = min(p, n_pods - 1);
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const uint32_t tt = min(lane + 64u * j, n_tiles - 1);
        const size_t cell = (size_t)pc * n_tiles + tt;
        const uint4 *q = reinterpret_cast<const uint4 *>(tile_keys + cell * kTopK);
        const uint4 a = q[0], b = q[1];
        // (lists of an in-step merged batch carry the step's tag, MS_MERGE_TAGS)
        B.e[j][0] = untag_key(((u64)a.y << 32) | a.x);
        B.e[j][1] = untag_key(((u64)a.w << 32) | a.z);
        B.e[j][2] = untag_key(((u64)b.y << 32) | b.x);
        B.e[j][3] = untag_key(((u64)b.w << 32) | b.z);
        B.f[j] = untag_flags(tile_flags[cell]);
    }
}

struct SeqCounters {
    uint32_t recompute, resweep, miss, slow, scan, rounds;
};


// Full scan of pod p's tile lists (the speculative winner was touched, or
// the pod had no feasible row at speculation): b = winner key, wslot = its
// LDS slot if it is a touched node.
template <int J>
__device__ __forceinline__ void validate_scan(SeqShared &S, const NodeTable &t, uint32_t n_rows, const PodFull &q,
                                              const TileLists<J> &B, uint32_t tiles, uint32_t lane, SeqCounters &ctr,
                                              u64 &b_out, int &wslot_out) {
    // (B was loaded on entry to the slow path: ~6% of config E's pods need it)
    // ---- every head's first map probe, issued together
    uint32_t hrow[J], hv[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        hrow[j] = row_of_key(B.e[j][0], t.base);
        hv[j] = (((tiles >> j) & 1u) && B.e[j][0]) ? S.map[map_hash(hrow[j])] : 0u;
    }
    // ---- every tile's best: first untouched list entry, touched ones re-evaluated
    u64 best = 0;
    int best_slot = -1;  // map slot of the lane's best when it came from a touched node
    uint32_t need = 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        if (!((tiles >> j) & 1u) || B.e[j][0] == 0) continue;  // no tile, or no feasible row at speculation
        int sl = map_resolve(S, hrow[j], hv[j]);
        if (sl < 0) {  // untouched head: exact, and the tile's best
            if (B.e[j][0] > best) {
                best = B.e[j][0];
                best_slot = -1;
            }
            continue;
        }
        // walk the list: touched entries are re-evaluated, the first untouched one ends it
        for (int k = 0;;) {
            const uint32_t row = row_of_key(pick4(B.e[j], k), t.base);
            uint32_t nu, nrf;
            const u64 r = eval_full(slot_row(S, sl), t.base + row, q, nu, nrf);
            ++ctr.recompute;
            if (r > best) {
                best = r;
                best_slot = sl;
            }
            if (++k == kTopK) {
                need |= 1u << j;  // K touched entries: the tile's next row is unknown, re-sweep it
                break;
            }
            const u64 e2 = pick4(B.e[j], k);
            if (e2 == 0) break;  // list ended: the remaining rows were infeasible and stay so
            sl = map_find(S, row_of_key(e2, t.base));
            if (sl < 0) {
                if (e2 > best) {
                    best = e2;
                    best_slot = -1;
                }
                break;
            }
        }
    }
    // ---- rare: tiles to re-sweep against current state, cooperatively (4 rows per lane)
    u64 need_any = __ballot(need != 0);
    while (need_any) {
        const uint32_t src = (uint32_t)__builtin_ctzll(need_any);
        const uint32_t bits = (uint32_t)__builtin_amdgcn_readlane((int)need, (int)src);
        const uint32_t tile = src + 64u * (uint32_t)__builtin_ctz(bits);
        if (lane == src) need &= need - 1;
        need_any = __ballot(need != 0);
        ++ctr.resweep;
#pragma unroll
        for (int sidx = 0; sidx < kFullSlots; ++sidx) {
            const uint32_t r = tile_slot_row(t, tile, lane * kFullSlots + sidx);  // (~0u past the tile: absent)
            FullRow x = load_row(t, r, n_rows);
            int sl = -1;
            if (r < n_rows) {
                sl = map_find(S, r);
                if (sl >= 0) x = slot_row(S, sl);
            }
            uint32_t nu, nrf;
            const u64 k = eval_full(x, t.base + r, q, nu, nrf);
            if (k > best) {
                best = k;
                best_slot = sl;
            }
        }
    }
    // ---- decide: 64-bit wave max; the owning lane knows the winner's slot
    const u64 b = wave_max_u64_dpp(best);
    const u64 own = __ballot(b != 0 && best == b);
    b_out = b;
    wslot_out = own ? __builtin_amdgcn_readlane(best_slot, (int)__builtin_ctzll(own)) : -1;
}

// Re-resolution of the pods of the lanes with `walk` set (pod index `pod`),
// 16 pods per pass with lane 4i + r on entry r of the pass's pod i: touched
// entries (in the map) are re-evaluated from their LDS records, the first
// untouched one is exact and bounds every row below it. Out, per walking lane:
// ck, its slot, cins (untouched: the pod's own record slot, whose first bind
// inserts the map entry) and need (four touched entries in a full list: the
// tile lists decide). ck == 0 without need: the list ended and none of its
// nodes is feasible now, so no node is (a FitError).
// EXT: a pod whose four entries are all touched continues into the merge's
// ranks 4..cert-1 (S.top_ext) by the same rule, 16 pods per pass: the first
// untouched one is exact (its record is fetched from the table into the pod's
// slot 4 pod, dead since all four of its top-4 nodes are touched) and bounds
// every row below it; `need` stays only when every certified entry is touched
// in a full list (the serial path then scans the tile lists). Without it those
// pods were resolved one at a time, each ending its round (round 6).
// Called by the whole wave (wave-uniform passes); clears `walk`.
template <bool EXT = false>
__device__ __forceinline__ void walk_top4(SeqShared &S, const NodeTable &t, uint32_t seed32, bool &walk, uint32_t pod,
                                          u64 &ck, uint32_t &cslot, bool &cins, bool &need, SeqCounters &ctr) {
    const uint32_t lane = lane_id();
    for (u64 wm = __ballot(walk); wm;) {
        const uint32_t nw = min(16u, (uint32_t)__builtin_popcountll(wm));
        const uint32_t rank = (uint32_t)__builtin_popcountll(wm & ((1ull << lane) - 1ull));
        if (walk && rank < 16u) S.walk[rank] = pod;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t qi = lane >> 2, r = lane & 3u;
        u64 v = 0;
        uint32_t vs = 0;
        bool unt = false, end = false;
        if (qi < nw) {
            const uint32_t pw = S.walk[qi];
            const u64 e = S.top4[pw][r];
            if (e == 0) {
                end = true;  // list ended: every feasible row was listed
            } else {
                const uint32_t er = row_of_key(e, t.base);
                const int es = map_find(S, er);
                if (es < 0) {
                    unt = true;
                    v = e;
                    vs = kTopK * pw + r;
                } else {
                    uint32_t nu, nrf;
                    v = eval_full(slot_row(S, es), er + t.base, load_pod(S.pods[pw], seed32), nu, nrf);
                    vs = (uint32_t)es;
                    ++ctr.recompute;
                }
            }
        }
        // entries past the quad's first untouched-or-end entry do not count
        const uint32_t qb = (uint32_t)(__ballot(unt || end) >> (4u * qi)) & 0xFu;
        const uint32_t f = qb ? (uint32_t)__builtin_ctz(qb) : 4u;
        const bool valid = qi < nw && !end && (r < f || (r == f && unt));
        const u64 ve = valid ? v : 0ull;
        const u64 m = quad_max_u64(ve);
        const uint32_t own = (uint32_t)(__ballot(valid && m != 0 && ve == m) >> (4u * qi)) & 0xFu;
        if (qi < nw && r == (own ? (uint32_t)__builtin_ctz(own) : 0u))
            S.walkres[qi] = {m, vs, (unt && m != 0 ? 1u : 0u) | (f == 4u ? 2u : 0u)};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (walk && rank < 16u) {
            const WalkResult w = S.walkres[rank];
            ck = w.key;
            cslot = w.slot;
            cins = (w.flags & 1u) != 0;
            need = (w.flags & 2u) != 0;
            walk = false;
        }
        __builtin_amdgcn_wave_barrier();
        wm = __ballot(walk);
    }
    if (!EXT) return;
    bool ext = need && S.cert[pod] > (uint8_t)kTopK;  // (need is set only on walking lanes)
    for (u64 wm = __ballot(ext); wm;) {
        const uint32_t nw = min(16u, (uint32_t)__builtin_popcountll(wm));
        const uint32_t rank = (uint32_t)__builtin_popcountll(wm & ((1ull << lane) - 1ull));
        if (ext && rank < 16u) S.walk[rank] = pod;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t qi = lane >> 2, r = lane & 3u;
        u64 v = 0;
        uint32_t vs = 0;
        bool unt = false, end = false, known = false;
        if (qi < nw) {
            const uint32_t pw = S.walk[qi];
            known = (uint32_t)kTopK + r < (uint32_t)S.cert[pw];
            const u64 e = known ? S.top_ext[pw][r] : 0ull;
            if (known && e == 0) {
                end = true;  // list ended within the certified ranks
            } else if (known) {
                const uint32_t er = row_of_key(e, t.base);
                const int es = map_find(S, er);
                if (es < 0) {
                    unt = true;
                    v = e;
                    vs = kTopK * pw;  // (the record is fetched below if this entry wins)
                } else {
                    uint32_t nu, nrf;
                    v = eval_full(slot_row(S, es), er + t.base, load_pod(S.pods[pw], seed32), nu, nrf);
                    vs = (uint32_t)es;
                    ++ctr.recompute;
                }
            }
        }
        const uint32_t qb = (uint32_t)(__ballot(known && (unt || end)) >> (4u * qi)) & 0xFu;
        const uint32_t f = qb ? (uint32_t)__builtin_ctz(qb) : 4u;
        const bool valid = known && !end && (r < f || (r == f && unt));
        const u64 ve = valid ? v : 0ull;
        const u64 m = quad_max_u64(ve);
        const uint32_t own = (uint32_t)(__ballot(valid && m != 0 && ve == m) >> (4u * qi)) & 0xFu;
        if (qi < nw && r == (own ? (uint32_t)__builtin_ctz(own) : 0u))
            S.walkres[qi] = {m, vs, (unt && m != 0 ? 1u : 0u) | (qb == 0u ? 2u : 0u)};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        bool fetch = false;
        if (ext && rank < 16u) {
            const WalkResult w = S.walkres[rank];
            if (w.key > ck) {  // (distinct nodes: keys never tie)
                ck = w.key;
                cslot = w.slot;
                cins = (w.flags & 1u) != 0;
                fetch = cins;
            }
            need = (w.flags & 2u) != 0;
            ext = false;
        }
        ctr.miss += (uint32_t)__builtin_popcountll(__ballot(fetch));
        if (fetch) store_merged_rec(t, ck, S.rec[cslot]);  // the untouched winner's current record
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        wm = __ballot(ext);
    }
}

// Deferred bind effects of a 64-pod group, lane i <-> pod i of the group:
//  prow/pslot: the (row, slot) map entry of a node pod i bound first in the batch;
//  padd: the slot pod i bound to, whose record still lacks pod i's NodeInfo.AddPod.
// Applied (all lanes at once) before anything reads the map or the records: a
// list scan, the next group's touched check, the write-back.
__device__ __forceinline__ void flush_pending(SeqShared &S, uint32_t &prow, uint32_t pslot, int &padd,
                                              const ms_pod_rec &mypod) {
    if (prow != 0xFFFFFFFFu) {
        uint32_t h = map_hash(prow);
        const uint32_t v = ((prow + 1) << kSlotBits) | pslot;
        while (atomicCAS(&S.map[h], 0u, v) != 0u) h = (h + 1) & (kMapCap - 1);
        prow = 0xFFFFFFFFu;
    }
    if (padd >= 0) {  // Requested += req, NonZeroRequested += nz, pod_count += 1
        unsigned long long *r = reinterpret_cast<unsigned long long *>(S.rec[padd]);
        atomicAdd(&r[F_REQ_CPU], (unsigned long long)mypod.req_milli_cpu);
        atomicAdd(&r[F_REQ_MEM], (unsigned long long)mypod.req_memory);
        atomicAdd(&r[F_NZ_CPU], (unsigned long long)mypod.nonzero_milli_cpu);
        atomicAdd(&r[F_NZ_MEM], (unsigned long long)mypod.nonzero_memory);
        atomicAdd(&r[F_CNT], 1ull);
        S.bound[padd] = (uint8_t)(S.bound[padd] + 1u);  // (decided lanes bind distinct slots)
        padd = -1;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ u64 readlane_u64(u64 v, uint32_t l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l);
    return ((u64)hi << 32) | lo;
}

// Diagnostic build only (make vstamps): cycles per validator phase, summed
// over the batch, land in stats[8..] (u64), printed at ms_destroy.
#ifdef MS_VSTAMPS
struct VStamps {
    u64 prev, acc[12];  // [9..11]: epilogue parts (counters, compaction, write-back), stored at stats u64 [12..14]
};
#define MS_VST_DECL VStamps vst = {__builtin_amdgcn_s_memtime(), {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}};
#define MS_VST(i)                                               \
    do {                                                        \
        __builtin_amdgcn_sched_barrier(0);                      \
        const u64 vst_now = __builtin_amdgcn_s_memtime();       \
        vst.acc[i] += vst_now - vst.prev;                       \
        vst.prev = vst_now;                                     \
        __builtin_amdgcn_sched_barrier(0);                      \
    } while (0)
#else
#define MS_VST_DECL
#define MS_VST(i) \
    do {          \
    } while (0)
#endif

// Stale-node list entry o: row and record (16-byte stores).
__device__ __forceinline__ void put_stale(uint32_t *rows, int64_t *recs, uint32_t o, uint32_t row, const int64_t *r) {
    rows[2 + o] = row;
    longlong2 *d = reinterpret_cast<longlong2 *>(recs + (size_t)o * kRecF);
#pragma unroll
    for (int f = 0; f < kRecF; f += 2) d[f / 2] = make_longlong2(r[f], r[f + 1]);
}

// One speculative batch's in-order validation (k_seq_step).
// stats: [0] overflow flags, [1] re-swept tiles, [2] recomputed entries, [3] pods,
//        [4] speculation misses (records loaded), [5] slow pods, [6] slow pods that scanned the tile lists
// top4/top4_recs: k_topk_merge's per-pod top-4 keys and their batch-start records
// prev_in/prev_out: {n_own, n_carried, rows...} of the stale nodes this batch
// sees / the next one will: rows [0, n_own) bound by the writing batch, then
// rows [n_own, n_own + n_carried) bound by its predecessor only (carry != 0:
// the next batch's speculation may predate both); prev_recs_in/out: their
// final records. prev_in null when this batch's sweep saw every earlier bind.
struct SeqArgs {
    NodeTable t;
    uint32_t n_rows;
    const ms_pod_rec *pods;
    uint32_t n_pods;
    uint32_t seed32;
    const u64 *tile_keys;
    const uint32_t *tile_flags;
    const u64 *spec;
    const uint32_t *spec_flags;
    const u64 *top4;
    const int64_t *top4_recs;
    const u64 *top_ext;  // optional: k_topk_merge's ranks 4..7 (certified count in spec_flags bits 28-31)
    uint32_t n_tiles;
    const uint32_t *prev_in;
    const int64_t *prev_recs_in;
    uint32_t *prev_out;
    int64_t *prev_recs_out;
    int carry;
    ms_result *results;
    uint32_t *stats;
    u64 *tl;  // (diagnostic timeline builds) this step's row: the validator's phase stamps
};

// The validator's LDS tables cleared by nthreads threads: touched-node map,
// per-slot bind counts, claim buckets.
__device__ __forceinline__ void validate_clear(SeqShared &S, uint32_t tid, uint32_t nthreads) {
    for (uint32_t i = tid; i < (uint32_t)kMapCap / 4; i += nthreads) reinterpret_cast<uint4 *>(S.map)[i] = make_uint4(0, 0, 0, 0);
    static_assert(kSeqSlots % 16 == 0, "bound[] is cleared 16 slots per lane");
    for (uint32_t i = tid; i < (uint32_t)kSeqSlots / 16; i += nthreads)
        reinterpret_cast<uint4 *>(S.bound)[i] = make_uint4(0, 0, 0, 0);
    for (uint32_t i = tid; i < (uint32_t)kClaimCap / 4; i += nthreads)
        reinterpret_cast<uint4 *>(S.claim)[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
}

// The validator's bulk prologue copies (the batch's top-4 records, ranks
// 4..7, the stale nodes' records: up to ~85 KB) issued by every thread of the
// workgroup; the caller waits for them and barriers before validate_batch
// (wg_dma = true) runs on one wave. Same units and layout as validate_batch's
// own copies.
__device__ __forceinline__ void validate_prologue_wg(SeqShared &S, const SeqArgs &va, uint32_t tid, uint32_t nthreads) {
    const uint32_t n_pods = va.n_pods;
    if (n_pods > (uint32_t)kSeqBatch) return;
    validate_clear(S, tid, nthreads);
    lds_dma16_wg(&S.rec[0][0], va.top4_recs, n_pods * kTopK * kRecF / 2, kSeqBatch * kTopK * kRecF / 2, tid, nthreads);
    if (va.top_ext)
        lds_dma16_wg(&S.top_ext[0][0], va.top_ext, n_pods * kTopK / 2, kSeqBatch * kTopK / 2, tid, nthreads);
    if (va.prev_in) {
        const uint32_t units = (va.carry ? kPrevCap : kSeqBatch) * kRecF / 2;
        lds_dma16_wg(&S.rec[kPrevSlot0][0], va.prev_recs_in, units, units, tid, nthreads);
    }
}

// The validator's whole prologue on all W waves of workgroup 0 (k_seq_step,
// MS_WG_PROLOGUE=2): validate_prologue_wave's work, its loads issued with the
// bulk copies (one memory round trip for the workgroup) and its speculative
// winner re-resolution spread over the waves, 16 pods per wave and pass (lane
// 4i + r on entry r of pod i), where the single wave took up to eight passes
// in a row. prologue_wg_issue clears the tables, issues everything and waits;
// prologue_wg_finish (after a barrier) stores, maps the stale nodes and
// resolves. validate_batch (pro 2) then starts at the decisions.
template <int W>
struct ProRegs {
    static constexpr uint32_t kNT = 64u * W;
    static constexpr int kPodU = (int)((kSeqBatch * sizeof(ms_pod_rec) / 8 + kNT - 1) / kNT);  // uint2 per thread
    static constexpr int kPW = (int)((kPrevWords + kNT - 1) / kNT);                            // prev_in words
    uint2 pod[kPodU];
    uint32_t prow[kPW];
    u64 sk;        // thread i < n_pods: pod i's speculative key
    uint32_t sf;   // and flags
    uint32_t n_prev;
};

template <int W>
__device__ __forceinline__ void prologue_wg_issue(SeqShared &S, const SeqArgs &va, uint32_t tid, ProRegs<W> &R) {
    constexpr uint32_t NT = ProRegs<W>::kNT;
    const uint32_t n_pods = va.n_pods;
    validate_prologue_wg(S, va, tid, NT);  // tables cleared, records / ranks 4..7 / stale records
    lds_dma16_wg(&S.top4[0][0], va.top4, n_pods * kTopK / 2, kSeqBatch * kTopK / 2, tid, NT);
    const uint2 *sp = reinterpret_cast<const uint2 *>(va.pods);
    const uint32_t n_pod_u = n_pods * (uint32_t)sizeof(ms_pod_rec) / 8;
#pragma unroll
    for (int k = 0; k < ProRegs<W>::kPodU; ++k) R.pod[k] = sp[min(tid + NT * k, n_pod_u - 1)];
    const uint32_t ts = min(tid, n_pods - 1);
    R.sk = va.spec[ts];
    R.sf = va.spec_flags[ts];
    const uint32_t *prev_in = va.prev_in;
#pragma unroll
    for (int k = 0; k < ProRegs<W>::kPW; ++k) R.prow[k] = prev_in ? prev_in[min(tid + NT * k, (uint32_t)kPrevWords - 1)] : 0u;
    R.n_prev = prev_in ? min(prev_in[0] + prev_in[1], (uint32_t)kPrevCap) : 0u;
    __builtin_amdgcn_s_waitcnt(0);
}

template <int W>
__device__ __forceinline__ void prologue_wg_finish(SeqShared &S, const SeqArgs &va, uint32_t tid, const ProRegs<W> &R) {
    constexpr uint32_t NT = ProRegs<W>::kNT;
    const uint32_t n_pods = va.n_pods, n_prev = R.n_prev;
    const uint32_t n_pod_u = n_pods * (uint32_t)sizeof(ms_pod_rec) / 8;
    uint2 *dp = reinterpret_cast<uint2 *>(S.pods);
#pragma unroll
    for (int k = 0; k < ProRegs<W>::kPodU; ++k)
        if (tid + NT * k < n_pod_u) dp[tid + NT * k] = R.pod[k];
    if (tid < n_pods) {  // (bits 28-31: the merge's certified ranks, 0 without ranks 4..7)
        S.spec_key[tid] = R.sk;
        S.spec_flags[tid] = R.sf & 0x0FFFFFFFu;
        S.cert[tid] = (uint8_t)max(R.sf >> 28, (uint32_t)kTopK);
    }
    if (tid == 0) {
        S.n_out = 0;
        S.n_prorec = 0;
    }
    // the stale nodes are "touched" (validate_prologue_wave); word a >= 2 of prev_in is stale node a - 2
#pragma unroll
    for (int k = 0; k < ProRegs<W>::kPW; ++k) {
        const uint32_t a = tid + NT * k;
        if (a >= 2 && a < n_prev + 2) {
            const uint32_t r = R.prow[k];
            uint32_t h = map_hash(r);
            while (atomicCAS(&S.map[h], 0u, ((r + 1) << kSlotBits) | (uint32_t)(kPrevSlot0 + a - 2)) != 0u)
                h = (h + 1) & (kMapCap - 1);
        }
    }
    __syncthreads();
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
    if (va.tl && tid == 0) va.tl[kTlMerged] = __builtin_amdgcn_s_memrealtime();  // (workgroup 0: stale nodes mapped)
#endif
    // each pod's speculative winner slot: its own top-4 record (normally entry
    // 0); a stale winner is re-resolved against the current state (walk_top4's
    // rule: touched entries from their records, the first untouched one exact;
    // all four touched, or none feasible: kForceSlow)
    const NodeTable &t = va.t;
    const uint32_t lane = tid & 63u, qi = lane >> 2, r = lane & 3u;
    uint32_t nrec = 0;
    for (uint32_t c0 = 16u * (tid >> 6); c0 < n_pods; c0 += 16u * W) {  // (wave-uniform trip count)
        const uint32_t p = c0 + qi;
        const bool inb = p < n_pods;
        const u64 sk = inb ? S.spec_key[p] : 0ull;
        const bool stale = sk && n_prev && map_find(S, row_of_key(sk, t.base)) >= 0;  // (quad-uniform)
        u64 v = 0;
        uint32_t vs = 0;
        bool unt = false, end = false;
        if (stale) {
            const u64 e = S.top4[p][r];
            if (e == 0) {
                end = true;
            } else {
                const uint32_t er = row_of_key(e, t.base);
                const int es = map_find(S, er);
                if (es < 0) {
                    unt = true;
                    v = e;
                    vs = kTopK * p + r;
                } else {
                    uint32_t nu, nrf;
                    v = eval_full(slot_row(S, es), er + t.base, load_pod(S.pods[p], va.seed32), nu, nrf);
                    vs = (uint32_t)es;
                    ++nrec;
                }
            }
        }
        const uint32_t qb = (uint32_t)(__ballot(unt || end) >> (4u * qi)) & 0xFu;
        const uint32_t f = qb ? (uint32_t)__builtin_ctz(qb) : 4u;
        const bool valid = stale && !end && (r < f || (r == f && unt));
        const u64 ve = valid ? v : 0ull;
        const u64 m = quad_max_u64(ve);
        const uint32_t own = (uint32_t)(__ballot(valid && m != 0 && ve == m) >> (4u * qi)) & 0xFu;
        if (inb && r == (own ? (uint32_t)__builtin_ctz(own) : 0u)) {
            uint32_t sslot = kTopK * p;
            if (stale) {
                if (f != 4u && m != 0) {
                    S.spec_key[p] = m;
                    sslot = vs;
                } else {
                    sslot = kForceSlow;
                }
            }
            S.spec_slot[p] = (uint16_t)sslot;
        }
    }
    const uint32_t rsum = wave_sum_u32_dpp(nrec);
    if (lane == 0 && rsum) atomicAdd(&S.n_prorec, rsum);  // (LDS: a global atomic here would hold the barrier)
    __syncthreads();
}

// The validator's prologue on its one wave (k_seq_step with
// MS_WG_PROLOGUE=1, whose workgroup issued the bulk copies: wg_dma): the
// batch's pods, top-4 keys and speculative winners into LDS, the stale nodes
// mapped, each pod's speculative winner slot resolved. Returns prev_in[0].
__device__ __forceinline__ uint32_t validate_prologue_wave(SeqShared &S, const SeqArgs &va, uint32_t lane, bool wg_dma,
                                                           SeqCounters &ctr) {
    const NodeTable &t = va.t;
    const uint32_t n_pods = va.n_pods, seed32 = va.seed32;
    const ms_pod_rec *__restrict__ pods = va.pods;
    const u64 *__restrict__ spec = va.spec;
    const uint32_t *__restrict__ spec_flags = va.spec_flags;
    const u64 *__restrict__ top4 = va.top4;
    const int64_t *__restrict__ top4_recs = va.top4_recs;
    const uint32_t *__restrict__ prev_in = va.prev_in;
    const int64_t *__restrict__ prev_recs_in = va.prev_recs_in;
    const int carry = va.carry;
    // prologue, one memory round trip: every load below is issued (from clamped,
    // always valid addresses; no branches) before the first wait. The records
    // go global -> LDS directly (no registers); stores past the batch stay
    // inside the LDS arrays and are never read.
    constexpr int kPodU = (kSeqBatch * (int)sizeof(ms_pod_rec) / 8) / 64;  // uint2 per lane
    constexpr int kTopU = (kSeqBatch * kTopK * 8 / 16) / 64;                // uint4 per lane
    constexpr int kRecU = (kSeqBatch * kTopK * kRecF * 8 / 16) / 64;
    constexpr int kPrevU = (kPrevCap * kRecF * 8 / 16) / 64;
    constexpr int kPrevW = (kPrevWords + 63) / 64;  // prev_in words per lane
    constexpr int kSpecU = kSeqBatch / 64;
    static_assert(kPodU * 64 * 8 == kSeqBatch * (int)sizeof(ms_pod_rec) && kTopU * 64 * 16 == kSeqBatch * kTopK * 8 &&
                      kRecU * 64 * 16 == kPrevSlot0 * kRecF * 8 && kPrevU * 64 * 16 == kPrevCap * kRecF * 8 &&
                      kSpecU * 64 == kSeqBatch,
                  "prologue copies tile the LDS arrays exactly");
    if (!wg_dma) {  // (else the whole workgroup issued these copies: validate_prologue_wg)
        lds_dma16<kRecU>(&S.rec[0][0], top4_recs, n_pods * kTopK * kRecF / 2, lane);
        if (va.top_ext) lds_dma16<kTopU>(&S.top_ext[0][0], va.top_ext, n_pods * kTopK / 2, lane);
        if (prev_in) {  // (a writer without carry left at most kSeqBatch entries)
            if (carry) lds_dma16<kPrevU>(&S.rec[kPrevSlot0][0], prev_recs_in, kPrevCap * kRecF / 2, lane);
            else lds_dma16<kPrevU / 2>(&S.rec[kPrevSlot0][0], prev_recs_in, kSeqBatch * kRecF / 2, lane);
        }
    }
    const uint32_t n_pod_u = n_pods * (uint32_t)sizeof(ms_pod_rec) / 8, n_top_u = n_pods * kTopK / 2;
    uint2 vpod[kPodU];
    uint4 vtop[kTopU];
    u64 vspec[kSpecU];
    uint32_t vflag[kSpecU], vprow[kPrevW];
    {
        const uint2 *sp = reinterpret_cast<const uint2 *>(pods);
        const uint4 *st = reinterpret_cast<const uint4 *>(top4);
#pragma unroll
        for (int k = 0; k < kPodU; ++k) vpod[k] = sp[min(lane + 64u * k, n_pod_u - 1)];
#pragma unroll
        for (int k = 0; k < kTopU; ++k) vtop[k] = st[min(lane + 64u * k, n_top_u - 1)];
#pragma unroll
        for (int k = 0; k < kSpecU; ++k) {
            vspec[k] = spec[min(lane + 64u * k, n_pods - 1)];
            vflag[k] = spec_flags[min(lane + 64u * k, n_pods - 1)];
        }
#pragma unroll
        for (int k = 0; k < kPrevW; ++k) vprow[k] = prev_in ? prev_in[min(lane + 64u * k, (uint32_t)kPrevWords - 1)] : 0u;
    }
    if (!wg_dma) validate_clear(S, lane, 64u);
    if (lane == 0) S.n_out = 0;
    {
        uint2 *dp = reinterpret_cast<uint2 *>(S.pods);
        uint4 *dt = reinterpret_cast<uint4 *>(&S.top4[0][0]);
#pragma unroll
        for (int k = 0; k < kPodU; ++k) dp[lane + 64u * k] = vpod[k];
#pragma unroll
        for (int k = 0; k < kTopU; ++k) dt[lane + 64u * k] = vtop[k];
#pragma unroll
        for (int k = 0; k < kSpecU; ++k) {  // (bits 28-31: the merge's certified ranks, 0 without ranks 4..7)
            S.spec_key[lane + 64u * k] = vspec[k];
            S.spec_flags[lane + 64u * k] = vflag[k] & 0x0FFFFFFFu;
            S.cert[lane + 64u * k] = (uint8_t)max(vflag[k] >> 28, (uint32_t)kTopK);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);  // the LDS DMA above has landed
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
    if (va.tl && lane == 0) va.tl[kTlWaited] = __builtin_amdgcn_s_memrealtime();  // (workgroup 0: wave-0 loads landed)
#endif
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // the stale nodes are "touched" here: this batch's speculation may have read
    // them before or during their batches' write-back. Word a >= 2 of prev_in
    // is stale node a - 2 (the two lists hold distinct rows).
    const uint32_t n_own_in = prev_in ? (uint32_t)__builtin_amdgcn_readfirstlane((int)vprow[0]) : 0u;
    const uint32_t n_prev =
        prev_in ? min(n_own_in + (uint32_t)__builtin_amdgcn_readlane((int)vprow[0], 1), (uint32_t)kPrevCap) : 0u;
#pragma unroll
    for (int k = 0; k < kPrevW; ++k) {
        const uint32_t a = lane + 64u * k;
        if (a >= 2 && a < n_prev + 2) {
            const uint32_t r = vprow[k];
            uint32_t h = map_hash(r);
            while (atomicCAS(&S.map[h], 0u, ((r + 1) << kSlotBits) | (uint32_t)(kPrevSlot0 + a - 2)) != 0u)
                h = (h + 1) & (kMapCap - 1);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
    if (va.tl && lane == 0) va.tl[kTlMerged] = __builtin_amdgcn_s_memrealtime();  // (workgroup 0: stale nodes mapped)
#endif
    // each pod's speculative winner slot: its own top-4 record (normally entry 0).
    // Pipelined: a winner that is a stale node (bound by a previous batch after
    // this batch's speculation may have read it) is re-resolved against the
    // current state, nothing of this batch being bound yet (walk_top4); all
    // four entries stale, or none feasible now: resolved in order (kForceSlow).
    for (uint32_t i0 = 0; i0 < (uint32_t)kSeqBatch; i0 += 64) {  // (wave-uniform trip count)
        const uint32_t i = i0 + lane;
        const u64 sk = i < n_pods ? S.spec_key[i] : 0ull;
        bool walk = sk && n_prev && map_find(S, row_of_key(sk, t.base)) >= 0;
        u64 ck = 0;
        uint32_t cslot = 0;
        bool cins = false, need = false;
        const bool stale = walk;
        walk_top4(S, t, seed32, walk, i, ck, cslot, cins, need, ctr);
        if (i < n_pods) {
            uint32_t sslot = kTopK * i;
            if (stale) {
                if (!need && ck != 0) {
                    S.spec_key[i] = ck;
                    sslot = cslot;
                } else {
                    sslot = kForceSlow;
                }
            }
            S.spec_slot[i] = (uint16_t)sslot;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return n_own_in;
}

template <int J>  // tile lists per lane: n_tiles <= 64 * J
__device__ __forceinline__ void validate_batch(SeqShared &S, const SeqArgs &va, uint32_t lane, int pro = 0) {
    const NodeTable &t = va.t;
    const uint32_t n_rows = va.n_rows, n_pods = va.n_pods, seed32 = va.seed32, n_tiles = va.n_tiles;
    const u64 *__restrict__ tile_keys = va.tile_keys;
    const uint32_t *__restrict__ tile_flags = va.tile_flags;
    const uint32_t *__restrict__ prev_in = va.prev_in;
    uint32_t *__restrict__ prev_out = va.prev_out;
    int64_t *__restrict__ prev_recs_out = va.prev_recs_out;
    const int carry = va.carry;
    ms_result *__restrict__ results = va.results;
    uint32_t *__restrict__ stats = va.stats;
    if (n_pods > (uint32_t)kSeqBatch || n_tiles > 64u * J) {  // host guarantees this
        if (lane == 0) atomicOr(&stats[0], 1u);
        return;
    }
    MS_VST_DECL
    SeqCounters ctr = {0, 0, 0, 0, 0, 0};
    // (pro 2: the whole prologue ran on the workgroup: prologue_wg_issue / _finish)
    // (pro 2: prev_in[0] is read only where it is used, in the carry branch at the end: a
    // scalar load issued here would hold every LDS wait of the decisions until it landed)
    const uint32_t n_own_wave = pro == 2 ? 0u : validate_prologue_wave(S, va, lane, pro == 1, ctr);
    if (pro == 2 && lane == 0) ctr.recompute = S.n_prorec;  // (summed over lanes at the end)
    uint32_t tiles = 0;  // tiles: bit j <=> this lane owns tile lane + 64 j
#pragma unroll
    for (int j = 0; j < J; ++j) tiles |= (lane + 64u * j < n_tiles) ? 1u << j : 0u;
    MS_VST(0);
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
    if (va.tl && lane == 0) va.tl[kTlWave0] = __builtin_amdgcn_s_memrealtime();  // (workgroup 0: prologue done)
#endif

    // Pods go in groups of 64, lane i <-> pod g+i, decided in rounds. A round
    // takes the group's undecided pods i0.. in parallel, each with its winner
    // against the state at the round's start: the speculative winner while its
    // node is untouched (not bound in this batch; current keys never exceed
    // speculative ones), else re-resolved from its top-4 on the lane itself
    // (touched entries re-evaluated from their LDS records, the first untouched
    // one exact and bounding every row below it). The first pod whose winner is
    // claimed by an earlier undecided pod (hash claim; collisions only make
    // false conflicts) or that needs its tile lists (four touched entries in a
    // full list, or no feasible node left) is the round's stop s. Pods i0..s-1
    // take their winners and bind at once: their winners are distinct, and a
    // bind only lowers its own node's keys. A claimed pod s is re-resolved in the
    // next round, which starts at s; a pod that needs its lists is resolved
    // alone (below) and the next round starts at s+1.
    for (uint32_t g = 0; g < n_pods; g += 64) {
        const uint32_t gn = min(64u, n_pods - g);
        const bool mine = lane < gn;
        const uint32_t pl = g + (mine ? lane : 0u);
        const u64 sk_l = mine ? S.spec_key[pl] : 0ull;
        const uint32_t srow_l = sk_l ? row_of_key(sk_l, t.base) : 0xFFFFFFFEu;
        const int dig_l = mine ? (int)S.pods[pl].name_digit : 0;
        const uint32_t ss_l = mine ? (uint32_t)S.spec_slot[pl] : 0u;
        const ms_pod_rec &mypod = S.pods[pl];
        uint32_t prow = 0xFFFFFFFFu, pslot = 0;  // this lane's pending map insert
        int padd = -1;                           // and pending AddPod (flush_pending)
        u64 rk = 0;                              // this lane's pod: winner key
        uint32_t rinfo = 0;                      // and code | plugin mask << 8
        MS_VST(1);
        // this lane's winner against the state at the start of the round that
        // computed it; kept while its node is not bound again (a bind only
        // lowers its own node's keys, so no other bind can change the max).
        // Every bind is a decided claimant's (or the serial pod's), so a lane
        // whose claim lost to an earlier lane, or whose node the serial pod
        // took, recomputes; collisions in the claim hash only recompute early.
        u64 ck = 0;
        uint32_t cslot = 0, crow = 0xFFFFFFFEu;
        bool cins = false, need = false, cvalid = false;  // first bind on an untouched node / needs the lists
        for (uint32_t i0 = 0; i0 < gn;) {
            const bool act = mine && lane >= i0 && sk_l != 0;
            bool walk = false;  // re-resolve from the top-4 (below, four lanes per pod)
            if (act && !cvalid) {
                cvalid = true;
                ck = 0;
                cins = false;
                need = false;
                // touched: bound earlier in the batch (a previous batch's node
                // whose record is in the map is touched only once bound again)
                const int sl = map_find(S, srow_l);
                if (ss_l != kForceSlow && !(sl >= 0 && (sl < kPrevSlot0 || S.bound[sl]))) {
                    ck = sk_l;
                    cslot = ss_l;
                    crow = srow_l;
                    cins = ss_l < (uint32_t)kPrevSlot0;  // pod pl's own record of an untouched node
                } else {
                    walk = true;
                }
            }
            walk_top4<true>(S, t, seed32, walk, pl, ck, cslot, cins, need, ctr);
            if (act && cvalid) crow = ck ? row_of_key(ck, t.base) : 0xFFFFFFFEu;
            MS_VST(7);
            const bool claims = act && !need && ck != 0 && dig_l >= 0;  // binds at ck if decided this round
            const uint32_t ch = claim_hash(crow);
            if (claims) atomicMin(&S.claim[ch], lane);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            // (a pod that cannot bind -- no NodeNumber digit -- still watches its
            // winner's bucket: a bind there can leave it with no feasible node)
            const bool lost = act && !need && ck != 0 && S.claim[ch] < lane;
            const bool conflict = act && (need || lost);
            if (lost) cvalid = false;
            const u64 bad = __ballot(conflict);
            const uint32_t s = bad ? (uint32_t)__builtin_ctzll(bad) : gn;
            const bool serial = bad && ((__ballot(need) >> s) & 1ull);
            __builtin_amdgcn_wave_barrier();
            if (claims) S.claim[ch] = ~0u;  // (every lane read its bucket above)
            MS_VST(8);
            if (mine && lane >= i0 && lane < s) {  // decided: exact against the round-start state
                rk = ck;
                if (ck == 0) {  // no feasible node: none at speculation (the empty tiles' filters)
                    // or binds filled every listed one (all tiles' filters, + NRF)
                    const uint32_t fm = sk_l == 0 ? S.spec_flags[pl] : S.spec_flags[pl] >> 16;
                    rinfo = MS_CODE_UNSCHEDULABLE | ((((fm & 0xFFu) ? MS_MASK_NODE_UNSCHEDULABLE : 0u) |
                                                      ((fm & 0xFF00u) ? MS_MASK_NODE_RESOURCES_FIT : 0u))
                                                     << 8);
                } else if (dig_l < 0) {
                    rinfo = MS_CODE_ERROR;  // NodeNumber.Score fails (nodenumber.go:74-77); nothing binds
                } else {
                    rinfo = MS_CODE_SUCCESS;
                    if (cins) {  // first bind on this node in the batch: pod pl's own record
                        prow = crow;
                        pslot = cslot;
                    }
                    padd = (int)cslot;
                }
            }
            flush_pending(S, prow, pslot, padd, mypod);
            ++ctr.rounds;
            MS_VST(4);
            if (s == gn) break;
            if (!serial) {  // claimed: re-resolved next round (then first, so unclaimed)
                i0 = s;
                continue;
            }
            // ---- slow pod p: resolved against current state
            const uint32_t p = g + s;
            ++ctr.slow;
            const PodFull q = load_pod(S.pods[p], seed32);
            u64 b = 0;
            int wslot = -1;
            uint32_t fmask = 0;
            // the global list (lanes 0-3: the top-4, 4..7: the merge's further
            // ranks, exact below cert): touched entries are re-evaluated from
            // their records, the first untouched one is exact and bounds every row
            // below it; an entry 0 within the certified ranks ends the list (every
            // feasible row was listed). No untouched or ending entry among them:
            // the rows below are unknown and the tile lists decide.
            const uint32_t C = S.cert[p];
            const bool known = lane < C;
            const u64 e = lane < (uint32_t)kTopK ? S.top4[p][lane] : known ? S.top_ext[p][lane - kTopK] : 0ull;
            const int esl = (known && e) ? map_find(S, row_of_key(e, t.base)) : -1;
            const u64 untouched = __ballot(known && e != 0 && esl < 0);
            const u64 stop = untouched | __ballot(known && e == 0);
            bool scan = false;
            TileLists<J> B;
            if (stop) {
                const uint32_t f = (uint32_t)__builtin_ctzll(stop);
                u64 v = 0;
                int vs = -1;
                if (lane < f) {  // (touched, non-zero)
                    uint32_t nu, nrf;
                    v = eval_full(slot_row(S, esl), row_of_key(e, t.base) + t.base, q, nu, nrf);
                    vs = esl;
                    ++ctr.recompute;
                } else if (lane == f) {
                    v = e;  // untouched: exact; or 0, the end of the list
                }
                b = wave_max_u64_dpp(v);
                const u64 own = __ballot(b != 0 && v == b);
                wslot = own ? __builtin_amdgcn_readlane(vs, (int)__builtin_ctzll(own)) : -1;
            } else {
                scan = true;  // every known entry touched: rows below them are unknown
                load_lists(B, tile_keys, tile_flags, p, n_pods, n_tiles, lane);
                ++ctr.scan;
                validate_scan<J>(S, t, n_rows, q, B, tiles, lane, ctr, b, wslot);
            }
            uint32_t info;
            if (b == 0) {  // per tile: speculative flags, + NRF if its feasible rows were all bound away
                if (scan) {
                    uint32_t fl = 0;
#pragma unroll
                    for (int j = 0; j < J; ++j)
                        if ((tiles >> j) & 1u) fl |= B.f[j] | (B.e[j][0] != 0 ? 0x100u : 0u);
                    fmask = (__ballot((fl & 0xFFu) != 0) ? 1u : 0u) | (__ballot((fl & 0xFF00u) != 0) ? 0x100u : 0u);
                } else {
                    fmask = S.spec_flags[p] >> 16;  // the same OR over tiles, kept by the merge (bits 16 / 24)
                }
                info = MS_CODE_UNSCHEDULABLE | ((((fmask & 0xFFu) ? MS_MASK_NODE_UNSCHEDULABLE : 0u) |
                                                 ((fmask & 0xFF00u) ? MS_MASK_NODE_RESOURCES_FIT : 0u))
                                                << 8);
            } else if (__builtin_amdgcn_readlane(dig_l, (int)s) < 0) {
                info = MS_CODE_ERROR;
            } else {
                info = MS_CODE_SUCCESS;
                // assume-on-select: NodeInfo.AddPod on the winner's LDS record
                const uint32_t row = row_of_key(b, t.base);
                int sl = wslot;
                if (sl < 0) {  // untouched winner: its batch-start record (pod p's top-4, or from the table)
                    const u64 hit = __ballot(lane < (uint32_t)kTopK && e == b);
                    sl = (int)(kTopK * p);
                    if (hit) {
                        sl += (int)__builtin_ctzll(hit);
                    } else {  // (a list scan's winner) into slot 4p: pod p binds elsewhere than its top-4
                        ++ctr.miss;
                        int64_t v = lane < (uint32_t)kSpecF ? rec_field(t, row, lane) : 0;
                        const int64_t capc = readlane64(v, F_ALLOC_CPU), capm = readlane64(v, F_ALLOC_MEM);
                        if (lane == (uint32_t)F_ROW) v = row;
                        if (lane == (uint32_t)F_INV_CPU) v = __float_as_uint(r100(capc));
                        if (lane == (uint32_t)F_INV_MEM) v = __float_as_uint(r100(capm));
                        if (lane < (uint32_t)kRecF) S.rec[sl][lane] = v;
                    }
                    if (lane == s) {
                        prow = row;
                        pslot = (uint32_t)sl;
                    }
                }
                if (lane == s) padd = sl;
                if (crow == row) cvalid = false;  // the serial pod took this lane's winner
            }
            if (lane == s) {
                rk = b;
                rinfo = info;
            }
            flush_pending(S, prow, pslot, padd, mypod);
#ifdef MS_VSTAMPS
            if (ctr.slow == 1) MS_VST(6);  // the batch's first slow pod (cold caches)
            else MS_VST(3);
#endif
            i0 = s + 1;
        }
        if (mine) {  // this lane's pod result
            ms_result r;
            r._pad = 0;
            r.code = (int32_t)(rinfo & 0xFFu);
            r.plugin_mask = rinfo >> 8;
            const bool ok = r.code == MS_CODE_SUCCESS;
            r.node = ok ? (int32_t)(0xFFFFFu - (uint32_t)(rk & 0xFFFFFu)) : -1;
            r.score = ok ? (int64_t)(rk >> 52) : 0;
            results[pl] = r;
        }
        MS_VST(1);
    }
    // counters (one atomic instruction: lane i adds counter i + 1; the recomputes
    // are per lane, the rest wave-uniform), then every touched node's record
    // goes back to the table
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
    if (va.tl && lane == 0) va.tl[kTlStaged] = __builtin_amdgcn_s_memrealtime();  // (workgroup 0: decisions done)
#endif
    {
        const uint32_t rsum = wave_sum_u32_dpp(ctr.recompute);
        const uint32_t v = lane == 0 ? ctr.resweep : lane == 1 ? rsum : lane == 2 ? n_pods : lane == 3 ? ctr.miss
                           : lane == 4 ? ctr.slow : lane == 5 ? ctr.scan : lane == 6 ? ctr.rounds : 0u;
#ifdef MS_VSTAMPS
        constexpr uint32_t kCounters = 7;
#else
        constexpr uint32_t kCounters = 6;
#endif
        if (lane < kCounters && v) atomicAdd(&stats[1 + lane], v);
    }
    MS_VST(9);
    // the bound slots (not a dead copy or an untouched stale node), compacted
    // with ballots into bl[], then written back one slot per lane
    uint32_t n_bl = 0;
    {
        constexpr int kChunks = kSeqSlots / 64;
        static_assert(kSeqSlots % 64 == 0, "bound[] scanned 64 slots at a time");
        uint32_t bv[kChunks];
#pragma unroll
        for (int c = 0; c < kChunks; ++c) bv[c] = S.bound[c * 64 + lane];
#pragma unroll
        for (int c = 0; c < kChunks; ++c) {
            const u64 m = __ballot(bv[c] != 0u);
            if (bv[c]) S.bl[n_bl + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull))] = (uint16_t)(c * 64 + lane);
            n_bl += (uint32_t)__builtin_popcountll(m);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    MS_VST(10);
    for (uint32_t o = lane; o < n_bl; o += 64) {
        const int64_t *r = S.rec[S.bl[o]];
        const uint32_t row = (uint32_t)r[F_ROW];
        t.req_cpu[row] = r[F_REQ_CPU];
        t.req_mem[row] = r[F_REQ_MEM];
        t.nz_cpu[row] = r[F_NZ_CPU];
        t.nz_mem[row] = r[F_NZ_MEM];
        t.pod_count[row] = (int32_t)r[F_CNT];
        if (t.drow)  // the next sweep's derived row (a sweep reading it now treats the row as stale)
            t.drow[row] = make_drow(r[F_ALLOC_CPU], r[F_ALLOC_MEM], r[F_REQ_CPU], r[F_REQ_MEM], r[F_NZ_CPU],
                                    r[F_NZ_MEM], (int32_t)(r[F_ALLOWED] - r[F_CNT]), (uint32_t)r[F_FD]);
        if (prev_out) put_stale(prev_out, prev_recs_out, o, row, r);
    }
    if (lane == 0) S.n_out = n_bl;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    MS_VST(11);
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
    if (va.tl && lane == 0) va.tl[kTlTasks] = __builtin_amdgcn_s_memrealtime();  // (workgroup 0: write-back issued)
#endif
    if (prev_out) {
        // carried: the previous batch's own binds that this batch did not bind again
        const uint32_t n_own = S.n_out;
        const uint32_t n_own_in = carry ? (pro == 2 ? (prev_in ? prev_in[0] : 0u) : n_own_wave) : 0u;
        if (carry)
            for (uint32_t i = lane; i < min(n_own_in, (uint32_t)kSeqBatch); i += 64) {
                const uint32_t sl = kPrevSlot0 + i;
                if (!S.bound[sl]) put_stale(prev_out, prev_recs_out, atomicAdd(&S.n_out, 1u), (uint32_t)S.rec[sl][F_ROW], S.rec[sl]);
            }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            prev_out[0] = n_own;
            prev_out[1] = S.n_out - n_own;
        }
    }
#ifdef MS_VSTAMPS
    MS_VST(5);
    if (lane == 0) {
        for (int i = 0; i < 9; ++i) atomicAdd(reinterpret_cast<u64 *>(stats + 8) + i, vst.acc[i]);
        for (int i = 9; i < 12; ++i) atomicAdd(reinterpret_cast<u64 *>(stats + 8) + i + 3, vst.acc[i]);
    }
#endif
}

// One step of the single-stream sequential engine: workgroup 0 validates
// batch k (one wave; the workgroup's LDS is the validator's, so it has a CU to
// itself) while the other workgroups sweep batch k+1 (a (tile, pod chunk)
// task per wave, k_sweep_full_topk's work). One launch per batch and no
// cross-stream hand-off: batch k+1's speculation may predate batch k's binds,
// which its validation treats as stale (prev lists). W waves per workgroup
// (launch_seq_step: 8 up to 256 tiles, MS_STEP_W4; the validator's VGPRs at
// one workgroup per CU).
// Batch k+1's in-step merge (SeqMergeIO, depth 1): n = 0 none.
struct StepMerge {
    u64 *top, *spec, *ext;
    uint32_t *spec_flags, *tags, *ctr;
    int64_t *recs;
    uint32_t tag, target, n, skip;
    const uint32_t *in_tags;  // batch k's tags (in_tag 0: merged by a launch, nothing to check)
    uint32_t in_tag;
    u64 *tl;                  // MS_VSTAMPS timeline (SeqMergeIO::tl): this step's row, or null
    uint32_t list_tag;        // MS_MERGE_TAGS: the 2-bit tag of this step's lists (SweepArgs::coh)
};

constexpr uint64_t kMergeSpinTicks = 10000;  // a worker's wait for the sweep, s_memrealtime (100 MHz): 100 us

// Worker wid (wave W-1 of every sweep workgroup first: idle in a 12-wave
// transposed sweep, which keeps 8 busy; with 8 waves it merges after its own
// pod group) merges pods wid, wid + W * nsw, ..
// of the next batch and tags each. MS_MERGE_TAGS: it polls the tagged lists
// themselves from the start of the step (merge_pod_lists); otherwise every
// sweep workgroup counts itself done on sm.ctr once its stores landed and the
// worker polls the counter first. Either wait is bounded (kMergeSpinTicks); a
// worker that gives up leaves its pods untagged and the next step's validation
// merges them (step_merge_fallback).
// MS_VSTAMPS (diagnostic build): the merge path's timeline relative to the
// workgroup's start (s_memrealtime, 10 ns), summed over worker waves at stats
// u64 [8+15] sweep done, [8+16] wait done, [8+17] merges done, [8+18] their
// count, [8+19] the workgroups' count (summed over workgroups).
template <int J, int W>
__device__ __forceinline__ void step_merge(const SweepArgs &sw, const StepMerge &sm, uint32_t sb, uint32_t nsw,
                                           uint32_t wave, uint32_t lane, uint32_t *stats, uint64_t t_begin) {
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
    const uint64_t t_swept = __builtin_amdgcn_s_memrealtime();
    (void)t_swept;
#endif
#if !MS_MERGE_TAGS
    __builtin_amdgcn_s_waitcnt(0);  // (gfx9: vmcnt covers stores) this wave's lists have landed
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(((gu32_t *)(sm.ctr)), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
#ifdef MS_VSTAMPS
        atomicAdd(reinterpret_cast<u64 *>(stats + 8) + 19, now - t_begin);
#endif
        if (sm.tl) sm.tl[blockIdx.x * 8 + kTlSwept] = now;
#endif
    }
#endif
    const uint32_t wid = (W - 1 - wave) * nsw + sb;
    if (wid >= sm.n || sm.skip) return;  // wave-uniform
    const uint64_t deadline = __builtin_amdgcn_s_memrealtime() + kMergeSpinTicks;
#if !MS_MERGE_TAGS
    for (;;) {
        const uint32_t v = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)__hip_atomic_load(((const gu32_t *)(sm.ctr)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if ((int32_t)(v - sm.target) >= 0) break;
        if (__builtin_amdgcn_s_memrealtime() > deadline) return;
        __builtin_amdgcn_s_sleep(1);
    }
    const uint32_t tag = 0;
#else
    const uint32_t tag = sm.list_tag;
#endif
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
    const uint64_t t_waited = __builtin_amdgcn_s_memrealtime();
    uint64_t t_poll = 0, t_rank = 0;  // the first pod's lists all arrived / its ranks merged
#define MS_TL_MERGE_STAMPS , p == wid ? &t_poll : nullptr, p == wid ? &t_rank : nullptr
#else
#define MS_TL_MERGE_STAMPS
#endif
    for (uint32_t p = wid; p < sm.n; p += W * nsw) {
        if (!merge_pod<J, true>(sw.tile_keys, sw.tile_flags, p, sw.n_tiles, sm.top, sm.spec, sm.spec_flags, sw.t,
                                sm.recs, sm.ext, lane, tag, deadline MS_TL_MERGE_STAMPS))
            return;  // (untagged: the next validation merges it)
#undef MS_TL_MERGE_STAMPS
        if (lane == 0) sm.tags[p] = sm.tag;
    }
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
    __builtin_amdgcn_s_waitcnt(0);
    if (lane == 0 && sm.tl) {
        sm.tl[blockIdx.x * 8 + kTlWaited] = t_waited;
        sm.tl[blockIdx.x * 8 + kTlSwept] = t_rank;  // (tagged lists: slot 1 holds the first pod's ranks merged)
        sm.tl[blockIdx.x * 8 + kTlValidated] = t_poll;  // (and slot 4 its lists' arrival)
        sm.tl[blockIdx.x * 8 + kTlMerged] = __builtin_amdgcn_s_memrealtime();
    }
#endif
#ifdef MS_VSTAMPS
    if (lane == 0) {
        u64 *st = reinterpret_cast<u64 *>(stats + 8);
        atomicAdd(st + 15, t_swept - t_begin);
        atomicAdd(st + 16, t_waited - t_begin);
        atomicAdd(st + 17, __builtin_amdgcn_s_memrealtime() - t_begin);
        atomicAdd(st + 18, 1ull);
    }
#else
    (void)stats;
    (void)t_begin;
#endif
}

// Validation k's check of its batch's in-step merge (workgroup 0, all W waves,
// before the prologue): pods whose worker gave up are merged here from the tile
// lists (written by the previous launch). Returns whether any was.
template <int J, int W>
__device__ __forceinline__ bool step_merge_fallback(const SeqArgs &va, const StepMerge &sm, bool any, uint32_t wave,
                                                    uint32_t lane) {
    if (!__syncthreads_or(any)) return false;
    for (uint32_t p = wave; p < va.n_pods; p += W)
        if (sm.in_tags[p] != sm.in_tag) {  // (wave-uniform)
            merge_pod<J>(va.tile_keys, va.tile_flags, p, va.n_tiles, const_cast<u64 *>(va.top4),
                         const_cast<u64 *>(va.spec), const_cast<uint32_t *>(va.spec_flags), va.t,
                         const_cast<int64_t *>(va.top4_recs), const_cast<u64 *>(va.top_ext), lane);
            if (lane == 0) atomicAdd(&va.stats[40], 1u);  // (u32 40: pods merged by the fallback)
        }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (no stale L1 lines of the merged entries)
    __syncthreads();
    return true;
}

template <int J, int W>
__global__ __launch_bounds__(64 * W) void k_seq_step(SeqArgs va, SweepArgs sw, uint32_t n_tasks, StepMerge sm) {
    // (the untagged-pod check below reads one tag per thread)
    static_assert(kSeqBatch <= 64 * W, "k_seq_step: one in-step merge tag per thread of the validating workgroup");
    __shared__ SeqShared S;
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)  // wave durations (s_memrealtime, 100 MHz): u64 stats[8+9] validator, [8+10] sweep waves, [8+11] their count
    const u64 t_begin = __builtin_amdgcn_s_memrealtime();
    if (sm.tl && threadIdx.x == 0 && blockIdx.x < kTimelineWgs) sm.tl[blockIdx.x * 8 + kTlBegin] = t_begin;
#endif
    if (blockIdx.x == 0) {
        // the prologue by all W waves (MS_WG_PROLOGUE=2: all of it; 1: the bulk copies,
        // the rest on the validating wave; 0: all on the validating wave, A/B)
#ifndef MS_WG_PROLOGUE
#define MS_WG_PROLOGUE 2
#endif
        // the tags of an in-step merged batch, loaded beside the prologue's loads
        const bool check = sm.in_tag != 0u && va.n_pods;
        uint32_t tg = sm.in_tag;
        if (check && threadIdx.x < va.n_pods) tg = sm.in_tags[threadIdx.x];
        if (MS_WG_PROLOGUE == 2 && va.n_pods) {
            ProRegs<W> R;
            prologue_wg_issue<W>(S, va, threadIdx.x, R);
            if (check && step_merge_fallback<J, W>(va, sm, tg != sm.in_tag, threadIdx.x >> 6, lane_id()))
                prologue_wg_issue<W>(S, va, threadIdx.x, R);  // again, with the merged entries
            __syncthreads();
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
            if (sm.tl && threadIdx.x == 0) sm.tl[kTlSwept] = __builtin_amdgcn_s_memrealtime();  // (bulk copies landed)
#endif
            prologue_wg_finish<W>(S, va, threadIdx.x, R);
        } else if (MS_WG_PROLOGUE && va.n_pods) {
            validate_prologue_wg(S, va, threadIdx.x, 64u * W);
            __builtin_amdgcn_s_waitcnt(0);
            if (check && step_merge_fallback<J, W>(va, sm, tg != sm.in_tag, threadIdx.x >> 6, lane_id())) {
                validate_prologue_wg(S, va, threadIdx.x, 64u * W);  // again, with the merged entries
                __builtin_amdgcn_s_waitcnt(0);
            }
            __syncthreads();
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
            if (sm.tl && threadIdx.x == 0) sm.tl[kTlSwept] = __builtin_amdgcn_s_memrealtime();  // (bulk copies landed)
#endif
        } else if (check) {
            step_merge_fallback<J, W>(va, sm, tg != sm.in_tag, threadIdx.x >> 6, lane_id());
        }
        if (threadIdx.x < 64 && va.n_pods) validate_batch<J>(S, va, threadIdx.x, MS_WG_PROLOGUE);
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
        if (threadIdx.x == 0 && va.n_pods) {
            const u64 now = __builtin_amdgcn_s_memrealtime();
#ifdef MS_VSTAMPS
            atomicAdd(reinterpret_cast<u64 *>(va.stats + 8) + 9, now - t_begin);
#endif
            if (sm.tl) sm.tl[kTlValidated] = now;
        }
#endif
        return;
    }
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    const uint32_t sb = blockIdx.x - 1, sg = gridDim.x - 1;  // sweep workgroup, count
    if (sw.t.drow && sw.fast) {  // transposed form: a tile per workgroup, its rows in the validator's (idle) LDS
        DRow *rows = reinterpret_cast<DRow *>(&S);
        // Groups outside the binary64 range are taken after the tile loop, listed
        // per wave in LDS past the staged rows: with the lane = row fallback
        // inline, its registers made the loop's invariants spill (28 B per lane,
        // 4.1 MB of scratch writes per config E step, a reload wait per tile).
        uint32_t *defer = reinterpret_cast<uint32_t *>(rows + kFullWaveTile) + wave * kTpDeferCap;
        uint32_t nd = 0;
        bool over = false;
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
        u64 *const tlw = (sm.tl && blockIdx.x < kTimelineWgs) ? sm.tl + blockIdx.x * 8 : nullptr;
#else
        u64 *const tlw = nullptr;
#endif
        for (uint32_t tile = sb; tile < sw.n_tiles; tile += sg) {
            const uint32_t r = sweep_tp_tile<W>(sw, tile, rows, wave, lane, tile == sb ? tlw : nullptr);  // (wave-uniform)
            if (r) {
                if (nd < kTpDeferCap) defer[nd++] = tile << 16 | r;
                else over = true;
            }
        }
        if (tlw && threadIdx.x == 0) tlw[kTlWave0] = __builtin_amdgcn_s_memrealtime();
        for (uint32_t i = 0; i < nd; ++i) sweep_tp_redo<W>(sw, defer[i] >> 16, defer[i] & 0xFFFFu, wave, lane);
        if (over) {  // (more deferred tiles than the list holds: every group of every tile, exactly)
            uint32_t all = 0;
            for (uint32_t grp = wave, i = 0; grp * kTpPods < sw.n_pods; grp += W, ++i) all |= 1u << i;
            for (uint32_t tile = sb; tile < sw.n_tiles; tile += sg) sweep_tp_redo<W>(sw, tile, all, wave, lane);
        }
        if (tlw && lane == 0)  // (diagnostic builds: the last wave's end, without a barrier that would hold the merging wave)
            atomicMax(reinterpret_cast<unsigned long long *>(tlw + kTlTasks),
                      (unsigned long long)__builtin_amdgcn_s_memrealtime());
    } else {
        for (uint32_t task = sb * W + wave; task < n_tasks; task += sg * W)
            sweep_topk_task(sw, task % sw.n_tiles, task / sw.n_tiles, lane);
    }
#if defined(MS_VSTAMPS) || defined(MS_TIMELINE_ONLY)
    if (sm.n) step_merge<J, W>(sw, sm, sb, sg, wave, lane, va.stats, t_begin);  // (workgroup-uniform)
#else
    if (sm.n) step_merge<J, W>(sw, sm, sb, sg, wave, lane, va.stats, 0);  // (workgroup-uniform)
#endif
#ifdef MS_VSTAMPS
    if (lane == 0 && sb * W + wave < n_tasks) {
        atomicAdd(reinterpret_cast<u64 *>(va.stats + 8) + 10, __builtin_amdgcn_s_memrealtime() - t_begin);
        atomicAdd(reinterpret_cast<u64 *>(va.stats + 8) + 11, 1ull);
    }
#endif
}

// ----------------------------------------------------------------------------
// Node-sharded exact sequential mode (minisched_gpu.h ms_seq_*): every shard
// publishes its speculative top-4 per pod with the nodes' records; after an
// all-gather every shard runs the same replicated in-order validation on the
// merged lists and commits the binds that land on its own nodes.
// ----------------------------------------------------------------------------
static_assert(sizeof(ms_seq_cand) == 72, "ms_seq_cand layout");

// One wave per pod: this shard's top-4 (k_topk_merge output) with records, and
// the OR over every tile of the shard of the filter flags (plugins rejecting
// at least one node: NU rejections are static and NRF ones only grow with
// binds, so the OR stays a valid part of the FitError mask later in the batch).
__global__ __launch_bounds__(64) void k_seq_pack_cands(NodeTable t, const u64 *__restrict__ top4,
                                                       const uint32_t *__restrict__ tile_flags, uint32_t n_tiles,
                                                       uint32_t n_pods, ms_seq_cand *__restrict__ cands,
                                                       uint32_t *__restrict__ flags) {
    const uint32_t p = blockIdx.x, lane = threadIdx.x;
    if (p >= n_pods) return;
    uint32_t fl = 0;
    for (uint32_t tt = lane; tt < n_tiles; tt += 64) fl |= untag_flags(tile_flags[(size_t)p * n_tiles + tt]);
    const uint32_t f = (__ballot((fl & 0xFFu) != 0) ? 1u : 0u) | (__ballot((fl & 0xFF00u) != 0) ? 0x100u : 0u);
    if (lane == 0) flags[p] = f;
    if (lane < (uint32_t)kTopK) {
        const u64 e = top4[(size_t)p * kTopK + lane];
        ms_seq_cand c = {};
        c.key = e;
        if (e) {
            const uint32_t r = row_of_key(e, t.base);
            c.alloc_milli_cpu = t.alloc_cpu[r];
            c.alloc_memory = t.alloc_mem[r];
            c.req_milli_cpu = t.req_cpu[r];
            c.req_memory = t.req_mem[r];
            c.nonzero_milli_cpu = t.nz_cpu[r];
            c.nonzero_memory = t.nz_mem[r];
            c.allowed_pods = t.allowed_pods[r];
            c.pod_count = t.pod_count[r];
            c.flags_digit = (uint32_t)t.flags[r] | ((uint32_t)t.digit[r] << 8);
        }
        cands[(size_t)p * kTopK + lane] = c;
    }
}

// One wave per pod: the global speculative top-4 from the shards' lists (the
// global rank-r entry, r < 4, is within its shard's top r+1), and the OR of
// the shards' flags.
__global__ __launch_bounds__(64) void k_seq_merge_shards(uint32_t n_pods, uint32_t n_shards,
                                                         const ms_seq_cand *__restrict__ cands_all,
                                                         const uint32_t *__restrict__ flags_all,
                                                         ms_seq_cand *__restrict__ merged,
                                                         uint32_t *__restrict__ merged_flags) {
    const uint32_t p = blockIdx.x, lane = threadIdx.x;
    if (p >= n_pods) return;
    const bool in = lane < n_shards * kTopK;
    const size_t src = (size_t)(lane / kTopK) * n_pods * kTopK + (size_t)p * kTopK + lane % kTopK;
    u64 k = in ? cands_all[src].key : 0ull;
    for (int r = 0; r < kTopK; ++r) {
        const u64 m = wave_max_u64_dpp(k);
        const u64 own = __ballot(m != 0 && k == m);  // keys embed the global ordinal: one owner
        const uint32_t ol = own ? (uint32_t)__builtin_ctzll(own) : 0u;
        if (own ? lane == ol : lane == 0) {
            ms_seq_cand c = {};
            if (own) c = cands_all[src];
            merged[(size_t)p * kTopK + r] = c;
        }
        if (own && lane == ol) k = 0;
    }
    uint32_t f = lane < n_shards ? flags_all[(size_t)lane * n_pods + p] : 0u;
    f = (__ballot((f & 0xFFu) != 0) ? 1u : 0u) | (__ballot((f & 0xFF00u) != 0) ? 0x100u : 0u);
    if (lane == 0) merged_flags[p] = f;
}

constexpr int kRepMapBits = 11;
constexpr int kRepMapCap = 1 << kRepMapBits;  // >= 2 x the nodes a batch binds (<= 256)

struct RepShared {
    ms_seq_cand c[MS_SEQ_SHARD_BATCH_MAX * kTopK];  // the merged candidates; a bound node's slot is its live record
    uint32_t map[kRepMapCap];                       // ((ordinal + 1) << 10) | slot; 0 = empty
    uint16_t bound_slot[MS_SEQ_SHARD_BATCH_MAX];    // live slots in bind order (write-back)
    uint32_t n_bound;
};
static_assert(sizeof(RepShared) <= 100 * 1024, "replicated validator LDS");

__device__ __forceinline__ uint32_t rep_hash(uint32_t ord) { return (ord * kGolden32) >> (32 - kRepMapBits); }

__device__ __forceinline__ int rep_find(const RepShared &S, uint32_t ord) {
    uint32_t h = rep_hash(ord);
    for (;;) {
        const uint32_t v = S.map[h];
        if (v == 0) return -1;
        if ((v >> 10) == ord + 1) return (int)(v & 1023u);
        h = (h + 1) & (kRepMapCap - 1);
    }
}

__device__ __forceinline__ FullRow cand_row(const ms_seq_cand &c) {
    return make_row(c.alloc_milli_cpu, c.alloc_memory, c.req_milli_cpu, c.req_memory, c.nonzero_milli_cpu,
                    c.nonzero_memory, c.allowed_pods - c.pod_count, c.flags_digit);
}

// The replicated in-order validation (one wave; identical on every shard).
// Lanes 0..3 take a pod's four merged candidates: entries bound earlier in the
// batch are re-evaluated from their live record, the first untouched one is
// exact and bounds everything below it (binds only lower the keys of the node
// they land on; unlisted nodes are below the 4th entry). A pod whose four
// entries are all touched while the list is full cannot be decided from the
// lists: the batch ends before it.
__global__ __launch_bounds__(64) void k_seq_validate_rep(NodeTable t, uint32_t n_pods,
                                                         const ms_pod_rec *__restrict__ pods, uint32_t seed32,
                                                         const ms_seq_cand *__restrict__ merged,
                                                         const uint32_t *__restrict__ merged_flags,
                                                         ms_result *__restrict__ results,
                                                         uint32_t *__restrict__ n_done,
                                                         const uint32_t *__restrict__ live) {
    __shared__ RepShared S;
    const uint32_t lane = threadIdx.x;
    if (live) n_pods = min(n_pods, *live);  // a cursor window: only its live pods are validated
    for (uint32_t i = lane; i < n_pods * kTopK; i += 64) S.c[i] = merged[i];
    for (uint32_t i = lane; i < (uint32_t)kRepMapCap; i += 64) S.map[i] = 0;
    if (lane == 0) S.n_bound = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    uint32_t p = 0;
    for (; p < n_pods; ++p) {
        const ms_pod_rec pr = pods[p];
        const PodFull q = load_pod(pr, seed32);
        const uint32_t slot = p * kTopK + (lane & 3u);
        const u64 e = lane < (uint32_t)kTopK ? S.c[slot].key : 0ull;
        const uint32_t ord = e ? 0xFFFFFu - (uint32_t)(e & 0xFFFFFu) : 0u;
        const int live = e ? rep_find(S, ord) : -1;
        const u64 untouched = __ballot(e != 0 && live < 0);
        const u64 listed = __ballot(e != 0);
        if (!untouched && __builtin_popcountll(listed) == kTopK) break;  // undecidable from the lists
        const uint32_t f = untouched ? (uint32_t)__builtin_ctzll(untouched) : (uint32_t)kTopK;
        u64 v = 0;
        if (lane < f && e != 0) {
            uint32_t nu, nrf;
            v = eval_full(cand_row(S.c[live]), ord, q, nu, nrf);
        } else if (lane == f) {
            v = e;
        }
        const u64 b = wave_max_u64_dpp(v);
        const u64 own = __ballot(b != 0 && v == b);
        ms_result r;
        r._pad = 0;
        r.plugin_mask = 0;
        if (b == 0) {  // FitError: nothing feasible at speculation, or every listed node bound full since
            const uint32_t fm = merged_flags[p] | (listed ? 0x100u : 0u);
            r.code = MS_CODE_UNSCHEDULABLE;
            r.node = -1;
            r.score = 0;
            r.plugin_mask = ((fm & 0xFFu) ? MS_MASK_NODE_UNSCHEDULABLE : 0u) |
                            ((fm & 0xFF00u) ? MS_MASK_NODE_RESOURCES_FIT : 0u);
        } else if (pr.name_digit < 0) {
            r.code = MS_CODE_ERROR;  // NodeNumber.Score fails (nodenumber.go:74-77); nothing binds
            r.node = -1;
            r.score = 0;
        } else {
            r.code = MS_CODE_SUCCESS;
            r.node = (int32_t)(0xFFFFFu - (uint32_t)(b & 0xFFFFFu));
            r.score = (int64_t)(b >> 52);
            // assume-on-select: NodeInfo.AddPod on the winner's live record
            const uint32_t wl = (uint32_t)__builtin_ctzll(own);
            const int wlive = __builtin_amdgcn_readlane(live, (int)wl);
            if (lane == 0) {
                int sl = wlive;
                if (sl < 0) {  // first bind on this node in the batch: its candidate slot becomes live
                    sl = (int)(p * kTopK + wl);
                    uint32_t h = rep_hash((uint32_t)r.node);
                    while (S.map[h] != 0) h = (h + 1) & (kRepMapCap - 1);
                    S.map[h] = (((uint32_t)r.node + 1) << 10) | (uint32_t)sl;
                    S.bound_slot[S.n_bound++] = (uint16_t)sl;
                }
                ms_seq_cand &c = S.c[sl];
                c.req_milli_cpu += pr.req_milli_cpu;
                c.req_memory += pr.req_memory;
                c.nonzero_milli_cpu += pr.nonzero_milli_cpu;
                c.nonzero_memory += pr.nonzero_memory;
                c.pod_count += 1;
            }
        }
        if (lane == 0) results[p] = r;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
    }
    // this shard's own bound nodes go back to its table (absolute values: the
    // candidates were read from this table and nothing else wrote it since)
    const uint32_t nb = S.n_bound;
    for (uint32_t i = lane; i < nb; i += 64) {
        const ms_seq_cand &c = S.c[S.bound_slot[i]];
        const uint32_t ord = 0xFFFFFu - (uint32_t)(c.key & 0xFFFFFu);
        if (ord < t.base || ord - t.base >= t.cap) continue;  // another shard's node
        const uint32_t row = ord - t.base;
        t.req_cpu[row] = c.req_milli_cpu;
        t.req_mem[row] = c.req_memory;
        t.nz_cpu[row] = c.nonzero_milli_cpu;
        t.nz_mem[row] = c.nonzero_memory;
        t.pod_count[row] = c.pod_count;
    }
    if (lane == 0) *n_done = p;
}

// ----------------------------------------------------------------------------
// decode / bind commit / deltas
// ----------------------------------------------------------------------------
__device__ __forceinline__ void decode_one(const ms_pod_rec *__restrict__ pods, const u64 *__restrict__ keys,
                                           const uint32_t *__restrict__ flags, uint32_t present,
                                           ms_result *__restrict__ out, uint32_t i) {
    out[i] = decode_key(keys[i], pods[i].name_digit, flags, i, present);
}

// present_dev (optional): the present count as the node-sharded combine left
// it on the device (non-zero iff some shard lists a node), instead of present.
__global__ void k_decode(const ms_pod_rec *__restrict__ pods, uint32_t n_pods, const u64 *__restrict__ keys,
                         const uint32_t *__restrict__ flags, uint32_t present, const uint32_t *__restrict__ present_dev,
                         ms_result *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_pods) decode_one(pods, keys, flags, present_dev ? *present_dev : present, out, i);
}

// Several batches' decodes in one launch (grid.y = job): the grouped drain of
// the pipelined multi-GPU step decodes its batches together.
struct DecodeJobs {
    ms_decode_job j[MS_DECODE_MAX_JOBS];
};

__global__ void k_decode_jobs(DecodeJobs jobs, uint32_t present) {
    const ms_decode_job &jb = jobs.j[blockIdx.y];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < jb.n_pods)
        decode_one(jb.pods, reinterpret_cast<const u64 *>(jb.keys), jb.flags, present, jb.results, i);
}

// The in-library node-sharded drain: several batches' pod slices, each with
// its own device-side present flag (ms_comm.cpp).
struct SliceJobs {
    SliceJob j[kMaxSliceJobs];
};

__global__ void k_decode_slices(SliceJobs jobs) {
    const SliceJob &jb = jobs.j[blockIdx.y];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < jb.n_pods) decode_one(jb.pods, jb.keys, jb.flags, jb.present ? *jb.present : 0u, jb.results, i);
}

// Node-sharded exact sequential with a device-side queue cursor (ms_comm.cpp):
// ctl[0] = next pod of the queue, ctl[1] = live pods of the current window,
// ctl[2] = pods the window's validation decided (k_seq_validate_rep n_done).
// window_in copies pods [cursor, cursor + live) into the fixed window (zeroes
// the rest: those entries are swept but never validated); window_out copies
// the decided results back to the queue order and advances the cursor, so the
// host issues batches without reading n_done.
__global__ void k_seq_window_in(const ms_pod_rec *__restrict__ pods, uint32_t n, uint32_t *__restrict__ ctl,
                                ms_pod_rec *__restrict__ win, uint32_t w) {
    const uint32_t cur = min(ctl[0], n);
    const uint32_t live = min(w, n - cur);
    for (uint32_t i = threadIdx.x; i < w; i += blockDim.x) {
        // 8-byte words (a struct select put the record on the stack)
        const uint2 *src = reinterpret_cast<const uint2 *>(pods + cur + min(i, live ? live - 1u : 0u));
        uint2 *dst = reinterpret_cast<uint2 *>(win + i);
#pragma unroll
        for (int k = 0; k < (int)(sizeof(ms_pod_rec) / 8); ++k) dst[k] = i < live ? src[k] : make_uint2(0u, 0u);
    }
    if (threadIdx.x == 0) ctl[1] = live;
}

__global__ void k_seq_window_out(const ms_result *__restrict__ win_res, uint32_t *__restrict__ ctl,
                                 ms_result *__restrict__ res, uint32_t n) {
    const uint32_t cur = min(ctl[0], n);
    const uint32_t done = min(ctl[2], n - cur);
    for (uint32_t i = threadIdx.x; i < done; i += blockDim.x) res[cur + i] = win_res[i];
    __syncthreads();  // every thread read ctl[0] before it moves
    if (threadIdx.x == 0) ctl[0] = cur + done;
}

__global__ void k_fill_keys(u64 *__restrict__ keys, uint32_t n, u64 v) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keys[i] = v;
}

__global__ void k_pods_widen(const ms_pod_compact *__restrict__ in, uint32_t n, ms_pod_rec *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint2 v = *reinterpret_cast<const uint2 *>(in + i);  // = the first 8 bytes of ms_pod_rec
    uint2 *o = reinterpret_cast<uint2 *>(out + i);
    o[0] = v;
    o[1] = o[2] = o[3] = o[4] = make_uint2(0u, 0u);
}

__global__ void k_results_narrow(const ms_result *__restrict__ in, uint32_t n, ms_result_compact *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ms_result r = in[i];
    ms_result_compact c;
    c.node = r.node;
    c.score = (uint16_t)r.score;
    c.code = (uint8_t)r.code;
    c.plugin_mask = (uint8_t)r.plugin_mask;
    out[i] = c;
}

__global__ void k_apply_binds(NodeTable t, const ms_pod_rec *__restrict__ pods, uint32_t n_pods,
                              const ms_result *__restrict__ res) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pods) return;
    const ms_result r = res[i];
    if (r.code != MS_CODE_SUCCESS || r.node < 0) return;
    const uint32_t node = (uint32_t)r.node;
    if (node < t.base || node - t.base >= t.cap) return;  // another shard owns it
    add_pod(t, node - t.base, pods[i], +1);
}

__global__ void k_bind_one(NodeTable t, uint32_t row, const ms_pod_rec *pod, int sign) {
    if (threadIdx.x == 0 && blockIdx.x == 0) add_pod(t, row, *pod, sign);
}

__global__ void k_apply_deltas(NodeTable t, const NodeDelta *__restrict__ d, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const NodeDelta x = d[i];
    const uint32_t r = x.local;
    if (x.absent) {
        t.flags[r] = kNodeAbsent;
        t.digit[r] = 0xFF;
        t.zone[r] = 0;
        t.label2[r] = 0;
        t.taints[r] = 0;
        t.allowed_pods[r] = 0;
        t.pod_count[r] = 0;
        t.alloc_cpu[r] = t.alloc_mem[r] = 0;
        t.req_cpu[r] = t.req_mem[r] = 0;
        t.nz_cpu[r] = t.nz_mem[r] = 0;
        return;
    }
    t.flags[r] = x.rec.unschedulable ? kNodeUnschedulable : 0;
    t.digit[r] = x.rec.name_digit <= 9 ? x.rec.name_digit : 0xFF;
    t.zone[r] = x.rec.zone;
    t.label2[r] = x.rec.label2;
    t.taints[r] = x.rec.taints & 0xFFFFu;
    t.allowed_pods[r] = x.rec.allowed_pods;
    t.pod_count[r] = x.rec.pod_count;
    t.alloc_cpu[r] = x.rec.alloc_milli_cpu;
    t.alloc_mem[r] = x.rec.alloc_memory;
    t.req_cpu[r] = x.rec.req_milli_cpu;
    t.req_mem[r] = x.rec.req_memory;
    t.nz_cpu[r] = x.rec.nonzero_milli_cpu;
    t.nz_mem[r] = x.rec.nonzero_memory;
}

__global__ void k_init_table(NodeTable t) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= t.cap) return;
    t.flags[r] = kNodeAbsent;
    t.digit[r] = 0xFF;
    t.zone[r] = 0;
    t.label2[r] = 0;
    t.taints[r] = 0;
    t.allowed_pods[r] = 0;
    t.pod_count[r] = 0;
    t.alloc_cpu[r] = t.alloc_mem[r] = 0;
    t.req_cpu[r] = t.req_mem[r] = 0;
    t.nz_cpu[r] = t.nz_mem[r] = 0;
}

__global__ void k_read_rows(NodeTable t, uint32_t first, uint32_t n, ms_node_rec *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = first + i;
    ms_node_rec x = {};
    const uint8_t f = t.flags[r];
    x.unschedulable = (f & kNodeUnschedulable) ? 1 : 0;
    x.name_digit = t.digit[r];
    x.zone = t.zone[r];
    x.label2 = t.label2[r];
    x.taints = t.taints[r];
    x.allowed_pods = (f & kNodeAbsent) ? -1 : t.allowed_pods[r];
    x.pod_count = t.pod_count[r];
    x.alloc_milli_cpu = t.alloc_cpu[r];
    x.alloc_memory = t.alloc_mem[r];
    x.req_milli_cpu = t.req_cpu[r];
    x.req_memory = t.req_mem[r];
    x.nonzero_milli_cpu = t.nz_cpu[r];
    x.nonzero_memory = t.nz_mem[r];
    out[i] = x;
}

// ----------------------------------------------------------------------------
// MS_PLUGINS_NU_NN_NA: Filter[NU]; Score[NodeNumber, NodeAffinity preferred term]
// with NodeAffinity's DefaultNormalizeScore(100, reverse=false) run by
// RunScorePlugins after every node on the whole, partially filled list
// (minisched.go:164-185). For raw scores <= 100 that in-loop hook leaves every
// entry at its raw score except the first feasible node in LIST order with a
// non-zero raw score (the anchor), which ends at 100: after the first non-zero
// entry the list maximum is 100 and every later normalisation is the
// identity (oracle/ms_oracle.c msor_schedule_na checks the closed form against
// the loop as written). So per pod the sweep keeps (a) the max packed key with
// raw NodeAffinity scores and (b) the anchor as a min-ordinal reduction; the
// decode takes max(a, key of the anchor scored w_nn*NN + w_na*100). The
// anchor's raw key never beats its boosted key, so including it in (a) is
// harmless. One pair per lane-slot, plain per-pair evaluation.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(kNunnThreads) void k_sweep_na(
    const uint8_t *__restrict__ nflags, const uint8_t *__restrict__ ndigit, const uint8_t *__restrict__ nzone,
    uint32_t n_rows, uint32_t node_base, const ms_pod_rec *__restrict__ pods, uint32_t n_pods, uint32_t chunk,
    uint32_t seed32, uint32_t w_nn, uint32_t w_na, u64 *__restrict__ keys, uint32_t *__restrict__ fkeys) {
    const uint32_t row0 = blockIdx.x * kNunnTile + threadIdx.x * kNunnSlots;
    uint8_t fl[kNunnSlots], dg[kNunnSlots], zn[kNunnSlots];
#pragma unroll
    for (int i = 0; i < kNunnSlots; ++i) {
        const uint32_t r = row0 + i;
        fl[i] = r < n_rows ? nflags[r] : kNodeAbsent;
        dg[i] = r < n_rows ? ndigit[r] : 0xFF;
        zn[i] = r < n_rows ? nzone[r] : 0;
    }
    const uint32_t pbeg = blockIdx.y * chunk;
    const uint32_t pend = min(n_pods, pbeg + chunk);
    for (uint32_t p = pbeg; p < pend; ++p) {
        const ms_pod_rec pr = pods[p];  // wave-uniform
        const uint32_t A = tb_pod(seed32, pr.ordinal);
        u64 best = 0;
        uint32_t anchor = 0;
#pragma unroll
        for (int i = 0; i < kNunnSlots; ++i) {
            const bool feas = !(fl[i] & kNodeAbsent) && !((fl[i] & kNodeUnschedulable) && !pr.tolerates_unschedulable);
            const uint32_t ord = node_base + row0 + i;
            const uint32_t nn = ((int)dg[i] == (int)pr.name_digit) ? 1u : 0u;
            const uint32_t raw = (pr.pref_zone != 0 && zn[i] == pr.pref_zone) ? pr.pref_weight : 0u;
            const u64 key = make_key(w_nn * 10u * nn + w_na * raw, tb_hash(A, ord), ord);
            best = feas ? umax64(best, key) : best;
            const uint32_t a = (((0xFFFFFu - ord) << 1) | nn) + 1u;
            anchor = (feas && raw) ? max(anchor, a) : anchor;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            best = umax64(best, __shfl_xor(best, off, 64));
            anchor = max(anchor, (uint32_t)__shfl_xor(anchor, off, 64));
        }
        if ((threadIdx.x & 63u) == 0u) {
            if (best) atomicMax(&keys[p], best);
            if (anchor) atomicMax(&fkeys[p], anchor);
        }
    }
}

__global__ void k_decode_na(const ms_pod_rec *__restrict__ pods, uint32_t n_pods, const u64 *__restrict__ keys,
                            const uint32_t *__restrict__ fkeys, uint32_t present, const uint32_t *__restrict__ present_dev,
                            uint32_t seed32, uint32_t w_nn, uint32_t w_na, ms_result *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pods) return;
    u64 k = keys[i];
    const uint32_t a = fkeys[i];
    if (a) {  // the normalise anchor, scored w_nn * NN + w_na * 100
        const uint32_t ord = 0xFFFFFu - ((a - 1u) >> 1), nn = (a - 1u) & 1u;
        k = umax64(k, make_key(w_nn * 10u * nn + w_na * 100u, tb_hash(tb_pod(seed32, pods[i].ordinal), ord), ord));
    }
    out[i] = decode_key(k, pods[i].name_digit, nullptr, 0, present_dev ? *present_dev : present);
}

inline uint32_t cdiv(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

// pods per chunk: enough blocks to fill the chip twice over, multiple of 64
inline uint32_t pod_chunk(uint32_t n_pods, uint32_t node_blocks, int num_cus) {
    const uint32_t target = (uint32_t)(num_cus > 0 ? num_cus : 256) * 8u * 2u;
    uint32_t chunks = cdiv(target, node_blocks > 0 ? node_blocks : 1);
    chunks = chunks < 1 ? 1 : chunks;
    const uint32_t max_chunks = cdiv(n_pods, 64);
    if (chunks > max_chunks) chunks = max_chunks;
    uint32_t c = cdiv(n_pods, chunks);
    return cdiv(c, 64) * 64;
}

}  // namespace


hipError_t launch_sweep_na(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                           uint32_t seed32, uint32_t w_nn, uint32_t w_na, unsigned long long *keys, uint32_t *fkeys,
                           int num_cus, hipStream_t s) {
    if (n_pods == 0 || n_rows == 0) return hipSuccess;
    const uint32_t gx = cdiv(n_rows, kNunnTile);
    const uint32_t chunk = pod_chunk(n_pods, gx, num_cus);
    hipLaunchKernelGGL(k_sweep_na, dim3(gx, cdiv(n_pods, chunk)), dim3(kNunnThreads), 0, s, t.flags, t.digit, t.zone,
                       n_rows, t.base, pods, n_pods, chunk, seed32, w_nn, w_na, keys, fkeys);
    return hipGetLastError();
}

hipError_t launch_decode_na(const ms_pod_rec *pods, uint32_t n_pods, const unsigned long long *keys,
                            const uint32_t *fkeys, uint32_t present_nodes, uint32_t seed32, uint32_t w_nn,
                            uint32_t w_na, ms_result *out, hipStream_t s, const uint32_t *present_dev) {
    if (n_pods == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_na, dim3(cdiv(n_pods, 256)), dim3(256), 0, s, pods, n_pods, keys, fkeys,
                       present_nodes, present_dev, seed32, w_nn, w_na, out);
    return hipGetLastError();
}

hipError_t launch_sweep_full(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                             uint32_t seed32, unsigned long long *keys, uint32_t *flags, int num_cus,
                             hipStream_t s) {
    if (n_pods == 0 || n_rows == 0) return hipSuccess;
    const uint32_t gx = cdiv(n_rows, kFullTile);
    const uint32_t chunk = pod_chunk(n_pods, gx, num_cus);
    const dim3 grid(gx, cdiv(n_pods, chunk));
    hipLaunchKernelGGL(k_sweep_full, grid, dim3(kFullThreads), 0, s, t, n_rows, pods, n_pods, chunk, seed32, keys,
                       flags);
    return hipGetLastError();
}

// The config-E sweep's binary64 LeastAllocated form (default on; MINISCHED_SEQ_FAST=0
// keeps the general form everywhere, for A/B runs and parity cross-checks).
static uint32_t seq_fast() {
    const char *e = getenv("MINISCHED_SEQ_FAST");
    return (e && e[0] == '0') ? 0u : 1u;
}

hipError_t launch_sweep_full_tiles(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods,
                                   uint32_t n_pods, uint32_t seed32, unsigned long long *tile_keys,
                                   uint32_t *tile_flags, uint32_t n_tiles, hipStream_t s) {
    if (n_pods == 0 || n_rows == 0) return hipSuccess;
    if (n_tiles != cdiv(n_rows, tile_rows_of(t))) return hipErrorInvalidValue;
    const uint32_t gx = cdiv(n_tiles, kFullThreads / 64);
    const uint32_t chunk = 8;  // pods per wave: node rows amortised against enough waves to fill the chip
    if (t.drow && seq_fast()) {  // transposed form: one workgroup per tile
        const SweepArgs a = {t, n_rows, pods, n_pods, kTpPods, seed32, tile_keys, tile_flags, n_tiles, 1u};
        hipLaunchKernelGGL(k_sweep_tp_topk, dim3(n_tiles), dim3(64 * kTpWaves), 0, s, a);
        return hipGetLastError();
    }
    const dim3 grid(gx, cdiv(n_pods, chunk));
    const SweepArgs a = {t, n_rows, pods, n_pods, chunk, seed32, tile_keys, tile_flags, n_tiles, seq_fast()};
    hipLaunchKernelGGL(k_sweep_full_topk, grid, dim3(kFullThreads), 0, s, a);
    return hipGetLastError();
}

// In-step merge (SeqMergeIO): the transposed sweep, a tile per workgroup, all
// of them resident (one per CU beside the validator's).
bool seq_step_merges(const NodeTable &t, uint32_t n_tiles, uint32_t n_next) {
    return n_next && t.drow && seq_fast() && n_tiles <= 64u * kSeqMaxJ;
}

hipError_t launch_seq_step(const NodeTable &t, uint32_t n_rows, uint32_t n_tiles, uint32_t seed32,
                           const ms_pod_rec *pods, uint32_t n_pods, const unsigned long long *tile_keys,
                           const uint32_t *tile_flags, const unsigned long long *spec, const uint32_t *spec_flags,
                           const unsigned long long *top4, const int64_t *top4_recs, const uint32_t *prev_in,
                           const int64_t *prev_recs_in, uint32_t *prev_out, int64_t *prev_recs_out,
                           ms_result *results, uint32_t *stats, const ms_pod_rec *next_pods, uint32_t n_next,
                           unsigned long long *next_tile_keys, uint32_t *next_tile_flags, int num_cus,
                           hipStream_t s, const unsigned long long *top_ext, SeqMergeIO *mio) {
    if (n_pods == 0 && n_next == 0) return hipSuccess;
    if (n_pods > (uint32_t)kSeqBatch || n_tiles > 64u * kSeqMaxJ || n_tiles != cdiv(n_rows, tile_rows_of(t)) ||
        (n_pods && (!top4_recs || (prev_in && !prev_recs_in) || (prev_out && !prev_recs_out))))
        return hipErrorInvalidValue;
    SeqArgs va = {t,        n_rows,       pods,    n_pods,     seed32, tile_keys, tile_flags,
                        spec,     spec_flags,   top4,    top4_recs,  top_ext, n_tiles, prev_in, prev_recs_in,
                        prev_out, prev_recs_out, 0,      results,    stats};
    // tasks: (tile, chunk of next pods) pairs, sized to fit one pass of the
    // sweep workgroups (one per CU beside the validator's)
    const uint32_t cus = (uint32_t)(num_cus > 1 ? num_cus : 256);
    const int J = n_tiles <= 64 ? 1 : n_tiles <= 128 ? 2 : n_tiles <= 256 ? 4 : n_tiles <= 512 ? 8 : 16;
#ifndef MS_STEP_W4
// Waves per workgroup for n_tiles <= 256 (J <= 4). 8 (round 6): with tiles sized to the
// CUs (t.tile_rows) the 12-wave form's 168 VGPRs spilled 121 in the merge; 8
// waves (the transposed sweep's busy ones, the 8th merging after its sweep)
// take 238 without spilling: config E 31.13 -> 30.3 ms with 208-row tiles,
// 31.3 with 256 (profiles/r06q_e_tiles_ab.txt).
#define MS_STEP_W4 8
#endif
    const uint32_t W = J <= 4 ? (uint32_t)MS_STEP_W4 : J == 8 ? 8u : 4u;
    uint32_t chunk = 8;
    if (n_next) chunk = std::min(64u, std::max(8u, cdiv(n_tiles * n_next, (cus - 1) * W)));
    const bool tp = t.drow && seq_fast();
    if (tp) chunk = kTpPods;  // transposed form: a tile per sweep workgroup
    SweepArgs sw = {t,       n_rows,         next_pods,       n_next,  chunk,
                    seed32,  next_tile_keys, next_tile_flags, n_tiles, seq_fast(), 0u};
    const uint32_t n_tasks = n_next ? n_tiles * cdiv(n_next, chunk) : 0u;
    const uint32_t room = cus > 1u ? cus - 1u : 1u;
    const uint32_t grid = 1u + (n_tasks ? std::min(room, tp ? n_tiles : cdiv(n_tasks, W)) : 0u);
    StepMerge sm = {};
    if (mio) {
        sm.in_tags = mio->in_tags;
        sm.in_tag = mio->in_tags ? mio->in_tag : 0u;
        if (mio->top && n_next && seq_step_merges(t, n_tiles, n_next)) {
            if (!mio->tags || !mio->ctr || !mio->spec || !mio->spec_flags) return hipErrorInvalidValue;
            mio->target += grid - 1u;  // every sweep workgroup counts once
            sm.top = mio->top;
            sm.spec = mio->spec;
            sm.ext = mio->ext;
            sm.spec_flags = mio->spec_flags;
            sm.tags = mio->tags;
            sm.ctr = mio->ctr;
            sm.recs = mio->recs;
            sm.tag = mio->tag;
            sm.target = mio->target;
            sm.n = n_next;
            sm.skip = mio->skip ? 1u : 0u;
            // the lists' tag: 1..3 over consecutive steps, so a list set (rewritten every
            // second step, zeroed at the start of a run) never holds the tag it waits for
            sm.list_tag = 1u + mio->tag % 3u;
            sw.coh = sm.list_tag;
        } else if (mio->top) {
            return hipErrorInvalidValue;  // (the caller asked for an in-step merge seq_step_merges rules out)
        }
        if (mio->tl && mio->tl_step < kTimelineSteps && grid <= kTimelineWgs)
            sm.tl = reinterpret_cast<u64 *>(mio->tl) + (size_t)mio->tl_step * kTimelineWgs * 8;
    }
    va.tl = sm.tl;
#define MS_STEP(JJ, WW) \
    hipLaunchKernelGGL((k_seq_step<JJ, WW>), dim3(grid), dim3(64 * WW), 0, s, va, sw, n_tasks, sm)
    if (J == 1) MS_STEP(1, MS_STEP_W4);  // (12 waves spilled 119 VGPRs here too)
    else if (J == 2) MS_STEP(2, MS_STEP_W4);
    else if (J == 4) MS_STEP(4, MS_STEP_W4);
    else if (J == 8) MS_STEP(8, 8);
    else MS_STEP(16, 4);
#undef MS_STEP
    return hipGetLastError();
}

hipError_t launch_topk_merge(const unsigned long long *tile_keys, const uint32_t *tile_flags, uint32_t n_pods,
                             uint32_t n_tiles, unsigned long long *top, unsigned long long *spec, uint32_t *spec_flags,
                             const NodeTable &t, int64_t *recs, hipStream_t s, unsigned long long *ext) {
    if (n_pods == 0 || n_tiles == 0) return hipSuccess;
    if (n_tiles > 64u * kSeqMaxJ) return hipErrorInvalidValue;
#define MS_MERGE(J)                                                                                           \
    hipLaunchKernelGGL(k_topk_merge<J>, dim3(n_pods), dim3(64), 0, s, tile_keys, tile_flags, n_pods, n_tiles, top, \
                       spec, spec_flags, t, recs, ext)
    if (n_tiles <= 64) MS_MERGE(1);
    else if (n_tiles <= 128) MS_MERGE(2);
    else if (n_tiles <= 256) MS_MERGE(4);
    else if (n_tiles <= 512) MS_MERGE(8);
    else MS_MERGE(16);
#undef MS_MERGE
    return hipGetLastError();
}

hipError_t launch_build_drows(const NodeTable &t, uint32_t n_rows, uint32_t n_total, hipStream_t s) {
    if (!t.drow || n_total == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_build_drows, dim3(cdiv(n_total, 256)), dim3(256), 0, s, t, n_rows, n_total);
    return hipGetLastError();
}

uint32_t seq_max_rows() { return 64u * kSeqMaxJ * kFullWaveTile; }

hipError_t launch_decode(const ms_pod_rec *pods, uint32_t n_pods, const unsigned long long *keys,
                         const uint32_t *flags, uint32_t present_nodes, ms_result *out, hipStream_t s,
                         const uint32_t *present_dev) {
    if (n_pods == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode, dim3(cdiv(n_pods, 256)), dim3(256), 0, s, pods, n_pods, keys, flags,
                       present_nodes, present_dev, out);
    return hipGetLastError();
}

hipError_t launch_decode_slices(const SliceJob *jobs, uint32_t n_jobs, hipStream_t s) {
    if (n_jobs == 0 || n_jobs > kMaxSliceJobs) return n_jobs ? hipErrorInvalidValue : hipSuccess;
    SliceJobs sj = {};
    uint32_t most = 0;
    for (uint32_t i = 0; i < n_jobs; ++i) {
        sj.j[i] = jobs[i];
        most = std::max(most, jobs[i].n_pods);
    }
    if (most == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_slices, dim3(cdiv(most, 256), n_jobs), dim3(256), 0, s, sj);
    return hipGetLastError();
}

hipError_t launch_seq_window_in(const ms_pod_rec *pods, uint32_t n, uint32_t *ctl, ms_pod_rec *win, uint32_t w,
                                hipStream_t s) {
    hipLaunchKernelGGL(k_seq_window_in, dim3(1), dim3(256), 0, s, pods, n, ctl, win, w);
    return hipGetLastError();
}

hipError_t launch_seq_window_out(const ms_result *win_res, uint32_t *ctl, ms_result *res, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_seq_window_out, dim3(1), dim3(256), 0, s, win_res, ctl, res, n);
    return hipGetLastError();
}

hipError_t launch_decode_jobs(const ms_decode_job *jobs, uint32_t n_jobs, uint32_t present_nodes, hipStream_t s) {
    DecodeJobs dj = {};
    uint32_t most = 0;
    for (uint32_t i = 0; i < n_jobs; ++i) {
        dj.j[i] = jobs[i];
        most = std::max(most, jobs[i].n_pods);
    }
    if (most == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_jobs, dim3(cdiv(most, 256), n_jobs), dim3(256), 0, s, dj, present_nodes);
    return hipGetLastError();
}

hipError_t launch_apply_binds(const NodeTable &t, const ms_pod_rec *pods, uint32_t n_pods, const ms_result *res,
                              hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    hipLaunchKernelGGL(k_apply_binds, dim3(cdiv(n_pods, 256)), dim3(256), 0, s, t, pods, n_pods, res);
    return hipGetLastError();
}

hipError_t launch_fill_keys(unsigned long long *keys, uint32_t n, unsigned long long v, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill_keys, dim3(cdiv(n, 256)), dim3(256), 0, s, reinterpret_cast<u64 *>(keys), n, (u64)v);
    return hipGetLastError();
}

hipError_t launch_pods_widen(const ms_pod_compact *in, uint32_t n, ms_pod_rec *out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pods_widen, dim3(cdiv(n, 256)), dim3(256), 0, s, in, n, out);
    return hipGetLastError();
}

hipError_t launch_results_narrow(const ms_result *in, uint32_t n, ms_result_compact *out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_results_narrow, dim3(cdiv(n, 256)), dim3(256), 0, s, in, n, out);
    return hipGetLastError();
}

hipError_t launch_bind_one(const NodeTable &t, uint32_t local, const ms_pod_rec *pod_dev, int sign,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_bind_one, dim3(1), dim3(64), 0, s, t, local, pod_dev, sign);
    return hipGetLastError();
}

hipError_t launch_apply_deltas(const NodeTable &t, const NodeDelta *d_deltas, uint32_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_apply_deltas, dim3(cdiv(n, 256)), dim3(256), 0, s, t, d_deltas, n);
    return hipGetLastError();
}

hipError_t launch_init_table(const NodeTable &t, hipStream_t s) {
    if (t.cap == 0) return hipSuccess;
    hipLaunchKernelGGL(k_init_table, dim3(cdiv(t.cap, 256)), dim3(256), 0, s, t);
    return hipGetLastError();
}

hipError_t launch_read_rows(const NodeTable &t, uint32_t first, uint32_t n, ms_node_rec *out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_read_rows, dim3(cdiv(n, 256)), dim3(256), 0, s, t, first, n, out);
    return hipGetLastError();
}

hipError_t launch_seq_pack_cands(const NodeTable &t, const unsigned long long *top4, const uint32_t *tile_flags,
                                 uint32_t n_tiles, uint32_t n_pods, ms_seq_cand *cands, uint32_t *flags, hipStream_t s) {
    if (n_pods == 0) return hipSuccess;
    hipLaunchKernelGGL(k_seq_pack_cands, dim3(n_pods), dim3(64), 0, s, t, top4, tile_flags, n_tiles, n_pods, cands,
                       flags);
    return hipGetLastError();
}

hipError_t launch_seq_validate_rep(const NodeTable &t, uint32_t n_pods, const ms_pod_rec *pods, uint32_t seed32,
                                   uint32_t n_shards, const ms_seq_cand *cands_all, const uint32_t *flags_all,
                                   ms_seq_cand *merged, uint32_t *merged_flags, ms_result *results, uint32_t *n_done,
                                   hipStream_t s, const uint32_t *live) {
    if (n_pods == 0) return hipSuccess;
    if (n_pods > MS_SEQ_SHARD_BATCH_MAX || n_shards == 0 || n_shards > MS_SEQ_MAX_SHARDS) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_seq_merge_shards, dim3(n_pods), dim3(64), 0, s, n_pods, n_shards, cands_all, flags_all, merged,
                       merged_flags);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_seq_validate_rep, dim3(1), dim3(64), 0, s, t, n_pods, pods, seed32, merged, merged_flags,
                       results, n_done, live);
    return hipGetLastError();
}

uint32_t seq_batch_limit() { return (uint32_t)kSeqBatch; }
uint32_t seq_rec_fields() { return (uint32_t)kRecF; }
uint32_t seq_prev_cap() { return (uint32_t)kPrevCap; }
uint32_t seq_topk() { return (uint32_t)kTopK; }

}  // namespace msgpu
