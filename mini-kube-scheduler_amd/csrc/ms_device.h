// ms_device.h — device helpers shared by the kernel translation units
// (ms_kernels.hip, ms_sweep_pp.hip). Not part of the public boundary.
#pragma once

#include "ms_internal.h"

namespace msgpu {

typedef unsigned long long u64;

__device__ __forceinline__ u64 umax64(u64 a, u64 b) { return a > b ? a : b; }

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// packed key (minisched_gpu.h): score<<52 | h<<20 | (0xFFFFF - ordinal)
__device__ __forceinline__ u64 make_key(uint32_t score, uint32_t h, uint32_t ord) {
    const uint32_t hi = (score << 20) | (h >> 12);
    const uint32_t lo = (h << 20) | (0xFFFFFu - ord);
    return ((u64)hi << 32) | lo;
}

// Full 64-lane sum (the same row_shr / row_bcast scan as wave_max_u32_dpp; an
// out-of-row source reads 0, the identity); wave-uniform result from lane 63.
__device__ __forceinline__ uint32_t wave_sum_u32_dpp(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Full 64-lane unsigned max; result is wave-uniform (read from lane 63).
__device__ __forceinline__ uint32_t wave_max_u32_dpp(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));  // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));  // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));  // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));  // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));  // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Per-lane maximum of 8 registers, reduced over the wave; pod j's maximum
// lands in lanes 8k with j = rev3(k) (lanes 0, 8, .., 56 hold pods 0, 4, 2, 6,
// 1, 5, 3, 7). Other lanes hold partial maxima.
__device__ __forceinline__ uint32_t reduce8(const uint32_t (&r)[8], uint32_t lane) {
    uint32_t s[4], t[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // lanes < 32: pod 2i, lanes >= 32: pod 2i+1
        const auto p = __builtin_amdgcn_permlane32_swap(r[2 * i], r[2 * i + 1], false, false);
        s[i] = max((uint32_t)p[0], (uint32_t)p[1]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // rows 0..3: pods 4i+0, 4i+2, 4i+1, 4i+3
        const auto p = __builtin_amdgcn_permlane16_swap(s[2 * i], s[2 * i + 1], false, false);
        t[i] = max((uint32_t)p[0], (uint32_t)p[1]);
    }
    // within each row: lanes 0-7 keep t[0]'s pod, lanes 8-15 t[1]'s (row_ror:8 = lane ^ 8)
    const bool hi8 = (lane & 8u) != 0;
    const uint32_t keep = hi8 ? t[1] : t[0], send = hi8 ? t[0] : t[1];
    uint32_t u = max(keep, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, 0x128, 0xF, 0xF, false));
    u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
    u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
    u = max(u, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x104, 0xF, 0xF, false)); // row_shl:4
    return u;
}

__device__ __forceinline__ uint32_t rev3(uint32_t k) { return ((k & 1u) << 2) | (k & 2u) | ((k >> 2) & 1u); }

// Row slot of the lowest set bit (v_ffbl; 0xFFFFFFFF for an empty mask —
// defined, unlike __builtin_ctz(0)).
__device__ __forceinline__ uint32_t first_slot(uint32_t m) {
    uint32_t s;
    asm("v_ffbl_b32 %0, %1" : "=v"(s) : "v"(m));
    return s;
}

// Combined key -> per-pod outcome (minisched.go:143-148 FitError, :70-75 the
// score-error path, :80 selectHost's node). Keys 0 and 1 carry no node: 1 =
// some shard lists a node but none is feasible (kKeyListed), 0 = no shard
// lists any. flags: per-pod filter bytes of the resource-aware set (byte 0 NU,
// byte 1 NRF) or nullptr for NU+NN / NodeAffinity, where NodeUnschedulable is
// the only filter: F = 0 with a node listed (key 1, or a non-zero present
// count) means it rejected every node.
__device__ __forceinline__ ms_result decode_key(u64 k, int8_t pod_digit, const uint32_t *flags, uint32_t i,
                                                uint32_t present) {
    ms_result r;
    r._pad = 0;
    if (k <= kKeyListed) {  // FitError: no feasible node anywhere
        r.node = -1;
        r.code = MS_CODE_UNSCHEDULABLE;
        r.score = 0;
        if (flags) {
            const uint32_t f = flags[i];
            r.plugin_mask = ((f & 0xFFu) ? MS_MASK_NODE_UNSCHEDULABLE : 0u) |
                            ((f & 0xFF00u) ? MS_MASK_NODE_RESOURCES_FIT : 0u);
        } else {
            // NU+NN: NodeUnschedulable is the only filter, so F == 0 with at
            // least one node listed means every node was rejected by it.
            r.plugin_mask = (k == kKeyListed || present) ? MS_MASK_NODE_UNSCHEDULABLE : 0u;
        }
    } else if (pod_digit < 0) {  // NodeNumber.Score error, F > 0
        r.node = -1;
        r.code = MS_CODE_ERROR;
        r.score = 0;
        r.plugin_mask = 0;
    } else {
        r.node = (int32_t)(0xFFFFFu - (uint32_t)(k & 0xFFFFFu));
        r.code = MS_CODE_SUCCESS;
        r.score = (int64_t)(k >> 52);
        r.plugin_mask = 0;
    }
    return r;
}

// NodeInfo.AddPod / RemovePod (sign -1) on local row `row` (upstream
// types.go: Requested += req, NonZeroRequested += nz, len(Pods) += 1).
__device__ __forceinline__ void add_pod(const NodeTable &t, uint32_t row, const ms_pod_rec &pr, int sign) {
    atomicAdd(&t.pod_count[row], sign);
    atomicAdd(reinterpret_cast<u64 *>(&t.req_cpu[row]), (u64)(sign * pr.req_milli_cpu));
    atomicAdd(reinterpret_cast<u64 *>(&t.req_mem[row]), (u64)(sign * pr.req_memory));
    atomicAdd(reinterpret_cast<u64 *>(&t.nz_cpu[row]), (u64)(sign * pr.nonzero_milli_cpu));
    atomicAdd(reinterpret_cast<u64 *>(&t.nz_mem[row]), (u64)(sign * pr.nonzero_memory));
}

}  // namespace msgpu
