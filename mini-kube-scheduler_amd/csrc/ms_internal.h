// ms_internal.h — shared between the HIP kernels and the C-ABI host library.
// Not part of the public boundary (that is include/minisched_gpu.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "minisched_gpu.h"

namespace msgpu {

// Node flag byte (device column `flags`).
constexpr uint8_t kNodeUnschedulable = 0x01;  // node.Spec.Unschedulable
constexpr uint8_t kNodeAbsent = 0x80;         // tombstone / never added: not in Nodes().List

// NodeAffinity sweep geometry: one node per lane-slot, 16 slots per lane.
constexpr int kNunnThreads = 256;
constexpr int kNunnSlots = 16;
constexpr int kNunnTile = kNunnThreads * kNunnSlots;  // nodes per block

// K3 (resource-aware sweep) geometry.
constexpr int kFullThreads = 256;
constexpr int kFullSlots = 4;
constexpr int kFullWaveTile = 64 * kFullSlots;            // nodes per wave  (validator tile; the most rows a tile holds)
constexpr int kFullTile = kFullThreads * kFullSlots;      // nodes per block

constexpr uint32_t kGolden32 = 0x9E3779B1u;  // LDS map hashing in the validator

// Bytes of padding after the flags/digit/zone columns (vector loads of a
// lane's rows may run past the last row).
constexpr uint32_t kColumnPad = 64;

// Device-resident node table, structure of arrays, indexed by LOCAL ordinal.
struct NodeTable {
    uint8_t *flags;
    uint8_t *digit;
    uint8_t *zone;  // zone label value id (MS_PLUGINS_NU_NN_NA), 0 = none
    uint8_t *label2;  // second label value id (MS_PLUGINS_NU_NN_NAM term key 1), 0 = none
    uint32_t *taints;  // taint ids (MS_PLUGINS_NU_TT_NN): bits 0-7 NoSchedule/NoExecute, 8-15 PreferNoSchedule
    int32_t *allowed_pods;
    int32_t *pod_count;
    int64_t *alloc_cpu, *alloc_mem;
    int64_t *req_cpu, *req_mem;
    int64_t *nz_cpu, *nz_mem;
    uint32_t cap;   // rows allocated
    uint32_t base;  // global ordinal of row 0
    // K1 "pp" bit planes, derived from flags/digit (k_build_planes after every
    // delta batch): planes[p * gcap + g], p = kPlane*, one u32 per group g of
    // kGroupRows consecutive rows (bit s = row g*kGroupRows + s).
    uint32_t *planes;
    uint32_t gcap;  // groups allocated = cdiv(cap, kGroupRows)
    // Rows per tile of the config-E sweep (the engine's table copy; 0 = kFullWaveTile).
    // run_sequential sizes tiles so that every CU beside the validator's gets one
    // (a multiple of 16, 64..256): 208 rows at 50k nodes = 241 tiles, not 196 x 256.
    // (In the 4 bytes of padding before drow: the structure's size is unchanged.)
    uint32_t tile_rows;
    // Derived rows of the config-E sweep's binary64 form (DRow), set only in the
    // table copy the sequential engine passes to its launches: rebuilt at the
    // start of each run (k_build_drows) and kept current by the validator's
    // write-back of the rows it binds. nullptr everywhere else.
    struct DRow *drow;
};

__host__ __device__ inline uint32_t tile_rows_of(const NodeTable &t) {
    return t.tile_rows ? t.tile_rows : (uint32_t)kFullWaveTile;
}

// One node as the config-E sweep's binary64 LeastAllocated form reads it
// (ms_kernels.hip make_drow; 64 B, one row per lane and load).
struct DRow {
    int64_t fr_cpu, fr_mem;  // Allocatable - Requested (NodeResourcesFit)
    double r_cpu, r_mem;     // RN(100 / Allocatable), 0 when Allocatable <= 0
    double a_cpu, a_mem;     // RN(RN((Allocatable - NonZeroRequested) * r) + 2^-43)
    int32_t room;            // AllowedPodNumber - len(Pods)
    uint32_t fd;             // flags | digit << 8
    uint32_t digit;          // name digit (0xFF: none)
    uint32_t rbits;          // kRb* below: the row's static filter outcomes, precomputed
};
static_assert(sizeof(DRow) == 64, "DRow layout");
// DRow::rbits. kRbUnsched and kRbNoRoom are set for present rows only.
constexpr uint32_t kRbAbsent = 1u;   // not in Nodes().List
constexpr uint32_t kRbUnsched = 2u;  // Spec.Unschedulable (NodeUnschedulable rejects unless tolerated)
constexpr uint32_t kRbNoRoom = 4u;   // AllowedPodNumber - len(Pods) < 1 (NodeResourcesFit rejects every pod)
constexpr uint32_t kRbSlow = 8u;     // the binary64 LeastAllocated form is not exact for this row
constexpr uint32_t kRbBlocked = 16u; // absent or unschedulable: no pod that does not tolerate it may bind here

constexpr uint32_t kGroupRows = 30;
enum : uint32_t {
    kPlaneD0 = 0,   // name digit bit 0 (15 = no digit)
    kPlaneD1,
    kPlaneD2,
    kPlaneD3,
    kPlaneSched,    // present && !Spec.Unschedulable
    kPlanePresent,  // present (not tombstoned)
    kPlaneOver,     // bit 0: the group holds more than 3 present rows of one digit (K1 pp's scan path);
                    // bit 1: some present row's digit is not its ordinal mod 10 (no fixed-slot path)
    kPlaneDigitPres,   // present && the name ends in a digit
    kPlaneDigitSched,  // present && !Spec.Unschedulable && the name ends in a digit
    kPlanes
};

// One queued node delta (upsert or delete) as it travels to the device.
struct NodeDelta {
    uint32_t local;   // local row
    uint32_t absent;  // 1 = delete (tombstone)
    ms_node_rec rec;
};
static_assert(sizeof(ms_node_rec) == 64, "ms_node_rec layout");
static_assert(sizeof(ms_pod_rec) == 40, "ms_pod_rec layout");
static_assert(sizeof(ms_result) == 24, "ms_result layout");
static_assert(sizeof(ms_pod_compact) == 8, "ms_pod_compact layout");
static_assert(sizeof(ms_result_compact) == 8, "ms_result_compact layout");

// A shard's key for a pod with no feasible node on it: 1 when the shard lists at
// least one node, else 0 (real keys are >= 2: ordinals stop at MS_MAX_ORDINAL =
// 0xFFFFD, so the ordinal field 0xFFFFF - ordinal is >= 2). The element-wise MAX
// over shards then also tells the decode whether the cluster lists any node.
constexpr unsigned long long kKeyListed = 1ull;

__host__ __device__ inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
__host__ __device__ inline uint32_t seed32_of(uint64_t seed) { return (uint32_t)(seed ^ (seed >> 32)); }

// Tie-break hash (minisched_gpu.h, rule "r3"; oracle/ms_oracle.c msor_tb_hash):
//   A = fmix32(seed32 ^ pod_ordinal); h = mix32(A + node_ordinal * kG24)
// mix32(x): x ^= x>>16; x *= 0x85ebca6b; x ^= x>>16; x *= 0xc2b2ae35 (both
// xor-shifts by 16, one SDWA v_xor each). node_ordinal < 2^20, so the
// product is one v_mad_u32_u24. For a fixed pod h is a bijection of the
// ordinal (odd multipliers, xor-shifts by 16 are involutions), so no two nodes
// of one pod share a hash and tb_unhash recovers the ordinal from h alone: the
// sweep reduces bare 32-bit hashes and never carries the row along.
constexpr uint32_t kG24 = 0x9E3779u;  // odd, 24-bit
constexpr uint32_t kG24Inv = 0xF2B382C9u;  // kG24^-1 mod 2^32
__host__ __device__ inline uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x85ebca6bu;
    x ^= x >> 16;
    x *= 0xc2b2ae35u;
    return x;
}
__host__ __device__ inline uint32_t unmix32(uint32_t h) {
    h *= 0x7ED1B41Du;  // 0xc2b2ae35^-1
    h ^= h >> 16;
    h *= 0xA5CB9243u;  // 0x85ebca6b^-1
    h ^= h >> 16;
    return h;
}
__host__ __device__ inline uint32_t tb_pod(uint32_t seed32, uint32_t pod_ordinal) {
    return fmix32(seed32 ^ pod_ordinal);
}
__host__ __device__ inline uint32_t tb_hash(uint32_t A, uint32_t node_ordinal) {
    return mix32(A + node_ordinal * kG24);
}
// The node ordinal whose tb_hash under pod half A is h.
__host__ __device__ inline uint32_t tb_unhash(uint32_t A, uint32_t h) { return (unmix32(h) - A) * kG24Inv; }

// ---- MS_PLUGINS_NU_NN_NAM launchers (ms_affinity.hip) ----------------------
// A term set as the device reads it (built on the host from ms_nam_term_set(_ext)):
// z[v] / l[v] bit t = term t (weight > 0) holds zone / label2 value id v; wsum[m]
// = the weight sum of the terms in 4-bit mask m. raw = wsum[z[zone] & l[label2]].
struct NamTab {
    uint8_t z[256];
    uint8_t l[256];
    uint16_t wsum[16];
};
// Row segments and scratch shape of one call's per-class passes (cls_max = the
// most classes a chunk can hold: min(pods, 2 (n_sets + 1))).
struct NamLayout {
    uint32_t segs = 1, seg_rows = 64, fpitch = 64, cls_max = 1;
};
NamLayout nam_layout(uint32_t n_rows, uint32_t cls_max);
size_t nam_scratch_bytes(const NamLayout &L, uint32_t n_pods, uint32_t n_sets);
// Node shards, step 1: per pod this context's composed rescale record (out:
// MS_NAM_SEG_BYTES per pod), computed per class.
hipError_t launch_nam_segment(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                              const void *sets, uint32_t n_sets, const NamLayout &L, void *scratch, void *out,
                              hipStream_t s);
// n identity records (a shard without rows).
hipError_t launch_nam_identity(void *out, uint32_t n, hipStream_t s);
// Per pod the composition of n records in[s * stride + p] (s ascending); skip_to >= 0:
// only the records after skip_to, and m_in[p] = the OR of "any" of those before it.
hipError_t launch_nam_compose(const void *in, uint32_t stride, uint32_t n, uint32_t n_pods, int32_t skip_to,
                              void *out, uint8_t *m_in, hipStream_t s);
// Per pod the best packed key over this context's rows (keys[p] written; listed:
// the context lists a row, so a pod with none feasible gets kKeyListed); after /
// m_in: launch_nam_compose's outputs for these pods (node shards), or null.
hipError_t launch_nam_keys(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                           const void *sets, uint32_t n_sets, uint32_t seed32, uint32_t w_nn, uint32_t w_na,
                           const void *after, const uint8_t *m_in, uint32_t listed, const NamLayout &L,
                           void *scratch, unsigned long long *keys, hipStream_t s);

// ---- launchers (ms_kernels.hip) -------------------------------------------
// All return hipError_t of the launch; none synchronises.
hipError_t launch_apply_deltas(const NodeTable &t, const NodeDelta *d_deltas, uint32_t n, hipStream_t s);
hipError_t launch_init_table(const NodeTable &t, hipStream_t s);
// K1 "pp" (ms_sweep_pp.hip): every (pod, node) pair through NU + NN + selectHost.
// results != nullptr: decoded ms_result per pod (single-shard cycle; keys is
// scratch, needed only above 122,880 rows), and with commit != 0 each winner's
// NodeInfo.AddPod in the same launch; else keys[i] = this shard's max packed
// key (0 = none), overwritten. present: global present-node count (decode).
hipError_t launch_sweep_pp(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                           uint32_t seed32, unsigned long long *keys, ms_result *results, uint32_t present,
                           int num_cus, hipStream_t s, int commit = 0, hipEvent_t done = nullptr);
// Two shard sweeps (keys only, rows <= kPpMaxFusedRows) in ONE launch: the
// per-launch ramp and drain are paid once for both batches (ms_sharded_submit
// coalesces consecutive submits). done: recorded after both.
hipError_t launch_sweep_pp2(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods1, uint32_t n1,
                            unsigned long long *keys1, const ms_pod_rec *pods2, uint32_t n2, unsigned long long *keys2,
                            uint32_t seed32, uint32_t present, int num_cus, hipStream_t s, hipEvent_t done);
// The compact host-array cycle (ms_schedule_batch_compact) in one launch, rows
// <= kPpMaxFusedRows: pods are ms_pod_compact records and results
// ms_result_compact, both in pinned host memory the kernel reads and writes
// over PCIe (no copy launches, no widen / narrow passes); binds committed.
hipError_t launch_sweep_pp_compact(const NodeTable &t, uint32_t n_rows, const ms_pod_compact *pods, uint32_t n_pods,
                                   uint32_t seed32, ms_result_compact *results, uint32_t present, int num_cus,
                                   hipStream_t s);
// (done, optional: recorded after the sweep, by its own dispatch when it is
// one launch: no separate event packet on s)
// Rows one K1 pp workgroup holds (16 waves x 64 lanes x 4 groups of 30):
// up to here the single-shard cycle is one launch with no key scratch.
constexpr uint32_t kPpMaxFusedRows = 16u * 64u * 4u * kGroupRows;
// Rebuilds the bit planes of the groups touched by deltas (or all groups when d_deltas is null).
hipError_t launch_build_planes(const NodeTable &t, const NodeDelta *d_deltas, uint32_t n, hipStream_t s);
// keys[0, n) = v (the atomicMax targets of the NodeAffinity / resource sweeps
// start at kKeyListed when the shard lists a node, else 0)
hipError_t launch_fill_keys(unsigned long long *keys, uint32_t n, unsigned long long v, hipStream_t s);
// MS_PLUGINS_NU_NN_NA sweep (one pair per lane-slot): keys[i] = max packed key
// with raw NodeAffinity scores, fkeys[i] = max over this shard's feasible nodes
// with a non-zero raw NodeAffinity score of ((0xFFFFF - ordinal) << 1 | NN
// match) + 1, i.e. the normalise hook's anchor (the first such node in LIST
// order); both atomicMax targets, zeroed by the caller. w: score weights.
hipError_t launch_sweep_na(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                           uint32_t seed32, uint32_t w_nn, uint32_t w_na, unsigned long long *keys, uint32_t *fkeys,
                           int num_cus, hipStream_t s);
// decode of the NU+NN+NA set: the anchor's score becomes w_na * 100
hipError_t launch_decode_na(const ms_pod_rec *pods, uint32_t n_pods, const unsigned long long *keys,
                            const uint32_t *fkeys, uint32_t present_nodes, uint32_t seed32, uint32_t w_nn,
                            uint32_t w_na, ms_result *out, hipStream_t s, const uint32_t *present_dev = nullptr);
hipError_t launch_sweep_full(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                             uint32_t seed32, unsigned long long *keys, uint32_t *flags, int num_cus,
                             hipStream_t s);
// Per-(pod, wave tile) speculative sweep for the sequential engine: the
// tile's top-K keys at tile_keys[(p * n_tiles + t) * K + j], 0-terminated,
// and its filter flags at tile_flags[p * n_tiles + t].
// spec[p] accumulates (atomicMax) pod p's speculative global winner key and
// spec_flags[p] the filter flags of tiles without a feasible row; both must be
// zero on entry (the validator zeroes the entries it consumed).
hipError_t launch_sweep_full_tiles(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods,
                                   uint32_t n_pods, uint32_t seed32, unsigned long long *tile_keys,
                                   uint32_t *tile_flags, uint32_t n_tiles, hipStream_t s);
// Per pod: global speculative top-4 from the tile lists (top[p*4 + r]), the
// speculative winner (rank 0) and the filters of tiles with no feasible row;
// recs (optional, n_pods * 4 * seq_rec_fields() i64) gets the four entries'
// batch-start node records for the in-order validator; ext (optional, n_pods * 4)
// ranks 4..7 for its slow pods, with the certified rank count in spec_flags
// bits 28-31 (the validators pass it as top_ext).
hipError_t launch_topk_merge(const unsigned long long *tile_keys, const uint32_t *tile_flags, uint32_t n_pods,
                             uint32_t n_tiles, unsigned long long *top, unsigned long long *spec, uint32_t *spec_flags,
                             const NodeTable &t, int64_t *recs, hipStream_t s, unsigned long long *ext = nullptr);
// Batch k+1's merge inside step k at depth 1 (MINISCHED_SEQ_MERGE=instep):
// once every sweep workgroup of the step has written batch k+1's tile lists
// (write-through stores, counted on ctr), their waves merge its pods into these
// buffers (launch_topk_merge's outputs), tagging each merged pod with `tag`.
// The wait is bounded: a worker that gives up leaves its pods untagged and
// validation k+1 merges them itself, so a grid that is not co-resident costs
// time, never correctness. ctr: a u32 zeroed at the run's start; target: the
// count after the run's earlier in-step merges, advanced by launch_seq_step.
// in_tags / in_tag: batch k's tags (in_tag 0: batch k was merged by a launch).
// skip: the workers leave every pod to the fallback (a test hook).
struct SeqMergeIO {
    const uint32_t *in_tags = nullptr;
    uint32_t in_tag = 0;
    unsigned long long *top = nullptr, *spec = nullptr, *ext = nullptr;
    uint32_t *spec_flags = nullptr, *tags = nullptr, *ctr = nullptr;
    int64_t *recs = nullptr;
    uint32_t tag = 0, target = 0;
    int skip = 0;
    // MS_VSTAMPS diagnostic build: per-workgroup timestamps of steps
    // tl_step < kTimelineSteps (u64 [step][workgroup][8], s_memrealtime)
    unsigned long long *tl = nullptr;
    uint32_t tl_step = ~0u;
};
constexpr uint32_t kTimelineSteps = 2048, kTimelineWgs = 256;  // (a config E run: 1627 steps)
// Whether launch_seq_step can merge n_next pods in-step (else launch_topk_merge follows).
bool seq_step_merges(const NodeTable &t, uint32_t n_tiles, uint32_t n_next);
// One single-stream step: in-order validation of batch k (n_pods, workgroup 0;
// writes results and commits binds to the table) while sweeping the next batch
// (n_next pods: tile lists, and with mio their in-step merge; else
// launch_topk_merge follows the step). prev_in / prev_recs_in: the stale nodes
// (bound by the previous batch) with their final records ({n_own, n_carried,
// rows} of 2 + seq_prev_cap() words; seq_prev_cap() * seq_rec_fields() i64),
// written by the previous validation into its prev_out / prev_recs_out.
// stats: u32[6] = overflow flags, re-swept tiles, recomputed entries, pods,
// speculation misses, pods whose speculative winner was touched. Any count may be 0.
hipError_t launch_seq_step(const NodeTable &t, uint32_t n_rows, uint32_t n_tiles, uint32_t seed32,
                           const ms_pod_rec *pods, uint32_t n_pods, const unsigned long long *tile_keys,
                           const uint32_t *tile_flags, const unsigned long long *spec, const uint32_t *spec_flags,
                           const unsigned long long *top4, const int64_t *top4_recs, const uint32_t *prev_in,
                           const int64_t *prev_recs_in, uint32_t *prev_out, int64_t *prev_recs_out,
                           ms_result *results, uint32_t *stats, const ms_pod_rec *next_pods, uint32_t n_next,
                           unsigned long long *next_tile_keys, uint32_t *next_tile_flags, int num_cus,
                           hipStream_t s, const unsigned long long *top_ext = nullptr, SeqMergeIO *mio = nullptr);
// Node-sharded sequential mode (minisched_gpu.h ms_seq_*): this shard's top-4
// candidates with records + all-tile filter flags per pod, from the top-4 merge
// output; and the replicated validation over the shards' gathered lists
// (merged / merged_flags: n_pods * 4 / n_pods scratch).
hipError_t launch_seq_pack_cands(const NodeTable &t, const unsigned long long *top4, const uint32_t *tile_flags,
                                 uint32_t n_tiles, uint32_t n_pods, ms_seq_cand *cands, uint32_t *flags, hipStream_t s);
// live (optional): validate only the first min(n_pods, *live) pods (a cursor window)
hipError_t launch_seq_validate_rep(const NodeTable &t, uint32_t n_pods, const ms_pod_rec *pods, uint32_t seed32,
                                   uint32_t n_shards, const ms_seq_cand *cands_all, const uint32_t *flags_all,
                                   ms_seq_cand *merged, uint32_t *merged_flags, ms_result *results, uint32_t *n_done,
                                   hipStream_t s, const uint32_t *live = nullptr);
// Device cursor of the in-library node-sharded sequential cycle: ctl = {cursor,
// live, n_done}; window_in stages pods [cursor, cursor + live) of n into win (w
// entries), window_out copies ctl[2] decided results to res[cursor ..] and
// advances the cursor (ms_kernels.hip).
hipError_t launch_seq_window_in(const ms_pod_rec *pods, uint32_t n, uint32_t *ctl, ms_pod_rec *win, uint32_t w,
                                hipStream_t s);
hipError_t launch_seq_window_out(const ms_result *win_res, uint32_t *ctl, ms_result *res, uint32_t n, hipStream_t s);
// Derived rows [0, n_total) of the sequential engine's table copy (t.drow): rows
// at or past n_rows are absent.
hipError_t launch_build_drows(const NodeTable &t, uint32_t n_rows, uint32_t n_total, hipStream_t s);
// Rows the sequential engine's validator supports (tile lists held in registers).
uint32_t seq_max_rows();
// present_dev (optional): read the present count from the device (node-sharded combine)
hipError_t launch_decode(const ms_pod_rec *pods, uint32_t n_pods, const unsigned long long *keys,
                         const uint32_t *flags, uint32_t present_nodes, ms_result *out, hipStream_t s,
                         const uint32_t *present_dev = nullptr);
// MS_PLUGINS_NU_TT_NN (ms_taint.hip): per-pod summaries of LIST-ordered row
// segments (tt_segments(n_rows) of them, segment s at summaries[s * n_pods + p],
// MS_TT_SUMMARY_BYTES each), and their merge: n_segs summaries per pod (segment
// s at in[s * stride + p]) into out[p] (merged summary) or, with out null,
// results[p] (commit: NodeInfo.AddPod on winners this table owns).
uint32_t tt_segments(uint32_t n_rows, uint32_t *seg_rows = nullptr);
hipError_t launch_tt_sweep(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                           uint32_t seed32, void *summaries, hipStream_t s);
// The two-pass bit-sliced TaintToleration cycle of one context (ms_taint.hip
// k_tt2_*): row planes once per cycle (launch_tt2_planes), then per chunk of up
// to max_pods pods census -> plan -> pick -> final into results (commit: binds).
uint32_t tt2_words(uint32_t n_rows);
size_t tt2_scratch_bytes(uint32_t n_rows, uint32_t max_pods);
hipError_t launch_tt2_planes(const NodeTable &t, uint32_t n_rows, void *scratch, hipStream_t s);
hipError_t launch_tt2_cycle(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                            uint32_t seed32, void *scratch, uint32_t max_pods, ms_result *results, int commit,
                            hipStream_t s);
// Node shards of the two-pass cycle: a shard's census (one MS_TT_CENSUS_BYTES
// record per pod, its segments merged, ordinals global); its pick under the plan
// of every shard's census (census_all[s * stride + p], shards in LIST order) ->
// one key per pod for the cross-shard uint64 MAX; the results from the census of
// every shard and the MAX of the keys.
hipError_t launch_tt2_census_shard(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                                   uint32_t seed32, void *scratch, uint32_t max_pods, void *census_out,
                                   hipStream_t s);
hipError_t launch_tt2_pick_shard(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                                 uint32_t seed32, void *scratch, uint32_t max_pods, const void *census_all,
                                 uint32_t stride, uint32_t n_shards, uint32_t shard, unsigned long long *keys_out,
                                 hipStream_t s);
// The plan records inside a two-pass scratch (tt2_scratch_bytes) for max_pods pods.
void *tt2_plans(void *scratch, uint32_t n_rows, uint32_t max_pods);
hipError_t launch_tt2_final_shard(const NodeTable &t, uint32_t n_rows, const ms_pod_rec *pods, uint32_t n_pods,
                                  uint32_t seed32, void *plans_buf, uint32_t max_pods, const void *census_all,
                                  uint32_t stride, uint32_t n_shards, const unsigned long long *keys_max,
                                  ms_result *results, hipStream_t s);
hipError_t launch_tt_combine(const void *in, uint32_t stride, uint32_t n_segs, const ms_pod_rec *pods, uint32_t n_pods,
                             uint32_t seed32, void *out, ms_result *results, const NodeTable &t, int commit,
                             hipStream_t s);
// One launch decoding several batches' pod slices, each with a device-side present flag.
constexpr uint32_t kMaxSliceJobs = 8;
struct SliceJob {
    const ms_pod_rec *pods;
    const unsigned long long *keys;
    const uint32_t *flags;    // NodeResourcesFit set: combined filter bytes; else nullptr
    const uint32_t *present;  // device present count, or nullptr: from the key (kKeyListed)
    ms_result *results;
    uint32_t n_pods, _pad;
};
hipError_t launch_decode_slices(const SliceJob *jobs, uint32_t n_jobs, hipStream_t s);
// n_jobs in [1, MS_DECODE_MAX_JOBS] (checked by the caller)
hipError_t launch_decode_jobs(const ms_decode_job *jobs, uint32_t n_jobs, uint32_t present_nodes, hipStream_t s);
hipError_t launch_apply_binds(const NodeTable &t, const ms_pod_rec *pods, uint32_t n_pods,
                              const ms_result *res, hipStream_t s);
hipError_t launch_bind_one(const NodeTable &t, uint32_t local, const ms_pod_rec *pod_dev, int sign,
                           hipStream_t s);
hipError_t launch_read_rows(const NodeTable &t, uint32_t first, uint32_t n, ms_node_rec *out, hipStream_t s);
// Compact records (ms_schedule_batch_compact): pods widened to ms_pod_rec (zero
// requests), results narrowed to ms_result_compact, on the device.
hipError_t launch_pods_widen(const ms_pod_compact *in, uint32_t n, ms_pod_rec *out, hipStream_t s);
hipError_t launch_results_narrow(const ms_result *in, uint32_t n, ms_result_compact *out, hipStream_t s);
// Largest speculative batch the sequential validator accepts.
uint32_t seq_batch_limit();
// i64 fields per validator node record; stale nodes per prev list.
uint32_t seq_rec_fields();
uint32_t seq_prev_cap();
// Entries per (pod, tile) speculative list: tile_keys has n_pods * n_tiles * seq_topk() u64.
uint32_t seq_topk();

}  // namespace msgpu
