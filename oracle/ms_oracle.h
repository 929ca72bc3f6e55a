/*
 * ms_oracle.h — CPU restatement of minisched's scheduling cycle.
 *
 * TEST INFRASTRUCTURE ONLY. This is the checker, never the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it. The product path (libminisched_gpu.so) never links or calls it.
 *
 * Parity status: the Go reference cannot be built or run here (no Go
 * toolchain, no k8s.io module cache; see DESIGN.md "Oracle"). The
 * restatement is pinned by the reference's only executable known answer,
 * the README scenario (sched.go:70-140: node0..node8 unschedulable -> pod1
 * FitError{NodeUnschedulable}; add node10 -> pod1 bound to node10), plus
 * hand-derived KATs read off nodenumber.go:50-95 and minisched.go:115-199,
 * 304-325. Everything beyond those KATs (selectHost tie-break, upstream
 * NodeResourcesFit/LeastAllocated) is "parity unpinned" by reference
 * outputs: it is a restatement of published upstream v1.22 semantics.
 */
#ifndef MS_ORACLE_H
#define MS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* plugin sets (same numbering as include/minisched_gpu.h) */
#define MSOR_PLUGINS_NU_NN 0        /* Filter[NodeUnschedulable], Score[NodeNumber]          */
#define MSOR_PLUGINS_NU_NRF_NN_LA 1 /* Filter[NU, NodeResourcesFit], Score[NN, LeastAllocated] */
#define MSOR_PLUGINS_NU_NN_NA 2     /* Filter[NU], Score[NN, NodeAffinity + DefaultNormalizeScore] */
#define MSOR_PLUGINS_NU_TT_NN 3     /* Filter[NU, TaintToleration], Score[NN, TaintToleration +
                                       DefaultNormalizeScore(reverse=true)]                 */

#define MSOR_MODE_BATCHED 0    /* every pod against the same node state          */
#define MSOR_MODE_SEQUENTIAL 1 /* queue order, assume-on-select NodeInfo.AddPod   */

#define MSOR_CODE_SUCCESS 0
#define MSOR_CODE_ERROR 1         /* framework.Error from a score plugin (non-FitError) */
#define MSOR_CODE_UNSCHEDULABLE 2 /* *framework.FitError                               */

#define MSOR_MASK_NU (1u << 0)
#define MSOR_MASK_NRF (1u << 1)
#define MSOR_MASK_TT (1u << 2)

#define MSOR_NODE_UNSCHEDULABLE 0x01u
#define MSOR_NODE_ABSENT 0x80u

/* Node table, structure of arrays; resource columns may be NULL for NU_NN. */
typedef struct {
    uint32_t n;
    const uint8_t *flags; /* bit0 Spec.Unschedulable, bit7 tombstone (not in LIST) */
    const uint8_t *digit; /* last char of node name as 0..9, 0xFF = non-digit      */
    int32_t *allowed_pods, *pod_count;
    int64_t *alloc_cpu, *alloc_mem; /* Allocatable.MilliCPU / .Memory              */
    int64_t *req_cpu, *req_mem;     /* Requested.MilliCPU / .Memory                */
    int64_t *nz_cpu, *nz_mem;       /* NonZeroRequested.MilliCPU / .Memory         */
    const uint8_t *zone;            /* zone label value id, 0 = none (NU_NN_NA)   */
    /* taint ids of the cluster's taint universe (NU_TT_NN): bits 0-7 taints with
     * effect NoSchedule or NoExecute, bits 8-15 taints with effect PreferNoSchedule */
    const uint32_t *taints;
    /* second node label value id, 0 = none (NU_NN_NAM: label key 1 of the terms) */
    const uint8_t *label2;
} msor_nodes;

typedef struct {
    uint32_t n;
    const uint32_t *ordinal; /* stable pod id fed to the tie-break hash           */
    const int8_t *digit;     /* last char of pod name as 0..9, -1 = non-digit     */
    const uint8_t *tol;      /* tolerates node.kubernetes.io/unschedulable:NoSchedule */
    const int64_t *req_cpu, *req_mem, *nz_cpu, *nz_mem; /* may be NULL for NU_NN */
    const uint8_t *pref_zone, *pref_weight; /* one preferred zone term (NU_NN_NA)  */
    /* NU_TT_NN: bit t set when some toleration of the pod tolerates taint id t
     * (v1 ToleratesTaint, host-side): tol_hard over bits 0-7, tol_soft over 8-15 */
    const uint8_t *tol_hard, *tol_soft;
} msor_pods;

uint32_t msor_fmix32(uint32_t h);
uint32_t msor_seed32(uint64_t seed);
uint32_t msor_pod_hash(uint64_t seed, uint32_t pod_ordinal);
uint32_t msor_mix32(uint32_t x);
uint32_t msor_tb_hash(uint32_t pod_hash, uint32_t node_ordinal);
uint32_t msor_h32(uint64_t seed, uint32_t pod_ordinal, uint32_t node_ordinal);
uint64_t msor_key(int64_t score, uint32_t h, uint32_t node_ordinal);
int64_t msor_least_requested(int64_t requested, int64_t capacity);

/* Schedules pods[0..n) in order. node_base = global ordinal of local node 0.
 * Outputs (each length pods->n, any may be NULL):
 *   out_node  global ordinal of the selected node or -1
 *   out_score summed score of the selected node (0 otherwise)
 *   out_code  MSOR_CODE_*
 *   out_mask  FitError UnschedulablePlugins as MSOR_MASK_* bits
 *   out_key   winning packed key (0 when no feasible node)
 * In MSOR_MODE_SEQUENTIAL the node resource columns are updated in place.
 * Returns 0, or -1 on invalid arguments. */
int msor_schedule(msor_nodes *nodes, const msor_pods *pods, int plugin_set, int mode,
                  uint64_t seed, uint32_t node_base, int32_t *out_node, int64_t *out_score,
                  int32_t *out_code, uint32_t *out_mask, uint64_t *out_key);

/* Same semantics, NU_NN only, pods evaluated in parallel with OpenMP
 * (the multi-core CPU baseline). threads <= 0 means all cores. */
int msor_schedule_nunn_omp(const msor_nodes *nodes, const msor_pods *pods, uint64_t seed,
                           uint32_t node_base, int threads, int32_t *out_node,
                           int64_t *out_score, int32_t *out_code, uint32_t *out_mask,
                           uint64_t *out_key);

/* "Faithful" single-thread form for NU_NN: per (pod, node) it re-parses the
 * last character of the node NAME (Atoi, nodenumber.go:81-87) and builds the
 * feasible list and the NodeScoreList like minisched.go:115-199 before
 * selectHost. names: n_nodes NUL-terminated strings. Used only as the
 * reference-shaped CPU baseline. */
int msor_schedule_nunn_names(const char *const *node_names, const uint8_t *node_flags,
                             uint32_t n_nodes, const char *const *pod_names,
                             const uint8_t *pod_tol, const uint32_t *pod_ordinal,
                             uint32_t n_pods, uint64_t seed, int32_t *out_node,
                             int64_t *out_score, int32_t *out_code, uint32_t *out_mask);

/* MSOR_PLUGINS_NU_NN_NA, batched (no mutable state: sequential is the same).
 * Score plugins in order [NodeNumber (weight w_nn), NodeAffinity preferred
 * term (weight w_na)]; NodeAffinity's ScoreExtensions is upstream
 * DefaultNormalizeScore(MaxNodeScore=100, reverse=false), which
 * RunScorePlugins calls on the WHOLE, partially filled list after every node
 * (minisched.go:164-185). literal=1 runs that loop as written (O(F^2) per
 * pod); literal=0 uses its closed form for raw scores <= 100: every entry
 * keeps its raw score except the first feasible node (LIST order) with a
 * non-zero raw score, which ends at 100. Weights: total = w_nn*NN + w_na*NA
 * (the reference's sum is unweighted, minisched.go:186; 1/1 reproduces it). */
int msor_schedule_na(const msor_nodes *nodes, const msor_pods *pods, int64_t w_nn, int64_t w_na, int literal,
                     uint64_t seed, uint32_t node_base, int32_t *out_node, int64_t *out_score,
                     int32_t *out_code, uint32_t *out_mask, uint64_t *out_key);

/* MSOR_PLUGINS_NU_NN_NAM (4), batched: NodeAffinity with SEVERAL preferred
 * terms. A pod's term set id is pref_zone | pref_weight << 8 (0 = no terms);
 * set s (1-based) is term_sets[16 (s-1) .. 16 s): four terms of 4 bytes
 * {label key (0: the zone label, 1: label2), value id (0xFF: Exists), weight
 * (1..100; 0 = unused slot), 0}. NodeAffinity.Score = the sum of the weights of
 * the matching terms (so raw scores reach 400), normalised by
 * DefaultNormalizeScore(100, reverse=false) on the whole list after every node
 * (minisched.go:164-185). literal=1 runs that loop (O(F^2) per pod);
 * literal=0 its closed form (msor_nam_inloop). Weights as msor_schedule_na. */
#define MSOR_PLUGINS_NU_NN_NAM 4
#define MSOR_NAM_TERMS 4
int msor_schedule_nam(const msor_nodes *nodes, const msor_pods *pods, const uint8_t *term_sets, uint32_t n_sets,
                      int64_t w_nn, int64_t w_na, int literal, uint64_t seed, uint32_t node_base, int32_t *out_node,
                      int64_t *out_score, int32_t *out_code, uint32_t *out_mask, uint64_t *out_key);
/* The same with term sets in general form (minisched_gpu.h ms_nam_term_set_ext):
 * MSOR_NAM_EXT_BYTES per set, four terms of MSOR_NAM_TERM_BYTES: two 256-bit
 * value-id sets (8 little-endian u32 each: the zone label's, then label2's; bit
 * 0 = the label is absent), weight (0..100), 3 pad bytes. A term matches a node
 * whose zone id and label2 id are both in its sets. */
#define MSOR_NAM_TERM_BYTES 68
#define MSOR_NAM_EXT_BYTES (4 * MSOR_NAM_TERM_BYTES)
int msor_schedule_nam_ext(const msor_nodes *nodes, const msor_pods *pods, const uint8_t *term_sets, uint32_t n_sets,
                          int64_t w_nn, int64_t w_na, int literal, uint64_t seed, uint32_t node_base,
                          int32_t *out_node, int64_t *out_score, int32_t *out_code, uint32_t *out_mask,
                          uint64_t *out_key);
/* The in-loop reverse=false hook on one list of raw scores r[0..F) (any
 * non-negative values): literal=1 the loop as written, 0 the closed form
 * (out[k] = T_{>k}(v_k), T_{>k} the composition of v -> floor(100 v / r_i) over
 * the later entries with r_i > 100, v_k = 100 for the first non-zero entry
 * and for r_k > 100, else r_k). Returns -1 on a negative raw score. */
int msor_nam_inloop(const int64_t *r, uint32_t F, int literal, int64_t *out);

/* upstream k8s@v1.22.0 pkg/scheduler/framework/plugins/helper/normalize_score.go */
void msor_default_normalize(int64_t max_priority, int reverse, int64_t *scores, uint32_t n);

/* MSOR_PLUGINS_NU_TT_NN, batched (stateless). Filter plugins in order
 * [NodeUnschedulable, TaintToleration]; score plugins [NodeNumber,
 * TaintToleration] with TaintToleration's ScoreExtensions =
 * DefaultNormalizeScore(MaxNodeScore=100, reverse=true), run by RunScorePlugins
 * on the WHOLE list after every node (minisched.go:164-185). literal=1 runs
 * that loop as written (O(F^2) per pod); literal=0 its closed form
 * (msor_tt_inloop). FitError mask bits: NU, TT (MSOR_MASK_TT). */
int msor_schedule_tt(const msor_nodes *nodes, const msor_pods *pods, int literal, uint64_t seed,
                     uint32_t node_base, int32_t *out_node, int64_t *out_score, int32_t *out_code,
                     uint32_t *out_mask, uint64_t *out_key);

/* The TaintToleration list after RunScorePlugins' in-loop hook: raw counts
 * c[0..F) (each in 0..8) in LIST order -> final normalised scores out[0..F).
 * literal=1: the loop as written; literal=0: the closed form.
 * Returns 0, or -1 when a count is out of range. */
int msor_tt_inloop(const int64_t *c, uint32_t F, int literal, int64_t *out);

#ifdef __cplusplus
}
#endif
#endif
