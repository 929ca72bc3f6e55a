/*
 * minisched_gpu.h — C ABI of the MI355X scheduling-cycle engine.
 *
 * This is the drop-in boundary for minisched's per-pod scheduling cycle
 * (reference: /root/reference/minisched/minisched.go). In the reference one
 * goroutine runs, per pod:
 *     Nodes().List            minisched.go:40
 *     RunFilterPlugins        minisched.go:115-151  (NodeUnschedulable)
 *     RunPreScorePlugins      minisched.go:153-162  (NodeNumber.PreScore)
 *     RunScorePlugins         minisched.go:164-199  (NodeNumber.Score, unweighted sum)
 *     selectHost              minisched.go:304-325  (argmax, random tie-break)
 * A cgo shim calls ms_schedule_batch() in place of minisched.go:40-85 and
 * keeps the queue (:34), Permit (:89-94), the bind goroutine (:96-112) and
 * ErrorFunc (:283-298) in Go. INTEGRATION.md shows that shim.
 *
 * Plain C types only: no HIP, torch or C++ types cross this boundary. Every
 * function returns 0 (MS_OK) or a negative MS_E_* code and never aborts the
 * process; per-pod outcomes are data in ms_result, not errors.
 *
 * Node ordinals are global (0 .. MS_MAX_ORDINAL = 2^20-3). A context owns the contiguous
 * ordinal range [node_base, node_base + max_nodes) — one shard when nodes are
 * split across GPUs. The tie-break that replaces rand.Intn
 * (minisched.go:316-321) is the packed key
 *     key = score<<52 | h32(seed,pod,node)<<20 | (0xFFFFF - node),
 *     h32 = mix32(fmix32(seed32 ^ pod_ordinal) + node * 0x9E3779),
 *     seed32 = (uint32)(seed ^ seed>>32),
 * (rule "r3"; fmix32 = murmur3 finaliser; mix32(x) = x^=x>>16, x*=0x85ebca6b,
 * x^=x>>16, x*=0xc2b2ae35; all arithmetic mod 2^32). Maximum wins: the highest
 * score, then the highest hash. For one pod h32 is a bijection of the node
 * ordinal, so hashes never tie. It is a pure function of (seed, pod, node) so the
 * result does not depend on scan order, sharding or reduction tree
 * (DESIGN.md §2).
 */
#ifndef MINISCHED_GPU_H
#define MINISCHED_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MS_ABI_VERSION 7

/* ---- return codes -------------------------------------------------------- */
#define MS_OK 0
#define MS_E_INVAL (-1)    /* bad argument / state                         */
#define MS_E_HIP (-2)      /* a HIP runtime call failed                    */
#define MS_E_RCCL (-3)     /* an RCCL call of the communicator failed      */
#define MS_E_OOM (-4)      /* device or pinned allocation failed          */
#define MS_E_CAPACITY (-5) /* ordinal outside this context's node range    */
#define MS_E_NODEV (-6)    /* no usable gfx950 device                      */

/* ---- plugin sets (minisched/initialize.go:80-138 hard-codes the first) --- */
#define MS_PLUGINS_NU_NN 0        /* Filter[NodeUnschedulable]; Score[NodeNumber]            */
#define MS_PLUGINS_NU_NRF_NN_LA 1 /* Filter[NU, NodeResourcesFit]; Score[NN, LeastAllocated] */
/* Filter[NU]; Score[NN (weight w0), NodeAffinity preferred (weight w1) with
 * ScoreExtensions = DefaultNormalizeScore(MaxNodeScore, reverse=false), run by
 * RunScorePlugins' in-loop hook (minisched.go:178-183) exactly as written]. */
#define MS_PLUGINS_NU_NN_NA 2
/* Filter[NU, TaintToleration]; Score[NN, TaintToleration with ScoreExtensions =
 * DefaultNormalizeScore(MaxNodeScore, reverse=true), run by RunScorePlugins'
 * in-loop hook exactly as written]. Taints are ids of a cluster-wide universe
 * the shim assigns: ms_node_rec.taints bits 0-7 = NoSchedule / NoExecute taint
 * ids on the node, bits 8-15 = PreferNoSchedule ids; ms_pod_rec bytes
 * pref_zone / pref_weight carry tol_hard / tol_soft: bit t set when some
 * toleration of the pod tolerates taint id t (v1 ToleratesTaint; for
 * PreferNoSchedule ids only tolerations with that or an empty effect can).
 * (k8s@v1.22.0 plugins/tainttoleration/taint_toleration.go, restated.) */
#define MS_PLUGINS_NU_TT_NN 3
/* Filter[NU]; Score[NN (weight w0), NodeAffinity with SEVERAL preferred terms
 * (weight w1), ScoreExtensions = DefaultNormalizeScore(MaxNodeScore,
 * reverse=false) run by the in-loop hook exactly as written]. A pod's terms are
 * a term set (ms_nam_term_set / ms_nam_term_set_ext) registered with
 * ms_nam_term_sets(_ext); the pod record
 * names it by id = pref_zone | pref_weight << 8 (0 = no terms). Raw scores are
 * sums of matching term weights, up to 400, so the hook rescales earlier
 * entries whenever a later node's raw score exceeds 100. Terms
 * test the node's zone label (ms_node_rec.zone) or its second label
 * (ms_node_rec.label2). */
#define MS_PLUGINS_NU_NN_NAM 4

/* ---- modes --------------------------------------------------------------- */
#define MS_MODE_BATCHED 0    /* all pods of the call see the same node state               */
#define MS_MODE_SEQUENTIAL 1 /* queue order; each winner's NodeInfo.AddPod lands before the
                                next pod is decided (assume-on-select)                       */

/* ---- per-pod outcome (ms_result.code) ------------------------------------ */
#define MS_CODE_SUCCESS 0       /* node selected                                        */
#define MS_CODE_ERROR 1         /* framework.Error from a score plugin: NodeNumber with a
                                   non-digit pod name (nodenumber.go:53-56,74-77); the
                                   reference's ErrorFunc sees a non-FitError              */
#define MS_CODE_UNSCHEDULABLE 2 /* *framework.FitError (minisched.go:143-148)            */

/* ms_result.plugin_mask = FitError Diagnosis.UnschedulablePlugins */
#define MS_MASK_NODE_UNSCHEDULABLE (1u << 0) /* "NodeUnschedulable" */
#define MS_MASK_NODE_RESOURCES_FIT (1u << 1) /* "NodeResourcesFit"  */
#define MS_MASK_TAINT_TOLERATION (1u << 2)   /* "TaintToleration"   */

#define MS_MAX_ORDINAL 0xFFFFDu /* (keys 0 and 1 are reserved: no feasible node) */

/* Flat node record (v1.Node + framework.NodeInfo columns the plugins read).
 * 64 bytes. Resource columns are ignored by MS_PLUGINS_NU_NN. */
typedef struct ms_node_rec {
    uint8_t unschedulable; /* node.Spec.Unschedulable                              */
    uint8_t name_digit;    /* last char of node name as 0..9; 0xFF = not a digit     */
    uint8_t zone;          /* value id of the node's topology.kubernetes.io/zone
                              label, 0 = unlabelled (MS_PLUGINS_NU_NN_NA)           */
    uint8_t label2;        /* value id of the node's second label (the shim's key,
                              e.g. node.kubernetes.io/instance-type), 0 = unlabelled
                              (MS_PLUGINS_NU_NN_NAM term key 1)                      */
    int32_t allowed_pods;  /* NodeInfo.Allocatable.AllowedPodNumber                 */
    int32_t pod_count;     /* len(NodeInfo.Pods)                                    */
    uint32_t taints;       /* MS_PLUGINS_NU_TT_NN: taint ids (bits 0-7 NoSchedule /
                              NoExecute, bits 8-15 PreferNoSchedule); else ignored  */
    int64_t alloc_milli_cpu, alloc_memory;     /* NodeInfo.Allocatable             */
    int64_t req_milli_cpu, req_memory;         /* NodeInfo.Requested               */
    int64_t nonzero_milli_cpu, nonzero_memory; /* NodeInfo.NonZeroRequested        */
} ms_node_rec;

/* Flat pod record. 40 bytes. */
typedef struct ms_pod_rec {
    uint32_t ordinal;                /* stable pod id fed to the tie-break           */
    int8_t name_digit;               /* last char of pod name as 0..9; -1 = not     */
    uint8_t tolerates_unschedulable; /* TolerationsTolerateTaint(unschedulable:NoSchedule) */
    /* MS_PLUGINS_NU_NN_NA: one PreferredSchedulingTerm {weight, zone In [pref_zone]}
     * (NodeAffinity.Score = weight when the node's zone label matches); 0 = none.
     * MS_PLUGINS_NU_TT_NN: pref_zone = tol_hard, pref_weight = tol_soft (the
     * tolerated NoSchedule / PreferNoSchedule taint ids, see the plugin set). */
    uint8_t pref_zone;
    uint8_t pref_weight;             /* 1..100 (API validation of the term weight)  */
    int64_t req_milli_cpu, req_memory;         /* Fit PreFilter request              */
    int64_t nonzero_milli_cpu, nonzero_memory; /* GetNonzeroRequests sum            */
} ms_pod_rec;

/* Per-pod result. 24 bytes. */
typedef struct ms_result {
    int32_t node;         /* global ordinal of the selected node; -1 if none     */
    int32_t code;         /* MS_CODE_*                                            */
    int64_t score;        /* summed score of the selected node                    */
    uint32_t plugin_mask; /* MS_MASK_* when code == MS_CODE_UNSCHEDULABLE, else 0 */
    uint32_t _pad;
} ms_result;

/* Compact records for the plugin sets that read no resources (MS_PLUGINS_NU_NN,
 * MS_PLUGINS_NU_NN_NA): 8 bytes each way instead of 40 + 24, for
 * ms_schedule_batch_compact. ms_pod_compact is the first 8 bytes of ms_pod_rec;
 * its resource requests are zero (a bind adds one pod to len(NodeInfo.Pods)). */
typedef struct ms_pod_compact {
    uint32_t ordinal;
    int8_t name_digit;
    uint8_t tolerates_unschedulable;
    uint8_t pref_zone;
    uint8_t pref_weight;
} ms_pod_compact;

typedef struct ms_result_compact {
    int32_t node;        /* global ordinal; -1 if none                              */
    uint16_t score;      /* summed score (< 2048)                                   */
    uint8_t code;        /* MS_CODE_*                                               */
    uint8_t plugin_mask; /* MS_MASK_* when code == MS_CODE_UNSCHEDULABLE, else 0     */
} ms_result_compact;

typedef struct ms_config {
    int32_t device;      /* HIP device ordinal (within HIP_VISIBLE_DEVICES)     */
    int32_t plugin_set;  /* MS_PLUGINS_*                                        */
    uint32_t max_nodes;  /* node capacity of this context                       */
    uint32_t node_base;  /* global ordinal of local node 0 (shard offset)       */
    uint32_t max_batch;  /* pods per internal chunk of ms_schedule_batch        */
    /* score plugin weights (MS_PLUGINS_NU_NN_NA / _NAM only; 0 means 1): [0] NodeNumber,
     * [1] NodeAffinity. The reference sums unweighted ("TODO: plugin weight",
     * minisched.go:186); weights 1/1 reproduce it. w0*10 + w1*100 < 2048. */
    uint16_t score_weight[2];
    uint64_t seed;       /* tie-break seed                                      */
} ms_config;

typedef struct ms_info {
    uint32_t max_nodes, node_base;
    uint32_t present_nodes;  /* nodes currently in the table (not tombstoned)  */
    uint32_t pending_deltas; /* queued upserts/deletes not yet on the device   */
    int32_t device, plugin_set;
    uint64_t seed;
    /* exact sequential engine counters since ms_create (diagnostics):
     * pods validated, tiles re-swept, speculative entries re-evaluated */
    uint32_t seq_pods, seq_resweep_tiles, seq_recomputes, _pad;
    /* communicator (ms_comm_init): this context's rank and the world size;
     * both 0 when the context is not joined to one */
    int32_t comm_rank, comm_world;
} ms_info;

typedef struct ms_ctx ms_ctx;

int ms_abi_version(void);
int ms_device_count(int *out_count);

int ms_create(const ms_config *cfg, ms_ctx **out_ctx);
int ms_destroy(ms_ctx *ctx);
/* Message of the last failure on ctx (or of the last failed ms_create on this
 * thread when ctx is NULL). Never NULL. */
const char *ms_last_error(const ms_ctx *ctx);
int ms_get_info(const ms_ctx *ctx, ms_info *out);

/* Host-side phase times of the last ms_schedule_batch / ms_schedule_batch_compact
 * call on ctx (diagnostics: where a slow host call spent its wall time). ns[]
 * is indexed by MS_PH_*; every phase is host wall time inside the call, and
 * the phases sum to ns[MS_PH_TOTAL] up to the bookkeeping between them.
 * Thread-safe like the other entry points: it takes the scheduling lock, so
 * it waits for a call in progress on another thread and never returns a
 * partly written profile. */
#define MS_CALL_PHASES 8
enum {
    MS_PH_TOTAL = 0,      /* the whole call                                            */
    MS_PH_LOCK_FLUSH = 1, /* scheduling lock + drain of queued node deltas              */
    MS_PH_STAGE_IN = 2,   /* pods host -> staging / H2D enqueue (pageable: runtime copy) */
    MS_PH_LAUNCH = 3,     /* kernel launches of the cycle (and collectives)             */
    MS_PH_STAGE_OUT = 4,  /* D2H enqueue / results staging -> caller's array            */
    MS_PH_WAIT = 5,       /* blocked in stream synchronisation                          */
    MS_PH_ALLOC = 6,      /* (re)allocation of staging buffers                          */
    MS_PH_CHUNKS = 7      /* number of copy/cycle chunks (a count, not ns)              */
};
typedef struct ms_call_profile {
    uint64_t ns[MS_CALL_PHASES];
} ms_call_profile;
int ms_last_call_profile(const ms_ctx *ctx, ms_call_profile *out);

/* ---- node deltas (informer Add/Update/Delete, eventhandler.go:60-76) ------
 * Enqueued under a mutex (safe from informer goroutines while another thread
 * schedules); drained stream-ordered at the start of the next schedule call
 * or by ms_nodes_flush. Later deltas to one ordinal win. */
int ms_nodes_upsert(ms_ctx *ctx, uint32_t n, const uint32_t *ordinals, const ms_node_rec *recs);
int ms_nodes_delete(ms_ctx *ctx, uint32_t n, const uint32_t *ordinals);
int ms_nodes_flush(ms_ctx *ctx);
/* Device -> host read-back of [first, first+n) (global ordinals); absent
 * nodes read back with allowed_pods = -1. */
int ms_nodes_read(ms_ctx *ctx, uint32_t first, uint32_t n, ms_node_rec *out);

/* ---- the scheduling cycle ---------------------------------------------------
 * Replaces minisched.go:40-85 for n_pods pods in queue order. Host arrays,
 * copied to and from the device within the call (no pointer is kept after it
 * returns); out[i] is written before return. With
 * MS_MODE_SEQUENTIAL every SUCCESS commits NodeInfo.AddPod on its node before
 * the next pod is decided (bit-exact to the one-at-a-time loop). */
int ms_schedule_batch(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods, int32_t mode,
                      ms_result *out);

/* ms_schedule_batch with compact records (MS_PLUGINS_NU_NN / _NU_NN_NA only):
 * the same cycle, binds and results, with 8 B per pod over PCIe each way. */
int ms_schedule_batch_compact(ms_ctx *ctx, uint32_t n_pods, const ms_pod_compact *pods, int32_t mode,
                              ms_result_compact *out);

/* Assume / forget for the live scheduler (upstream cache.AssumePod/ForgetPod):
 * add / remove one pod's requests on a node. */
int ms_commit_bind(ms_ctx *ctx, uint32_t ordinal, const ms_pod_rec *pod);
int ms_uncommit_bind(ms_ctx *ctx, uint32_t ordinal, const ms_pod_rec *pod);

/* ---- device-resident entry points (bench, node-sharded multi-GPU) ---------
 * Pointers are device pointers; `stream` is a hipStream_t (NULL = the
 * context's own stream). Nothing is synchronised: the caller orders work on
 * the stream.
 *
 * ms_sweep_device: this shard's part of filter+score+selectHost for a batch.
 *   keys[i]  = max packed key over this shard's feasible nodes; with none, 1
 *              when this shard lists at least one node, else 0 (real keys
 *              are >= 2), so the MAX over the shards also tells the decode
 *              whether the cluster lists any node
 *   flags[i] = byte 0: some node here rejected by NodeUnschedulable (0/1),
 *              byte 1: some node here rejected by NodeResourcesFit  (0/1)
 *   Both arrays are overwritten. MS_PLUGINS_NU_NN takes no flags (NULL; the
 *   mask follows from the key and the cluster's present-node count).
 *   Shards combine keys with an element-wise uint64 MAX and flags with a
 *   byte-wise uint8 MAX (= OR of 0/1 bytes): one reduction each.
 *   MS_PLUGINS_NU_NN_NA: keys use raw NodeAffinity scores and flags[i] is the
 *   normalise anchor, ((0xFFFFF - ordinal) << 1 | NodeNumber match) + 1 of this
 *   shard's first feasible node with a non-zero NodeAffinity score (0 = none);
 *   shards combine it with an element-wise uint32 MAX.
 * ms_decode_device: combined keys/flags -> ms_result. present_nodes: the
 *   global count of present nodes, or 0 to take it from the combined key (1 =
 *   some node listed); used when flags is NULL.
 * ms_apply_binds_device: NodeInfo.AddPod on this shard for every SUCCESS
 *   in results (the batched-mode bind commit). */
int ms_sweep_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev, uint64_t *keys_dev,
                    uint32_t *flags_dev, void *stream);
int ms_decode_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev,
                     const uint64_t *keys_dev, const uint32_t *flags_dev, uint32_t present_nodes,
                     ms_result *results_dev, void *stream);
/* ms_decode_device_jobs: ms_decode_device for up to MS_DECODE_MAX_JOBS
 *   batches in one launch (jobs is a host array; its pointers are device
 *   pointers). Used by the pipelined multi-GPU step, which drains several
 *   batches' combined keys at once. Each job needs its own results array. */
#define MS_DECODE_MAX_JOBS 8
typedef struct ms_decode_job {
    const ms_pod_rec *pods;
    const uint64_t *keys;
    const uint32_t *flags; /* may be NULL (MS_PLUGINS_NU_NN) */
    ms_result *results;
    uint32_t n_pods;
    uint32_t _pad;
} ms_decode_job;
int ms_decode_device_jobs(ms_ctx *ctx, uint32_t n_jobs, const ms_decode_job *jobs, uint32_t present_nodes,
                          void *stream);
int ms_apply_binds_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev,
                          const ms_result *results_dev, void *stream);
/* ms_select_batch_device: the stateless batched cycle (filter + score +
 *   selectHost + decode) of a single-shard context on device-resident pods,
 *   with no bind commit: results_dev[i] as ms_schedule_batch would return it
 *   in MS_MODE_BATCHED. For NU+NN this is one fused kernel launch. Replaces
 *   minisched.go:40-85 for pods whose placements do not interact (config D).
 *   Node state the plugins read (NU, NN) is unchanged by binds, so for NU+NN
 *   it also equals the queue-order loop (minisched.go:28-30). */
int ms_select_batch_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev, ms_result *results_dev,
                           void *stream);
/* ---- node-sharded exact sequential mode (MS_PLUGINS_NU_NRF_NN_LA) ---------
 * Queue order with assume-on-select over nodes split across contexts (one per
 * GPU), batch after batch; every shard s runs, for pods [a, a + n):
 *   1. ms_seq_candidates_device: flushes deltas, then this shard's speculative
 *      top-4 per pod against its current table: cands[p*4 + r] (key 0 = none)
 *      with the node's record, and flags[p] = OR over this shard's nodes of
 *      the filter plugins rejecting them (byte 0 NU, byte 1 NRF).
 *   2. the caller all-gathers cands and flags over the shards (shard-major:
 *      cands_all[s][p][4], flags_all[s][p]) — one collective each;
 *   3. ms_seq_validate_device (identical on every shard): merges the shards'
 *      lists into each pod's global speculative top-4, walks the pods in queue
 *      order against them — a node bound earlier in the batch is re-evaluated
 *      from its record plus those binds, the first untouched entry is exact —
 *      and stops before the first pod the lists cannot decide (its four
 *      candidates all bound earlier, more nodes below them). Writes
 *      results[0, *n_done) and *n_done (>= 1 when n > 0), and commits the
 *      binds that land on this shard's own nodes (NodeInfo.AddPod), so every
 *      bind reaches its owner and no other shard. The caller continues at
 *      a + *n_done. No deltas are drained between 1 and 3. */
typedef struct ms_seq_cand {
    uint64_t key; /* packed key at speculation; 0 = no candidate */
    int64_t alloc_milli_cpu, alloc_memory, req_milli_cpu, req_memory, nonzero_milli_cpu, nonzero_memory;
    int32_t allowed_pods, pod_count;
    uint32_t flags_digit; /* bit0 unschedulable, bit7 absent | name digit << 8 */
    uint32_t _pad;
} ms_seq_cand; /* 72 bytes */
#define MS_SEQ_SHARD_BATCH_MAX 256u
#define MS_SEQ_MAX_SHARDS 16u
int ms_seq_candidates_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev, ms_seq_cand *cands_dev,
                             uint32_t *flags_dev, void *stream);
int ms_seq_validate_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev, uint32_t n_shards,
                           const ms_seq_cand *cands_all_dev, const uint32_t *flags_all_dev, ms_result *results_dev,
                           uint32_t *n_done_dev, void *stream);
/* ---- node-sharded MS_PLUGINS_NU_TT_NN ---------------------------------------
 * TaintToleration's in-loop reverse normalisation makes a node's score depend
 * on its rank among the pod's feasible nodes in LIST order, so shards do not
 * combine by a MAX. Instead every shard writes, per pod, a summary of its
 * nodes (MS_TT_SUMMARY_BYTES, opaque: feasible count, filter flags, the first
 * three and the last feasible node, the best node per (raw count, rank
 * parity) class); summaries of consecutive shards merge associatively, and
 * the decode applies the closed form of the loop and selectHost.
 *   1. ms_tt_summaries_device: this shard's summaries (summaries_dev: n_pods x
 *      MS_TT_SUMMARY_BYTES);
 *   2. the caller gathers them shard-major (summaries_all[s][p], shards in
 *      ordinal order = LIST order);
 *   3. ms_tt_decode_device: the merge over the n_shards shards and each pod's
 *      result (no bind commit). */
#define MS_TT_SUMMARY_BYTES 192u
int ms_tt_summaries_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev, void *summaries_dev,
                           void *stream);
int ms_tt_decode_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev, uint32_t n_shards,
                        const void *summaries_all_dev, ms_result *results_dev, void *stream);
/* The same cycle in the two-pass bit-sliced form (ABI 6): per
 * pod a 32-byte census of the shard's nodes (feasible count, filter flags, the
 * first three and the last feasible node, which (raw count, rank parity)
 * classes occur, with and without a NodeNumber match), then a key per pod from
 * every shard's census and its own rows, combined by uint64 MAX like NU+NN:
 *   1. ms_tt_census_device: this shard's census (census_dev: n_pods x
 *      MS_TT_CENSUS_BYTES);
 *   2. the caller gathers them shard-major (census_all[s][p], shards in
 *      ordinal order = LIST order);
 *   3. ms_tt_pick_device: this shard's keys (keys_dev, n_pods x u64) under the
 *      plan every shard's census implies;
 *   4. the element-wise uint64 MAX of the shards' keys;
 *   5. ms_tt_final_device (any shard): each pod's result (no bind commit). */
#define MS_TT_CENSUS_BYTES 32u
int ms_tt_census_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev, void *census_dev, void *stream);
int ms_tt_pick_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev, uint32_t n_shards,
                      uint32_t shard_index, const void *census_all_dev, unsigned long long *keys_dev, void *stream);
int ms_tt_final_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev, uint32_t n_shards,
                       const void *census_all_dev, const unsigned long long *keys_max_dev, ms_result *results_dev,
                       void *stream);

/* ---- MS_PLUGINS_NU_NN_NAM: several preferred NodeAffinity terms ----------- */
/* One PreferredSchedulingTerm: its NodeSelectorTerm tests one node label
 * (key 0: ms_node_rec.zone, 1: ms_node_rec.label2) with operator In [value]
 * (value id 1..254) or Exists (value 0xFF); weight 1..100, 0 = unused slot. */
typedef struct ms_pref_term {
    uint8_t key, value, weight, _pad;
} ms_pref_term;
#define MS_NAM_TERMS 4
typedef struct ms_nam_term_set {
    ms_pref_term term[MS_NAM_TERMS];
} ms_nam_term_set; /* 16 bytes */
/* Registers the context's term sets: pod term set id s (1..n_sets) is
 * sets[s - 1]; ids above n_sets count as no terms. Copied; replaces the
 * previous table (stream-ordered after earlier calls). Up to 65535 sets. */
int ms_nam_term_sets(ms_ctx *ctx, uint32_t n_sets, const ms_nam_term_set *sets);
/* The same in general form (ABI 7): a PreferredSchedulingTerm whose
 * NodeSelectorTerm holds any NodeSelectorRequirements (In, NotIn, Exists,
 * DoesNotExist, Gt, Lt; several per term, ANDed) on the two encoded label keys
 * (0: the zone label, ms_node_rec.zone; 1: the second label, label2). Per key,
 * mask[key] is the set of value ids of nodes that satisfy every requirement of
 * the term on that key: bit (v & 31) of mask[key][v >> 5] for value id v, id 0 =
 * the node lacks the label; all ones when the term has no requirement on the
 * key. The term matches a node when both masks hold the node's ids; a term with
 * no requirement at all matches no node (k8s@v1.22.0 component-helpers
 * nodeaffinity: an empty nodeSelectorTerm matches nothing), so the shim gives it
 * zero masks. weight 1..100, 0 = unused slot. Value ids are the shim's (the same
 * table as the node records'); it re-registers its sets when the table grows,
 * since Exists, NotIn, DoesNotExist, Gt and Lt also cover ids it had not seen.
 * ms_nam_term_sets' {key, value} terms are the masks {value} (In) or all ids
 * but 0 (Exists, value 0xFF) on that key and all ones on the other. */
typedef struct ms_pref_term_ext {
    uint32_t mask[2][8];
    uint8_t weight, _pad[3];
} ms_pref_term_ext; /* 68 bytes */
typedef struct ms_nam_term_set_ext {
    ms_pref_term_ext term[MS_NAM_TERMS];
} ms_nam_term_set_ext; /* 272 bytes */
int ms_nam_term_sets_ext(ms_ctx *ctx, uint32_t n_sets, const ms_nam_term_set_ext *sets);
/* Node shards (contexts with their own node_base, ordinals = LIST order) of
 * one MS_PLUGINS_NU_NN_NAM cycle, for a caller with its own collectives:
 *   1. ms_nam_segment_device: per pod, this shard's rescale composition (an
 *      opaque MS_NAM_SEG_BYTES record: the composed map of its nodes' in-loop
 *      rescales on 0..100 and whether a feasible node scored > 0);
 *   2. the caller gathers them shard-major (segs_all[s][p], shards in ordinal
 *      order);
 *   3. ms_nam_keys_device: this shard's packed keys (keys_dev, n_pods x u64) of
 *      the pods' FINAL scores: its nodes' raw scores through the rescales of
 *      every later node of the cluster, the first non-zero node of the cluster
 *      at 100. The element-wise uint64 MAX over the shards is selectHost over
 *      the cluster; ms_decode_device (flags NULL) turns it into results. */
#define MS_NAM_SEG_BYTES 104u
int ms_nam_segment_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev, void *seg_dev, void *stream);
int ms_nam_keys_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev, uint32_t n_shards,
                       uint32_t shard_index, const void *segs_all_dev, unsigned long long *keys_dev, void *stream);

/* Whole exact sequential cycle on device-resident pods (single shard; on a
 * context joined to a communicator, the node-sharded cycle below). */
int ms_schedule_sequential_device(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev,
                                  ms_result *results_dev, void *stream);

/* ---- multi-GPU inside the library: one RCCL communicator per job ------------
 * One process (or host thread) per GPU, one context per rank, each owning the
 * contiguous node shard [node_base, node_base + max_nodes) of the cluster's
 * ordinals (ranks in ordinal order; the shards need not be equal). Rank 0
 * creates an id with ms_comm_id_create and hands its bytes to every rank out
 * of band; every rank then calls ms_comm_init (collective: it returns once all
 * ranks joined). The context then owns the communicator and its collective
 * stream, and frees them in ms_destroy. Replaces selectHost over the union of
 * the shards (minisched.go:304-325): keys embed the global ordinal, so the
 * MAX reduction equals the single-GPU argmax whatever the tree.
 *
 * With a communicator, ms_schedule_batch and ms_schedule_sequential_device are
 * collective: every rank calls them with the same pods (queue order) and gets
 * every pod's result; each rank commits the binds that land on its own nodes.
 *   batched (and NU+NN / NodeAffinity sequential, which equal it): this
 *   shard's sweep, ONE grouped reduce-scatter (uint64 MAX of the packed keys,
 *   the filter bytes / uint32 NodeAffinity anchors, the "a node is listed"
 *   flag), the decode of this rank's pod slice, an all-gather of the results;
 *   resource-aware sequential: per batch of pods, every shard's speculative
 *   top-4 with records, one grouped all-gather, the replicated in-order
 *   validation (ms_seq_* above); the queue cursor stays on the device, so
 *   batches are issued without a host round trip (the host reads the cursor
 *   once per round of ceil(remaining / batch) batches).
 * ms_select_batch_device is single-shard and fails on such a context. */
#define MS_COMM_ID_BYTES 128
typedef struct ms_comm_id {
    char internal[MS_COMM_ID_BYTES]; /* ncclUniqueId */
} ms_comm_id;
int ms_comm_id_create(ms_comm_id *out);
int ms_comm_init(ms_ctx *ctx, const ms_comm_id *id, int32_t rank, int32_t world);

/* Pipelined node-sharded batched cycle on device-resident pods (the bench's
 * and a service loop's step). ms_sharded_submit sweeps this shard on `stream`
 * (after the work already there: the pods), runs the batch's collective on the
 * context's collective stream (the grouped reduce-scatter; for
 * MS_PLUGINS_NU_TT_NN an all-to-all of the per-pod summaries) and, once more
 * than the pipeline depth (4) batches are in flight, decodes the oldest ones
 * on the context's decode stream: batch k's collective overlaps the sweeps of
 * the following batches. ms_sharded_drain decodes every remaining batch and
 * makes `stream` wait for all decodes. results_dev receives this rank's pod
 * slice [first, first + count) of the batch (ms_sharded_slice) and is
 * complete once the stream work of a later ms_sharded_drain completes.
 * pods_dev must stay valid AND UNMODIFIED until then: the decode of a batch
 * reads its pods (name digit, ordinal) up to `depth` submits later, so a loop
 * that refills pod buffers rotates at least depth + 1 of them.
 * Every rank submits the same batches in the same order. No binds are
 * committed (stateless: NU+NN, NodeAffinity, TaintToleration; for the
 * resource-aware set each batch sees the state of its submit). Deltas and
 * binds issued meanwhile wait for the sweeps in flight. For MS_PLUGINS_NU_NN
 * two consecutive submits on one stream share ONE sweep launch: a submission's
 * sweep may be enqueued only by the next submit (or by a drain, a node delta
 * flush or any other call on the context, which sweep it alone first), so
 * the stream carries its work only after that call; its collective and the
 * order of collectives are unchanged (MINISCHED_SHARD_COALESCE=0: one launch
 * per submit). */
int ms_sharded_slice(const ms_ctx *ctx, uint32_t n_pods, uint32_t *first, uint32_t *count);
int ms_sharded_submit(ms_ctx *ctx, uint32_t n_pods, const ms_pod_rec *pods_dev, ms_result *results_dev,
                      void *stream);
int ms_sharded_drain(ms_ctx *ctx, void *stream);

#ifdef __cplusplus
}
#endif
#endif
