/*
 * ms_oracle.c — CPU restatement of minisched's scheduling cycle.
 *
 * TEST INFRASTRUCTURE ONLY (see ms_oracle.h for the parity status). Each
 * function names the reference file:line it restates. Citations of the form
 * k8s@v1.22.0:<path> are upstream Kubernetes sources that are NOT in the
 * container (the submodule is empty, .gitmodules:1-3); they are restated from
 * the published v1.22.0 code.
 */
#include "ms_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- tie-break (replaces minisched.go:316-321 rand.Intn reservoir) -------- */

uint32_t msor_fmix32(uint32_t h) { /* murmur3 finaliser */
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

uint32_t msor_seed32(uint64_t seed) { return (uint32_t)(seed ^ (seed >> 32)); }

uint32_t msor_pod_hash(uint64_t seed, uint32_t pod_ordinal) {
    return msor_fmix32(msor_seed32(seed) ^ pod_ordinal);
}

/* murmur3-style mixer: two xor-shifts by 16 around the fmix32 multipliers */
uint32_t msor_mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x85ebca6bu;
    x ^= x >> 16;
    x *= 0xc2b2ae35u;
    return x;
}

/* Tie-break hash, rule "r3" (include/minisched_gpu.h): the pod half A is
 * msor_pod_hash and the node enters additively as ordinal * 0x9E3779 (a 24-bit
 * odd constant). For one pod it is a bijection of the node ordinal, so two
 * nodes never tie on it. */
uint32_t msor_tb_hash(uint32_t pod_hash, uint32_t node) {
    return msor_mix32(pod_hash + node * 0x9E3779u);
}

uint32_t msor_h32(uint64_t seed, uint32_t pod, uint32_t node) {
    return msor_tb_hash(msor_pod_hash(seed, pod), node);
}

/* key = score<<52 | h32<<20 | (0xFFFFF - ordinal); max wins. */
uint64_t msor_key(int64_t score, uint32_t h, uint32_t node) {
    return ((uint64_t)score << 52) | ((uint64_t)h << 20) | (uint64_t)(0xFFFFFu - node);
}

/* ---- upstream LeastAllocated ---------------------------------------------- */
/* k8s@v1.22.0:pkg/scheduler/framework/plugins/noderesources/least_allocated.go
 * leastRequestedScore: capacity 0 -> 0; requested > capacity -> 0;
 * else ((capacity - requested) * MaxNodeScore) / capacity (int64 floor). */
int64_t msor_least_requested(int64_t requested, int64_t capacity) {
    if (capacity == 0) return 0;
    if (requested > capacity) return 0;
    return ((capacity - requested) * 100) / capacity;
}

/* ---- NodeUnschedulable.Filter -------------------------------------------- */
/* k8s@v1.22.0:pkg/scheduler/framework/plugins/nodeunschedulable/
 * node_unschedulable.go: Spec.Unschedulable && !TolerationsTolerateTaint(
 * {node.kubernetes.io/unschedulable, NoSchedule}) -> UnschedulableAndUnresolvable.
 * The toleration match itself is evaluated once per pod on the host
 * (pod->tol), exactly as upstream evaluates it once per Filter call. */
static int nu_rejects(uint8_t flags, uint8_t tol) {
    return (flags & MSOR_NODE_UNSCHEDULABLE) && !tol;
}

/* ---- NodeResourcesFit.Filter (fitsRequest) -------------------------------- */
/* k8s@v1.22.0:pkg/scheduler/framework/plugins/noderesources/fit.go fitsRequest:
 * "Too many pods" when len(Pods)+1 > AllowedPodNumber; if every pod request is
 * zero only that check applies; else MilliCPU > Allocatable-Requested or
 * Memory > Allocatable-Requested -> Unschedulable. */
static int nrf_rejects(const msor_nodes *nd, uint32_t i, const msor_pods *pd, uint32_t j) {
    int bad = 0;
    if (nd->pod_count[i] + 1 > nd->allowed_pods[i]) bad = 1;
    int64_t rc = pd->req_cpu[j], rm = pd->req_mem[j];
    if (rc == 0 && rm == 0) return bad;
    if (rc > nd->alloc_cpu[i] - nd->req_cpu[i]) bad = 1;
    if (rm > nd->alloc_mem[i] - nd->req_mem[i]) bad = 1;
    return bad;
}

/* ---- LeastAllocated score (cpu weight 1, memory weight 1) ------------------ */
/* k8s@v1.22.0:.../noderesources/resource_allocation.go score +
 * calculateResourceAllocatableRequest: requested = NonZeroRequested + pod
 * non-zero request; weights pinned at scheduler/plugin/plugins_test.go:839-858. */
static int64_t la_score(const msor_nodes *nd, uint32_t i, const msor_pods *pd, uint32_t j) {
    int64_t s_cpu = msor_least_requested(nd->nz_cpu[i] + pd->nz_cpu[j], nd->alloc_cpu[i]);
    int64_t s_mem = msor_least_requested(nd->nz_mem[i] + pd->nz_mem[j], nd->alloc_mem[i]);
    return (s_cpu * 1 + s_mem * 1) / 2;
}

/* ---- NodeNumber.Score ----------------------------------------------------- */
/* minisched/plugins/score/nodenumber/nodenumber.go:73-95: 10 when the pod's
 * last-char digit equals the node's, 0 otherwise (0 also for a non-digit node
 * name). A non-digit POD name makes PreScore skip CycleState.Write
 * (nodenumber.go:53-56) so Score returns framework.Error (:74-77). */
static int nn_score(int8_t pod_digit, uint8_t node_digit) {
    return (node_digit != 0xFF && (int)node_digit == (int)pod_digit) ? 10 : 0;
}

static int has_resources(const msor_nodes *nd) {
    return nd->allowed_pods && nd->pod_count && nd->alloc_cpu && nd->alloc_mem && nd->req_cpu &&
           nd->req_mem && nd->nz_cpu && nd->nz_mem;
}

/* One scheduling cycle for pod j: minisched.go:32-85 between NewCycleState
 * (:37) and selectHost (:80), with the deterministic tie-break. */
static void schedule_one(msor_nodes *nd, const msor_pods *pd, uint32_t j, int plugin_set,
                         uint64_t seed, uint32_t node_base, int32_t *o_node, int64_t *o_score,
                         int32_t *o_code, uint32_t *o_mask, uint64_t *o_key) {
    uint32_t mask = 0, feasible = 0;
    uint64_t best = 0;
    const uint32_t ph = msor_pod_hash(seed, pd->ordinal[j]);
    const int8_t pdig = pd->digit[j];
    /* RunFilterPlugins (minisched.go:115-151): every node in LIST order, the
     * first failing plugin of a node is recorded (:130-137). Score plugins
     * (:164-199) and the unweighted sum (:187-196) are folded into the same
     * pass: scores of infeasible nodes are never used. */
    for (uint32_t i = 0; i < nd->n; ++i) {
        uint8_t f = nd->flags[i];
        if (f & MSOR_NODE_ABSENT) continue; /* not in Nodes().List (minisched.go:40) */
        if (nu_rejects(f, pd->tol[j])) { mask |= MSOR_MASK_NU; continue; }
        if (plugin_set == MSOR_PLUGINS_NU_NRF_NN_LA && nrf_rejects(nd, i, pd, j)) {
            mask |= MSOR_MASK_NRF;
            continue;
        }
        ++feasible;
        int64_t score = nn_score(pdig, nd->digit[i]);
        if (plugin_set == MSOR_PLUGINS_NU_NRF_NN_LA) score += la_score(nd, i, pd, j);
        uint32_t ord = node_base + i;
        uint64_t key = msor_key(score, msor_tb_hash(ph, ord), ord);
        if (key > best) best = key; /* selectHost (minisched.go:304-325) */
    }
    *o_mask = 0;
    *o_key = best;
    if (feasible == 0) { /* FitError (minisched.go:143-148) */
        *o_code = MSOR_CODE_UNSCHEDULABLE;
        *o_mask = mask;
        *o_node = -1;
        *o_score = 0;
        return;
    }
    if (pdig < 0) { /* NodeNumber.Score error -> RunScorePlugins aborts (:170-172) */
        *o_code = MSOR_CODE_ERROR;
        *o_node = -1;
        *o_score = 0;
        return;
    }
    *o_code = MSOR_CODE_SUCCESS;
    *o_node = (int32_t)(0xFFFFFu - (uint32_t)(best & 0xFFFFFu));
    *o_score = (int64_t)(best >> 52);
}

int msor_schedule(msor_nodes *nd, const msor_pods *pd, int plugin_set, int mode, uint64_t seed,
                  uint32_t node_base, int32_t *out_node, int64_t *out_score, int32_t *out_code,
                  uint32_t *out_mask, uint64_t *out_key) {
    if (!nd || !pd || !nd->flags || !nd->digit || !pd->ordinal || !pd->digit || !pd->tol) return -1;
    if (plugin_set != MSOR_PLUGINS_NU_NN && plugin_set != MSOR_PLUGINS_NU_NRF_NN_LA) return -1;
    if (mode != MSOR_MODE_BATCHED && mode != MSOR_MODE_SEQUENTIAL) return -1;
    const int res = has_resources(nd);
    if (plugin_set == MSOR_PLUGINS_NU_NRF_NN_LA &&
        (!res || !pd->req_cpu || !pd->req_mem || !pd->nz_cpu || !pd->nz_mem))
        return -1;
    if ((uint64_t)node_base + nd->n >= 0xFFFFFu) return -1;
    for (uint32_t j = 0; j < pd->n; ++j) {
        int32_t node, code;
        int64_t score;
        uint32_t mask;
        uint64_t key;
        schedule_one(nd, pd, j, plugin_set, seed, node_base, &node, &score, &code, &mask, &key);
        if (out_node) out_node[j] = node;
        if (out_score) out_score[j] = score;
        if (out_code) out_code[j] = code;
        if (out_mask) out_mask[j] = mask;
        if (out_key) out_key[j] = key;
        /* assume-on-select: upstream NodeInfo.AddPod / calculateResource
         * (k8s@v1.22.0:pkg/scheduler/framework/types.go) on the winner only. */
        if (mode == MSOR_MODE_SEQUENTIAL && code == MSOR_CODE_SUCCESS && res && pd->req_cpu) {
            uint32_t i = (uint32_t)node - node_base;
            nd->req_cpu[i] += pd->req_cpu[j];
            nd->req_mem[i] += pd->req_mem[j];
            nd->nz_cpu[i] += pd->nz_cpu[j];
            nd->nz_mem[i] += pd->nz_mem[j];
            nd->pod_count[i] += 1;
        } else if (mode == MSOR_MODE_SEQUENTIAL && code == MSOR_CODE_SUCCESS && nd->pod_count) {
            nd->pod_count[(uint32_t)node - node_base] += 1;
        }
    }
    return 0;
}

int msor_schedule_nunn_omp(const msor_nodes *nd, const msor_pods *pd, uint64_t seed,
                           uint32_t node_base, int threads, int32_t *out_node,
                           int64_t *out_score, int32_t *out_code, uint32_t *out_mask,
                           uint64_t *out_key) {
    if (!nd || !pd || !nd->flags || !nd->digit || !pd->ordinal || !pd->digit || !pd->tol) return -1;
    if ((uint64_t)node_base + nd->n >= 0xFFFFFu) return -1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
    const long np = (long)pd->n;
#pragma omp parallel for schedule(dynamic, 16)
    for (long j = 0; j < np; ++j) {
        int32_t node, code;
        int64_t score;
        uint32_t mask;
        uint64_t key;
        schedule_one((msor_nodes *)nd, pd, (uint32_t)j, MSOR_PLUGINS_NU_NN, seed, node_base,
                     &node, &score, &code, &mask, &key);
        if (out_node) out_node[j] = node;
        if (out_score) out_score[j] = score;
        if (out_code) out_code[j] = code;
        if (out_mask) out_mask[j] = mask;
        if (out_key) out_key[j] = key;
    }
    return 0;
}

/* ---- reference-shaped single-thread form ---------------------------------- */

/* strconv.Atoi of a one-character string: only '0'..'9' parse. */
static int atoi_last_char(const char *s, int *ok) {
    size_t n = strlen(s);
    char c = n ? s[n - 1] : '\0';
    if (c >= '0' && c <= '9') { *ok = 1; return c - '0'; }
    *ok = 0;
    return 0;
}

typedef struct { const char *name; uint32_t ord; int64_t score; } node_score;

int msor_schedule_nunn_names(const char *const *node_names, const uint8_t *node_flags,
                             uint32_t n_nodes, const char *const *pod_names,
                             const uint8_t *pod_tol, const uint32_t *pod_ordinal,
                             uint32_t n_pods, uint64_t seed, int32_t *out_node,
                             int64_t *out_score, int32_t *out_code, uint32_t *out_mask) {
    if (n_nodes >= 0xFFFFFu) return -1;
    uint32_t *feasible = (uint32_t *)malloc(sizeof(uint32_t) * (n_nodes ? n_nodes : 1));
    node_score *list = (node_score *)malloc(sizeof(node_score) * (n_nodes ? n_nodes : 1));
    if (!feasible || !list) { free(feasible); free(list); return -1; }
    for (uint32_t j = 0; j < n_pods; ++j) {
        /* RunFilterPlugins (minisched.go:115-151) */
        uint32_t F = 0, mask = 0;
        for (uint32_t i = 0; i < n_nodes; ++i) {
            if (node_flags[i] & MSOR_NODE_ABSENT) continue;
            if (nu_rejects(node_flags[i], pod_tol[j])) { mask |= MSOR_MASK_NU; continue; }
            feasible[F++] = i;
        }
        out_mask[j] = 0;
        if (F == 0) {
            out_code[j] = MSOR_CODE_UNSCHEDULABLE; out_mask[j] = mask;
            out_node[j] = -1; out_score[j] = 0;
            continue;
        }
        /* RunPreScorePlugins -> NodeNumber.PreScore (nodenumber.go:50-64) */
        int pod_ok;
        int podnum = atoi_last_char(pod_names[j], &pod_ok);
        /* RunScorePlugins (minisched.go:164-199): per node, Score(pod, n.Name) */
        int err = 0;
        for (uint32_t k = 0; k < F; ++k) {
            if (!pod_ok) { err = 1; break; } /* CycleState.Read fails (:74-77) */
            int node_ok;
            int nodenum = atoi_last_char(node_names[feasible[k]], &node_ok);
            list[k].name = node_names[feasible[k]];
            list[k].ord = feasible[k];
            list[k].score = (node_ok && podnum == nodenum) ? 10 : 0;
        }
        if (err) {
            out_code[j] = MSOR_CODE_ERROR; out_node[j] = -1; out_score[j] = 0;
            continue;
        }
        /* selectHost (minisched.go:304-325) with the packed-key tie-break */
        const uint32_t ph = msor_pod_hash(seed, pod_ordinal[j]);
        uint64_t best = 0;
        uint32_t best_k = 0;
        for (uint32_t k = 0; k < F; ++k) {
            uint64_t key = msor_key(list[k].score, msor_tb_hash(ph, list[k].ord),
                                    list[k].ord);
            if (key > best) { best = key; best_k = k; }
        }
        out_code[j] = MSOR_CODE_SUCCESS;
        out_node[j] = (int32_t)list[best_k].ord;
        out_score[j] = list[best_k].score;
    }
    free(feasible);
    free(list);
    return 0;
}

/* ---- NodeAffinity (preferred terms) + the in-loop normalise hook ---------- */

/* k8s@v1.22.0:pkg/scheduler/framework/plugins/helper/normalize_score.go
 * DefaultNormalizeScore: maxCount = max score; 0 -> (reverse: all maxPriority)
 * unchanged; else score = maxPriority * score / maxCount, reversed as
 * maxPriority - score. */
void msor_default_normalize(int64_t max_priority, int reverse, int64_t *scores, uint32_t n) {
    int64_t max_count = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (scores[i] > max_count) max_count = scores[i];
    if (max_count == 0) {
        if (reverse)
            for (uint32_t i = 0; i < n; ++i) scores[i] = max_priority;
        return;
    }
    for (uint32_t i = 0; i < n; ++i) {
        int64_t sc = max_priority * scores[i] / max_count;
        if (reverse) sc = max_priority - sc;
        scores[i] = sc;
    }
}

/* k8s@v1.22.0:pkg/scheduler/framework/plugins/nodeaffinity/node_affinity.go
 * Score: the sum of the weights of the pod's PreferredSchedulingTerms whose
 * selector matches the node; here one term {weight, zone In [pref_zone]}. */
static int64_t na_raw(const msor_nodes *nd, uint32_t i, const msor_pods *pd, uint32_t j) {
    const uint8_t z = pd->pref_zone[j];
    return (z != 0 && nd->zone[i] == z) ? (int64_t)pd->pref_weight[j] : 0;
}

int msor_schedule_na(const msor_nodes *nd, const msor_pods *pd, int64_t w_nn, int64_t w_na, int literal,
                     uint64_t seed, uint32_t node_base, int32_t *out_node, int64_t *out_score,
                     int32_t *out_code, uint32_t *out_mask, uint64_t *out_key) {
    if (!nd || !pd || !nd->flags || !nd->digit || !nd->zone || !pd->ordinal || !pd->digit || !pd->tol ||
        !pd->pref_zone || !pd->pref_weight)
        return -1;
    if ((uint64_t)node_base + nd->n >= 0xFFFFFu) return -1;
    uint32_t *feas = (uint32_t *)malloc(sizeof(uint32_t) * (nd->n ? nd->n : 1));
    int64_t *nn = (int64_t *)malloc(sizeof(int64_t) * (nd->n ? nd->n : 1));
    int64_t *na = (int64_t *)malloc(sizeof(int64_t) * (nd->n ? nd->n : 1));
    if (!feas || !nn || !na) { free(feas); free(nn); free(na); return -1; }
    for (uint32_t j = 0; j < pd->n; ++j) {
        /* RunFilterPlugins (minisched.go:115-151): NodeUnschedulable only */
        uint32_t F = 0, mask = 0;
        for (uint32_t i = 0; i < nd->n; ++i) {
            if (nd->flags[i] & MSOR_NODE_ABSENT) continue;
            if (nu_rejects(nd->flags[i], pd->tol[j])) { mask |= MSOR_MASK_NU; continue; }
            feas[F++] = i;
        }
        int32_t node = -1, code;
        int64_t score = 0;
        uint64_t best = 0;
        if (F == 0) {
            code = MSOR_CODE_UNSCHEDULABLE;
        } else if (pd->digit[j] < 0) { /* NodeNumber.Score fails at the first node (:170-172) */
            code = MSOR_CODE_ERROR;
            mask = 0;
            best = 1; /* any non-zero key: F > 0 */
        } else {
            /* RunScorePlugins (minisched.go:164-185): createPluginToNodeScores
             * zero-fills both lists (:327-334); for each feasible node in order,
             * NodeNumber then NodeAffinity score it, and NodeAffinity's
             * NormalizeScore runs on its whole list right away (:178-183). */
            memset(na, 0, sizeof(int64_t) * F);
            int first = -1;
            for (uint32_t k = 0; k < F; ++k) {
                nn[k] = nn_score(pd->digit[j], nd->digit[feas[k]]);
                na[k] = na_raw(nd, feas[k], pd, j);
                if (literal) {
                    msor_default_normalize(100, 0, na, k + 1); /* entries > k are still 0 */
                } else if (first < 0 && na[k] > 0) {
                    first = (int)k;
                }
            }
            if (!literal && first >= 0) na[first] = 100;
            /* sum (:187-196), weights applied; selectHost (:304-325) */
            const uint32_t ph = msor_pod_hash(seed, pd->ordinal[j]);
            for (uint32_t k = 0; k < F; ++k) {
                const uint32_t ord = node_base + feas[k];
                const uint64_t key = msor_key(w_nn * nn[k] + w_na * na[k], msor_tb_hash(ph, ord), ord);
                if (key > best) best = key;
            }
            code = MSOR_CODE_SUCCESS;
            mask = 0;
            node = (int32_t)(0xFFFFFu - (uint32_t)(best & 0xFFFFFu));
            score = (int64_t)(best >> 52);
        }
        if (code == MSOR_CODE_ERROR) best = 0, node = -1;
        if (out_node) out_node[j] = node;
        if (out_score) out_score[j] = score;
        if (out_code) out_code[j] = code;
        if (out_mask) out_mask[j] = code == MSOR_CODE_UNSCHEDULABLE ? mask : 0;
        if (out_key) out_key[j] = best;
    }
    free(feas);
    free(nn);
    free(na);
    return 0;
}

/* ---- NodeAffinity with several preferred terms (plugin set 4) ------------- */

/* k8s@v1.22.0:pkg/scheduler/framework/plugins/nodeaffinity/node_affinity.go
 * Score: for each PreferredSchedulingTerm with a non-zero weight whose
 * NodeSelectorTerm matches the node, count += weight. A term (general form,
 * MSOR_NAM_EXT_BYTES per set) holds per label key (0: the zone label, 1: the
 * second label) the set of value ids for which every requirement of the term on
 * that key holds (id 0 = the label is absent; the shim derives the sets from
 * In / NotIn / Exists / DoesNotExist / Gt / Lt, tests/_pyref.py restates those
 * on label strings); it matches a node whose two ids are both in its sets. */
static int nam_bit(const uint8_t *mask, uint32_t v) { /* bit v of 8 little-endian u32 words */
    return (mask[4 * (v >> 5) + ((v & 31u) >> 3)] >> (v & 7u)) & 1;
}
static int64_t nam_raw(const msor_nodes *nd, uint32_t i, const uint8_t *set) {
    int64_t r = 0;
    for (int t = 0; t < MSOR_NAM_TERMS; ++t) {
        const uint8_t *term = set + MSOR_NAM_TERM_BYTES * t;
        const uint8_t w = term[64];
        if (w == 0) continue;
        if (nam_bit(term, nd->zone[i]) && nam_bit(term + 32, nd->label2[i])) r += w;
    }
    return r;
}

/* The 16-B form {key, value, weight, 0} x 4 (In [value] or Exists on one key) as
 * the general form: that key's set is {value} or every id but 0, the other's all. */
static void nam_set_to_ext(const uint8_t *set, uint8_t *ext) {
    memset(ext, 0, MSOR_NAM_EXT_BYTES);
    for (int t = 0; t < MSOR_NAM_TERMS; ++t) {
        const uint8_t key = set[4 * t], val = set[4 * t + 1], w = set[4 * t + 2];
        uint8_t *term = ext + MSOR_NAM_TERM_BYTES * t;
        if (w == 0 || val == 0) continue; /* unused slot, or "unlabelled": never matches */
        uint8_t *km = term + 32 * (key ? 1 : 0), *om = term + 32 * (key ? 0 : 1);
        memset(om, 0xFF, 32);
        if (val == 0xFF) {
            memset(km, 0xFF, 32);
            km[0] &= 0xFEu;
        } else {
            km[val >> 3] |= (uint8_t)(1u << (val & 7u));
        }
        term[64] = w;
    }
}

/* Closed form of the in-loop hook for reverse=false: once an
 * entry is non-zero the list maximum is 100 after every step, so step i is the
 * identity when r_i <= 100 and the rescale f_{r_i}(v) = floor(100 v / r_i) of
 * every earlier entry when r_i > 100 (entry i itself ends at 100); the first
 * non-zero entry (the anchor) starts at 100 whatever its raw score. Entry k
 * therefore ends at T_{>k}(v_k), T_{>k} = the composition of the later
 * rescales: computed by one reverse scan keeping T as a 101-entry table
 * (T <- T o f_r at each rescale; every f_r maps 1..100 below itself, so T
 * reaches 0 everywhere after at most 100 rescales and stays there). */
static void nam_closed(const int64_t *r, uint32_t F, int64_t *out) {
    int64_t T[101], U[101];
    for (int v = 0; v <= 100; ++v) T[v] = v;
    int64_t anchor = -1;
    for (uint32_t k = 0; k < F; ++k)
        if (r[k] > 0) { anchor = k; break; }
    for (int64_t k = (int64_t)F - 1; k >= 0; --k) {
        const int64_t v = (k == anchor || r[k] > 100) ? 100 : r[k];
        out[k] = T[v];
        if (r[k] > 100 && T[100] != 0) {
            for (int v2 = 0; v2 <= 100; ++v2) U[v2] = T[(100 * v2) / r[k]];
            memcpy(T, U, sizeof(T));
        }
    }
}

int msor_nam_inloop(const int64_t *r, uint32_t F, int literal, int64_t *out) {
    for (uint32_t k = 0; k < F; ++k)
        if (r[k] < 0) return -1;
    if (literal) {
        for (uint32_t k = 0; k < F; ++k) out[k] = 0; /* createPluginToNodeScores (:327-334) */
        for (uint32_t k = 0; k < F; ++k) {
            out[k] = r[k];
            msor_default_normalize(100, 0, out, F); /* the WHOLE list, later entries still 0 */
        }
        return 0;
    }
    nam_closed(r, F, out);
    return 0;
}

int msor_schedule_nam(const msor_nodes *nd, const msor_pods *pd, const uint8_t *term_sets, uint32_t n_sets,
                      int64_t w_nn, int64_t w_na, int literal, uint64_t seed, uint32_t node_base, int32_t *out_node,
                      int64_t *out_score, int32_t *out_code, uint32_t *out_mask, uint64_t *out_key) {
    if (n_sets && !term_sets) return -1;
    uint8_t *ext = (uint8_t *)malloc((size_t)MSOR_NAM_EXT_BYTES * (n_sets ? n_sets : 1));
    if (!ext) return -1;
    for (uint32_t s = 0; s < n_sets; ++s) nam_set_to_ext(term_sets + 16u * s, ext + (size_t)MSOR_NAM_EXT_BYTES * s);
    const int rc = msor_schedule_nam_ext(nd, pd, ext, n_sets, w_nn, w_na, literal, seed, node_base, out_node,
                                         out_score, out_code, out_mask, out_key);
    free(ext);
    return rc;
}

int msor_schedule_nam_ext(const msor_nodes *nd, const msor_pods *pd, const uint8_t *term_sets, uint32_t n_sets,
                          int64_t w_nn, int64_t w_na, int literal, uint64_t seed, uint32_t node_base,
                          int32_t *out_node, int64_t *out_score, int32_t *out_code, uint32_t *out_mask,
                          uint64_t *out_key) {
    if (!nd || !pd || !nd->flags || !nd->digit || !nd->zone || !nd->label2 || !pd->ordinal || !pd->digit || !pd->tol ||
        !pd->pref_zone || !pd->pref_weight || (n_sets && !term_sets))
        return -1;
    if ((uint64_t)node_base + nd->n >= 0xFFFFFu) return -1;
    static const uint8_t none[MSOR_NAM_EXT_BYTES] = {0};
    uint32_t *feas = (uint32_t *)malloc(sizeof(uint32_t) * (nd->n ? nd->n : 1));
    int64_t *raw = (int64_t *)malloc(sizeof(int64_t) * (nd->n ? nd->n : 1));
    int64_t *na = (int64_t *)malloc(sizeof(int64_t) * (nd->n ? nd->n : 1));
    if (!feas || !raw || !na) { free(feas); free(raw); free(na); return -1; }
    int rc = 0;
    for (uint32_t j = 0; j < pd->n; ++j) {
        const uint32_t sid = (uint32_t)pd->pref_zone[j] | (uint32_t)pd->pref_weight[j] << 8;
        /* (ids past the registered sets count as no terms: minisched_gpu.h ms_nam_term_sets) */
        const uint8_t *set = (sid && sid <= n_sets) ? term_sets + (size_t)MSOR_NAM_EXT_BYTES * (sid - 1u) : none;
        /* RunFilterPlugins (minisched.go:115-151): NodeUnschedulable only */
        uint32_t F = 0, mask = 0;
        for (uint32_t i = 0; i < nd->n; ++i) {
            if (nd->flags[i] & MSOR_NODE_ABSENT) continue;
            if (nu_rejects(nd->flags[i], pd->tol[j])) { mask |= MSOR_MASK_NU; continue; }
            feas[F++] = i;
        }
        int32_t node = -1, code;
        int64_t score = 0;
        uint64_t best = 0;
        if (F == 0) {
            code = MSOR_CODE_UNSCHEDULABLE;
        } else if (pd->digit[j] < 0) { /* NodeNumber.Score fails at the first node (:170-172) */
            code = MSOR_CODE_ERROR;
            mask = 0;
        } else {
            /* RunScorePlugins (minisched.go:164-185): NodeNumber then NodeAffinity per
             * feasible node; NodeAffinity's NormalizeScore on its whole list each time */
            for (uint32_t k = 0; k < F; ++k) raw[k] = nam_raw(nd, feas[k], set);
            msor_nam_inloop(raw, F, literal, na);
            const uint32_t ph = msor_pod_hash(seed, pd->ordinal[j]);
            for (uint32_t k = 0; k < F; ++k) { /* sum (:187-196), weights applied; selectHost (:304-325) */
                const uint32_t ord = node_base + feas[k];
                const uint64_t key = msor_key(w_nn * nn_score(pd->digit[j], nd->digit[feas[k]]) + w_na * na[k],
                                              msor_tb_hash(ph, ord), ord);
                if (key > best) best = key;
            }
            code = MSOR_CODE_SUCCESS;
            mask = 0;
            node = (int32_t)(0xFFFFFu - (uint32_t)(best & 0xFFFFFu));
            score = (int64_t)(best >> 52);
        }
        if (out_node) out_node[j] = node;
        if (out_score) out_score[j] = score;
        if (out_code) out_code[j] = code;
        if (out_mask) out_mask[j] = code == MSOR_CODE_UNSCHEDULABLE ? mask : 0;
        if (out_key) out_key[j] = best;
    }
    free(feas);
    free(raw);
    free(na);
    return rc;
}

/* ---- TaintToleration + the in-loop reverse normalise hook ------------------ */

/* k8s@v1.22.0:pkg/scheduler/framework/plugins/tainttoleration/taint_toleration.go
 * Filter: v1helper.FindMatchingUntoleratedTaint over the node's taints with
 * effect NoSchedule or NoExecute -> UnschedulableAndUnresolvable. Taints are
 * ids of the cluster's taint universe; the toleration match (v1 ToleratesTaint)
 * is evaluated per (pod, taint id) on the host, as the Filter evaluates it per
 * call. */
static int tt_rejects(uint32_t taints, uint8_t tol_hard) { return (taints & 0xFFu & ~(uint32_t)tol_hard) != 0; }

/* Score: countIntolerableTaintsPreferNoSchedule — the node's PreferNoSchedule
 * taints no PreferNoSchedule-or-empty-effect toleration of the pod tolerates
 * (getAllTolerationPreferNoSchedule). */
static int64_t tt_raw(uint32_t taints, uint8_t tol_soft) {
    return (int64_t)__builtin_popcount((taints >> 8) & 0xFFu & ~(uint32_t)tol_soft);
}

/* DefaultNormalizeScore(100, reverse=true) as one value map: the whole list is
 * rewritten with the same map at every step of the loop. */
static int64_t tt_map(int64_t m, int64_t v) { return m == 0 ? 100 : 100 - (100 * v) / m; }

/* Closed form of the loop (msor_tt_inloop, literal = 0). The loop normalises
 * the whole F-entry list after writing entry k; entries > k are still the
 * zeros of createPluginToNodeScores (minisched.go:327-334) and are rewritten
 * like every other. Every step applies one map v -> 100 - floor(100 v / M_k)
 * (M_k = the list maximum; all 100 when M_k = 0) to every entry, the entries
 * not yet scored included (they stay equal: one "future" value u). With counts
 * <= 8 the list holds both 0 and 100 after step 2 (step 0 leaves the first
 * entry at 0 and u at 100, or both at 100 when c0 = 0; then step 1 or 2 makes
 * a 0 and keeps a 100), so every later step before the last has M_k = 100 and
 * is the flip v -> 100 - v: entry j >= 3 is written at step j as c_j, mapped to
 * 100 - c_j, and flipped F-2-j more times before the last step. The last step
 * (no future entry left) is the one map with M = the list's maximum. */
static void tt_closed(const int64_t *c, uint32_t F, int64_t *out) {
    if (F <= 4) { /* (small lists: the loop itself) */
        int64_t s[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < F; ++k) {
            s[k] = c[k];
            msor_default_normalize(100, 1, s, F);
        }
        for (uint32_t k = 0; k < F; ++k) out[k] = s[k];
        return;
    }
    int64_t s[3], u = 0; /* entries 0..2 and the future value after step 2 */
    for (uint32_t k = 0; k < 3; ++k) {
        s[k] = c[k];
        int64_t m = u;
        for (uint32_t i = 0; i <= k; ++i) m = s[i] > m ? s[i] : m;
        for (uint32_t i = 0; i <= k; ++i) s[i] = tt_map(m, s[i]);
        u = tt_map(m, u);
    }
    const int nf_odd = (int)((F - 4) & 1u); /* flips of steps 3..F-2 */
    int64_t m_last = c[F - 1];
    for (uint32_t j = 0; j + 1 < F; ++j) {
        int64_t p;
        if (j < 3) p = nf_odd ? 100 - s[j] : s[j];
        else p = ((F - 2 - j) & 1u) ? c[j] : 100 - c[j];
        out[j] = p;
        if (p > m_last) m_last = p;
    }
    for (uint32_t j = 0; j + 1 < F; ++j) out[j] = tt_map(m_last, out[j]);
    out[F - 1] = tt_map(m_last, c[F - 1]);
}

int msor_tt_inloop(const int64_t *c, uint32_t F, int literal, int64_t *out) {
    for (uint32_t k = 0; k < F; ++k)
        if (c[k] < 0 || c[k] > 8) return -1;
    if (!literal) {
        tt_closed(c, F, out);
        return 0;
    }
    /* minisched.go:164-185: Score writes entry k, NormalizeScore rewrites the
     * whole list (entries > k still 0) */
    for (uint32_t k = 0; k < F; ++k) out[k] = 0;
    for (uint32_t k = 0; k < F; ++k) {
        out[k] = c[k];
        msor_default_normalize(100, 1, out, F);
    }
    return 0;
}

int msor_schedule_tt(const msor_nodes *nd, const msor_pods *pd, int literal, uint64_t seed,
                     uint32_t node_base, int32_t *out_node, int64_t *out_score, int32_t *out_code,
                     uint32_t *out_mask, uint64_t *out_key) {
    if (!nd || !pd || !nd->flags || !nd->digit || !nd->taints || !pd->ordinal || !pd->digit || !pd->tol ||
        !pd->tol_hard || !pd->tol_soft)
        return -1;
    if ((uint64_t)node_base + nd->n >= 0xFFFFFu) return -1;
    const uint32_t cap = nd->n ? nd->n : 1;
    uint32_t *feas = (uint32_t *)malloc(sizeof(uint32_t) * cap);
    int64_t *cnt = (int64_t *)malloc(sizeof(int64_t) * cap);
    int64_t *tt = (int64_t *)malloc(sizeof(int64_t) * cap);
    if (!feas || !cnt || !tt) { free(feas); free(cnt); free(tt); return -1; }
    for (uint32_t j = 0; j < pd->n; ++j) {
        /* RunFilterPlugins (minisched.go:115-151): NU then TT, first failure per node */
        uint32_t F = 0, mask = 0;
        for (uint32_t i = 0; i < nd->n; ++i) {
            if (nd->flags[i] & MSOR_NODE_ABSENT) continue;
            if (nu_rejects(nd->flags[i], pd->tol[j])) { mask |= MSOR_MASK_NU; continue; }
            if (tt_rejects(nd->taints[i], pd->tol_hard[j])) { mask |= MSOR_MASK_TT; continue; }
            cnt[F] = tt_raw(nd->taints[i], pd->tol_soft[j]);
            feas[F++] = i;
        }
        int32_t node = -1, code;
        int64_t score = 0;
        uint64_t best = 0;
        if (F == 0) {
            code = MSOR_CODE_UNSCHEDULABLE;
        } else if (pd->digit[j] < 0) { /* NodeNumber.Score fails at the first node (:170-172) */
            code = MSOR_CODE_ERROR;
        } else {
            msor_tt_inloop(cnt, F, literal, tt);
            const uint32_t ph = msor_pod_hash(seed, pd->ordinal[j]);
            for (uint32_t k = 0; k < F; ++k) { /* sum (:187-196) and selectHost (:304-325) */
                const uint32_t ord = node_base + feas[k];
                const uint64_t key = msor_key(nn_score(pd->digit[j], nd->digit[feas[k]]) + tt[k],
                                              msor_tb_hash(ph, ord), ord);
                if (key > best) best = key;
            }
            code = MSOR_CODE_SUCCESS;
            node = (int32_t)(0xFFFFFu - (uint32_t)(best & 0xFFFFFu));
            score = (int64_t)(best >> 52);
        }
        if (out_node) out_node[j] = node;
        if (out_score) out_score[j] = score;
        if (out_code) out_code[j] = code;
        if (out_mask) out_mask[j] = code == MSOR_CODE_UNSCHEDULABLE ? mask : 0;
        if (out_key) out_key[j] = code == MSOR_CODE_SUCCESS ? best : 0;
    }
    free(feas);
    free(cnt);
    free(tt);
    return 0;
}
