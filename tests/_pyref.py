"""Pure-Python restatement of minisched's cycle on v1-style objects.

Small cases only. It follows minisched.go literally (feasible list, per-plugin
NodeScoreList, unweighted sum, linear selectHost) on names and tolerations,
so that it cross-checks both the record encoding and the C oracle.
Test infrastructure, never product code.
"""
from __future__ import annotations

from minisched_amd.encode import ZONE_LABEL, name_digit, pod_requests, tolerates_unschedulable

MASK_NU, MASK_NRF = 1, 2


def fmix32(h):
    h &= 0xFFFFFFFF
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


def seed32(seed):
    return (seed ^ (seed >> 32)) & 0xFFFFFFFF


def mix32(x):
    """Mixer of rule r3: xor-shift 16, multiply, xor-shift 16, multiply."""
    x &= 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0xC2B2AE35) & 0xFFFFFFFF
    return x


def h32(seed, pod_ord, node_ord):
    """Tie-break hash, rule r3 (include/minisched_gpu.h)."""
    a = fmix32(seed32(seed) ^ pod_ord)
    return mix32(a + node_ord * 0x9E3779)


def key(score, h, node_ord):
    return (score << 52) | (h << 20) | (0xFFFFF - node_ord)


def least_requested(requested, capacity):
    if capacity == 0:
        return 0
    if requested > capacity:
        return 0
    return ((capacity - requested) * 100) // capacity


class NodeState:
    """framework.NodeInfo columns for one node (k8s@v1.22.0 types.go)."""

    def __init__(self, node):
        self.node = node
        self.req_cpu = self.req_mem = self.nz_cpu = self.nz_mem = 0
        self.pods = 0


def schedule(nodes, pods, resources=False, sequential=False, seed=1):
    """nodes: list of encode.Node (ordinal = list index); pods: list of encode.Pod.
    Returns list of (code, node_ordinal, score, mask)."""
    state = [NodeState(n) for n in nodes]
    out = []
    for pod in pods:
        tol = tolerates_unschedulable(pod.tolerations)
        rc, rm, nc, nm = pod_requests(pod)
        # RunFilterPlugins (minisched.go:115-151)
        feasible, plugins = [], set()
        for i, st in enumerate(state):
            n = st.node
            if n.unschedulable and not tol:  # NodeUnschedulable
                plugins.add(MASK_NU)
                continue
            if resources:  # NodeResourcesFit.fitsRequest
                bad = st.pods + 1 > n.allocatable.get("pods", 110)
                if not (rc == 0 and rm == 0):
                    bad |= rc > n.allocatable.get("cpu", 0) - st.req_cpu
                    bad |= rm > n.allocatable.get("memory", 0) - st.req_mem
                if bad:
                    plugins.add(MASK_NRF)
                    continue
            feasible.append(i)
        if not feasible:
            m = 0
            for b in plugins:
                m |= b
            out.append((2, -1, 0, m))
            continue
        # PreScore: NodeNumber (nodenumber.go:50-64)
        podnum = name_digit(pod.name)
        if podnum < 0:  # Score -> CycleState.Read error (nodenumber.go:74-77)
            out.append((1, -1, 0, 0))
            continue
        # RunScorePlugins: per plugin lists, then unweighted sum
        nn = []
        for i in feasible:
            d = name_digit(nodes[i].name)
            nn.append(10 if (d >= 0 and d == podnum) else 0)
        total = list(nn)
        if resources:
            for k, i in enumerate(feasible):
                st = state[i]
                a = nodes[i].allocatable
                s_cpu = least_requested(st.nz_cpu + nc, a.get("cpu", 0))
                s_mem = least_requested(st.nz_mem + nm, a.get("memory", 0))
                total[k] += (s_cpu + s_mem) // 2
        # selectHost with the deterministic packed key
        best, best_i = -1, -1
        for k, i in enumerate(feasible):
            kk = key(total[k], h32(seed, pod.ordinal, i), i)
            if kk > best:
                best, best_i = kk, k
        w = feasible[best_i]
        out.append((0, w, total[best_i], 0))
        if sequential:
            st = state[w]
            st.req_cpu += rc
            st.req_mem += rm
            st.nz_cpu += nc
            st.nz_mem += nm
            st.pods += 1
    return out


def default_normalize_score(max_priority, reverse, scores):
    """k8s@v1.22.0 pkg/scheduler/framework/plugins/helper/normalize_score.go, in place."""
    max_count = max([s for s in scores] + [0])
    if max_count == 0:
        if reverse:
            for i in range(len(scores)):
                scores[i] = max_priority
        return
    for i in range(len(scores)):
        sc = max_priority * scores[i] // max_count
        scores[i] = max_priority - sc if reverse else sc


def schedule_na(nodes, pods, weights=(1, 1), seed=1):
    """MS_PLUGINS_NU_NN_NA on v1-style objects, minisched.go:164-199 as written:
    createPluginToNodeScores zero-fills one list per plugin; for each feasible
    node, NodeNumber then NodeAffinity score it and NodeAffinity's
    NormalizeScore (DefaultNormalizeScore(100, false)) runs on its whole list
    right away; then the (here weighted) sum and selectHost."""
    out = []
    for pod in pods:
        tol = tolerates_unschedulable(pod.tolerations)
        feasible, plugins = [], 0
        for i, n in enumerate(nodes):
            if n.unschedulable and not tol:
                plugins |= MASK_NU
                continue
            feasible.append(i)
        if not feasible:
            out.append((2, -1, 0, plugins))
            continue
        podnum = name_digit(pod.name)
        if podnum < 0:
            out.append((1, -1, 0, 0))
            continue
        nn = [0] * len(feasible)
        na = [0] * len(feasible)
        for k, i in enumerate(feasible):
            d = name_digit(nodes[i].name)
            nn[k] = 10 if (d >= 0 and d == podnum) else 0
            pz = pod.preferred_zone
            na[k] = pz[1] if (pz is not None and nodes[i].labels.get(ZONE_LABEL) == pz[0]) else 0
            default_normalize_score(100, False, na)
        total = [weights[0] * a + weights[1] * b for a, b in zip(nn, na)]
        best, best_k = -1, -1
        for k, i in enumerate(feasible):
            kk = key(total[k], h32(seed, pod.ordinal, i), i)
            if kk > best:
                best, best_k = kk, k
        out.append((0, feasible[best_k], total[best_k], 0))
    return out


# ---- MS_PLUGINS_NU_NN_NAM on v1-style objects --------------------------------
def _parse_int64(v):
    """strconv.ParseInt(v, 10, 64); None on error (restated here on purpose, not
    imported: the encoder's id sets are checked against this)."""
    s = v[1:] if v[:1] in ("+", "-") else v
    if not s or not all("0" <= c <= "9" for c in s):
        return None
    x = int(v)
    return x if -(1 << 63) <= x <= (1 << 63) - 1 else None


def requirement_matches(req, labels):
    """labels.Requirement.Matches (k8s.io/apimachinery, the operators a
    NodeSelectorRequirement maps to in k8s@v1.22.0 component-helpers)."""
    has = req.key in labels
    v = labels.get(req.key)
    if req.operator == "In":
        return has and v in req.values
    if req.operator == "NotIn":
        return (not has) or v not in req.values
    if req.operator == "Exists":
        return has
    if req.operator == "DoesNotExist":
        return not has
    if req.operator in ("Gt", "Lt"):
        if not has:
            return False
        x, b = _parse_int64(v), _parse_int64(req.values[0])
        if x is None or b is None:
            return False
        return x > b if req.operator == "Gt" else x < b
    raise ValueError(req.operator)


def term_matches(term, labels):
    """nodeSelectorTerm.match: an empty term matches nothing; else every requirement."""
    return bool(term.requirements) and all(requirement_matches(r, labels) for r in term.requirements)


def nam_raw(terms, labels):
    """NodeAffinity.Score: the sum of the weights of the matching preferred terms."""
    return sum(t.weight for t in terms if t.weight > 0 and term_matches(t, labels))


def schedule_nam(nodes, pods, pod_terms, weights=(1, 1), seed=1):
    """MS_PLUGINS_NU_NN_NAM, minisched.go:164-199 as written (the in-loop
    DefaultNormalizeScore on the whole NodeAffinity list after every node):
    pod_terms[j] = the pod's list of PreferredTerm objects."""
    out = []
    for j, pod in enumerate(pods):
        tol = tolerates_unschedulable(pod.tolerations)
        feasible, plugins = [], 0
        for i, n in enumerate(nodes):
            if n.unschedulable and not tol:
                plugins |= MASK_NU
                continue
            feasible.append(i)
        if not feasible:
            out.append((2, -1, 0, plugins))
            continue
        podnum = name_digit(pod.name)
        if podnum < 0:
            out.append((1, -1, 0, 0))
            continue
        nn = [0] * len(feasible)
        na = [0] * len(feasible)
        for k, i in enumerate(feasible):
            d = name_digit(nodes[i].name)
            nn[k] = 10 if (d >= 0 and d == podnum) else 0
            na[k] = nam_raw(pod_terms[j], nodes[i].labels)
            default_normalize_score(100, False, na)
        total = [weights[0] * a + weights[1] * b for a, b in zip(nn, na)]
        best, best_k = -1, -1
        for k, i in enumerate(feasible):
            kk = key(total[k], h32(seed, pod.ordinal, i), i)
            if kk > best:
                best, best_k = kk, k
        out.append((0, feasible[best_k], total[best_k], 0))
    return out
