"""v1.Node / v1.Pod -> flat records (what the cgo shim computes per object).

Only the fields the in-scope plugins read cross the boundary:
  * name_digit  — strconv.Atoi(name[len-1:]) (nodenumber.go:51-52, :81-83):
                  only '0'..'9' parse; anything else is "not a digit".
  * tolerates_unschedulable — v1helper.TolerationsTolerateTaint(pod tolerations,
                  {Key: node.kubernetes.io/unschedulable, Effect: NoSchedule})
                  (k8s@v1.22.0 nodeunschedulable, restated).
  * requests    — Fit PreFilter computePodResourceRequest and
                  NodeInfo.calculateResource / GetNonzeroRequests (k8s@v1.22.0).
  * zone / pref_zone, pref_weight — MS_PLUGINS_NU_NN_NA: the node's
                  topology.kubernetes.io/zone label and the pod's one preferred
                  NodeAffinity term {weight, zone In [value]}, as value ids that
                  one ZoneIds table assigns on both sides (0 = none).
  * taints / tol_hard, tol_soft — MS_PLUGINS_NU_TT_NN: the node's Spec.Taints
                  as taint ids that one TaintIds table assigns (at most 8
                  NoSchedule/NoExecute and 8 PreferNoSchedule taints in the
                  cluster), and per pod the ids some toleration tolerates
                  (Toleration.ToleratesTaint, restated below).
Quantities are already integers here: cpu in millicores, memory in bytes.

Resources the device cannot evaluate are refused, never dropped (VERDICT r5
item 3). Upstream Fit.fitsRequest (k8s@v1.22.0 noderesources/fit.go) also
compares ephemeral-storage and every scalar (extended, hugepages-*) resource a
pod requests against Allocatable - Requested; ms_pod_rec carries cpu and memory
only. So pod_requests raises UnsupportedResource for any other request name in
a container, an init container or the overhead (an explicit 0 too: it makes
upstream's "all requests are 0" early return false). Node allocatable entries
for other names are accepted and ignored: with no admitted pod requesting them,
Requested stays 0 <= Allocatable and fitsRequest never reads them (it loops over
the POD's scalar names), so no decision depends on them. Plugin sets without
NodeResourcesFit read no resources at all (pod_records(check_resources=False)).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from ._lib import NODE_REC, POD_REC

TAINT_NODE_UNSCHEDULABLE = "node.kubernetes.io/unschedulable"
ZONE_LABEL = "topology.kubernetes.io/zone"
TAINT_EFFECT_NO_SCHEDULE = "NoSchedule"
TAINT_EFFECT_NO_EXECUTE = "NoExecute"
TAINT_EFFECT_PREFER_NO_SCHEDULE = "PreferNoSchedule"
TAINT_IDS_PER_KIND = 8  # ms_node_rec.taints: bits 0-7 hard, 8-15 PreferNoSchedule
DEFAULT_MILLI_CPU_REQUEST = 100
DEFAULT_MEMORY_REQUEST = 200 * 1024 * 1024
DEVICE_RESOURCES = ("cpu", "memory")  # the request names ms_pod_rec carries


class UnsupportedResource(ValueError):
    """A pod requests a resource NodeResourcesFit would check but the device
    records cannot carry (ephemeral-storage, hugepages-*, extended resources)."""


def name_digit(name: str) -> int:
    """Last character as 0..9, or -1 (strconv.Atoi of a 1-char string)."""
    if not name:
        raise ValueError("empty object name (the reference would panic slicing name[-1:])")
    c = name[-1]
    return ord(c) - 48 if "0" <= c <= "9" else -1


@dataclass(frozen=True)
class Taint:
    key: str
    value: str = ""
    effect: str = TAINT_EFFECT_NO_SCHEDULE


@dataclass
class Toleration:
    key: str = ""
    operator: str = ""  # "" == Equal
    value: str = ""
    effect: str = ""


def toleration_tolerates(t: Toleration, key: str, value: str, effect: str) -> bool:
    """k8s.io/api core/v1 Toleration.ToleratesTaint (v0.22.0)."""
    if t.effect and t.effect != effect:
        return False
    if t.key and t.key != key:
        return False
    if t.operator in ("", "Equal"):
        return t.value == value
    if t.operator == "Exists":
        return True
    return False


def tolerates_unschedulable(tolerations: List[Toleration]) -> bool:
    return any(
        toleration_tolerates(t, TAINT_NODE_UNSCHEDULABLE, "", TAINT_EFFECT_NO_SCHEDULE) for t in tolerations
    )


@dataclass
class Container:
    # "cpu" (milli), "memory" (bytes); any other name is refused by pod_requests
    requests: Dict[str, int] = field(default_factory=dict)


@dataclass
class Pod:
    name: str
    ordinal: int
    tolerations: List[Toleration] = field(default_factory=list)
    containers: List[Container] = field(default_factory=list)
    init_containers: List[Container] = field(default_factory=list)
    overhead: Optional[Dict[str, int]] = None
    # one PreferredSchedulingTerm: (zone label value, weight 1..100)
    preferred_zone: Optional[Tuple[str, int]] = None


@dataclass
class Node:
    name: str
    unschedulable: bool = False
    # cpu (milli), memory (bytes), pods; other names (ephemeral-storage, ...) are ignored
    allocatable: Dict[str, int] = field(default_factory=dict)
    labels: Dict[str, str] = field(default_factory=dict)
    taints: List[Taint] = field(default_factory=list)


class TaintIds:
    """Taint -> id, shared by node and pod encoding (the shim's map for
    MS_PLUGINS_NU_TT_NN, minisched_gpu.h). Filter taints (NoSchedule and
    NoExecute: TaintToleration.Filter's filterPredicate) take ids 0..7 in
    ms_node_rec.taints bits 0-7; PreferNoSchedule taints (the ones Score counts,
    countIntolerableTaintsPreferNoSchedule) take ids 0..7 in bits 8-15. A taint
    is identified by (key, value, effect): Toleration.ToleratesTaint reads
    exactly those three. A ninth taint of one kind raises OverflowError: the
    device form (and the closed form of the in-loop reverse normaliser, whose
    raw counts must stay <= 8) holds no more, so such a cluster must not be
    scheduled with this plugin set. Taints with any other effect are ignored
    by both plugins and get no id. (k8s@v1.22.0
    plugins/tainttoleration/taint_toleration.go, restated.)"""

    def __init__(self):
        self.hard: Dict[Taint, int] = {}
        self.soft: Dict[Taint, int] = {}

    def id_of(self, t: Taint) -> Tuple[Optional[str], int]:
        """("hard" | "soft" | None, id) of taint t, assigning a new id on first sight."""
        if t.effect in (TAINT_EFFECT_NO_SCHEDULE, TAINT_EFFECT_NO_EXECUTE):
            table, kind = self.hard, "hard"
        elif t.effect == TAINT_EFFECT_PREFER_NO_SCHEDULE:
            table, kind = self.soft, "soft"
        else:
            return None, -1
        if t not in table:
            if len(table) >= TAINT_IDS_PER_KIND:
                raise OverflowError(f"more than {TAINT_IDS_PER_KIND} distinct {kind} taints in the cluster: "
                                    "MS_PLUGINS_NU_TT_NN cannot encode it")
            table[t] = len(table)
        return kind, table[t]

    def node_bits(self, taints: List[Taint]) -> int:
        """ms_node_rec.taints of a node's Spec.Taints. Taints are unique per
        (key, effect) on a node (API validation), so bit counts equal entry
        counts; a duplicate raises."""
        seen = set()
        bits = 0
        for t in taints:
            if (t.key, t.effect) in seen:
                raise ValueError(f"duplicate taint {t.key}:{t.effect} on one node (API validation)")
            seen.add((t.key, t.effect))
            kind, i = self.id_of(t)
            if kind == "hard":
                bits |= 1 << i
            elif kind == "soft":
                bits |= 1 << (8 + i)
        return bits

    def pod_masks(self, tolerations: List["Toleration"]) -> Tuple[int, int]:
        """(tol_hard, tol_soft): bit t set when some toleration tolerates taint
        id t. Filter: FindMatchingUntoleratedTaint over the hard taints with all
        tolerations. Score: the tolerations with an empty or PreferNoSchedule
        effect (getAllTolerationPreferNoSchedule) against the PreferNoSchedule
        taints; ToleratesTaint's own effect check makes that prefilter a no-op.
        Pods must be encoded after every node of the cluster (the ids a pod's
        masks refer to are the ones assigned so far)."""
        hard = soft = 0
        for t, i in self.hard.items():
            if any(toleration_tolerates(x, t.key, t.value, t.effect) for x in tolerations):
                hard |= 1 << i
        pref = [x for x in tolerations if x.effect in ("", TAINT_EFFECT_PREFER_NO_SCHEDULE)]
        for t, i in self.soft.items():
            if any(toleration_tolerates(x, t.key, t.value, t.effect) for x in pref):
                soft |= 1 << i
        return hard, soft


class ZoneIds:
    """Label value -> id 1..254, shared by node and pod encoding (the shim's map).
    Id 0xFF is not handed out: in a multi-term NodeAffinity set (ms_pref_term)
    value 0xFF means Exists, so a label value with that id could not be named
    by an In term."""

    MAX_IDS = 254

    def __init__(self):
        self.ids: Dict[str, int] = {}

    def __call__(self, value: Optional[str]) -> int:
        if value is None:
            return 0
        if value not in self.ids:
            if len(self.ids) >= self.MAX_IDS:
                raise ValueError(f"more than {self.MAX_IDS} label values")
            self.ids[value] = len(self.ids) + 1
        return self.ids[value]


def unsupported_request(p: Pod) -> Optional[str]:
    """The first request name of p outside DEVICE_RESOURCES (containers, init
    containers, overhead), or None."""
    lists = [c.requests for c in p.containers] + [c.requests for c in p.init_containers]
    if p.overhead:
        lists.append(p.overhead)
    for r in lists:
        for name in r:
            if name not in DEVICE_RESOURCES:
                return name
    return None


# ---- MS_PLUGINS_NU_NN_NAM: preferred NodeAffinity terms in general form (ABI 7) ----
NAM_OPERATORS = ("In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt")
_INT64 = re.compile(r"^[+-]?[0-9]+$")


class UnsupportedTerm(ValueError):
    """A preferred term the device records cannot express (a requirement on a
    label key other than the two encoded ones, more than MS_NAM_TERMS terms)."""


@dataclass(frozen=True)
class NodeSelectorRequirement:
    key: str
    operator: str  # In, NotIn, Exists, DoesNotExist, Gt, Lt
    values: Tuple[str, ...] = ()


@dataclass
class PreferredTerm:
    weight: int  # 1..100 (API validation)
    requirements: List[NodeSelectorRequirement] = field(default_factory=list)


def parse_int64(v: str) -> Optional[int]:
    """strconv.ParseInt(v, 10, 64), None on error."""
    if not _INT64.match(v):
        return None
    x = int(v)
    return x if -(1 << 63) <= x < (1 << 63) else None


def requirement_holds(req: NodeSelectorRequirement, value: Optional[str]) -> bool:
    """k8s.io/apimachinery labels.Requirement.Matches on one label (value None:
    the node lacks the key), for the operators NodeSelectorRequirement maps to
    (k8s@v1.22.0 component-helpers nodeaffinity nodeSelectorRequirementsAsSelector)."""
    op = req.operator
    if op == "In":
        return value is not None and value in req.values
    if op == "NotIn":
        return value is None or value not in req.values
    if op == "Exists":
        return value is not None
    if op == "DoesNotExist":
        return value is None
    if op in ("Gt", "Lt"):
        if value is None:
            return False
        x = parse_int64(value)
        if x is None:
            return False
        bound = parse_int64(req.values[0])
        return x > bound if op == "Gt" else x < bound
    raise UnsupportedTerm(f"operator {op!r}")


class NamTerms:
    """Term sets of MS_PLUGINS_NU_NN_NAM in general form (ms_nam_term_set_ext):
    label key 0 is the zone label, key 1 `label2_key`; value ids come from the two
    tables the node records use (ZoneIds). Per term and key the id set holds id v
    when every requirement of the term on that key holds for value v (bit 0: for
    a node without the label); a key without requirements holds every id. A term
    with no requirement matches no node (an empty nodeSelectorTerm). Ids a table
    has not handed out yet are left out: the shim re-registers its sets when a
    table grows (NotIn, Exists, DoesNotExist, Gt and Lt cover new values too)."""

    def __init__(self, label2_key: str, zone_ids: "ZoneIds", label2_ids: "ZoneIds"):
        self.keys = (ZONE_LABEL, label2_key)
        self.tables = (zone_ids, label2_ids)

    def id_set(self, k: int, reqs: List[NodeSelectorRequirement]) -> int:
        m = 0
        for value, vid in [(None, 0)] + list(self.tables[k].ids.items()):
            if all(requirement_holds(r, value) for r in reqs):
                m |= 1 << vid
        return m

    def term(self, t: PreferredTerm) -> Tuple[int, int, int]:
        if not 1 <= t.weight <= 100:
            raise ValueError("PreferredSchedulingTerm weight must be in 1..100 (API validation)")
        for r in t.requirements:
            if r.key not in self.keys:
                raise UnsupportedTerm(f"requirement on label {r.key!r}: the records carry {self.keys} only")
            if r.operator not in NAM_OPERATORS:
                raise UnsupportedTerm(f"operator {r.operator!r}")
            if r.operator in ("In", "NotIn") and not r.values:
                raise ValueError(f"{r.operator} needs values (API validation)")
            if r.operator in ("Exists", "DoesNotExist") and r.values:
                raise ValueError(f"{r.operator} takes no values (API validation)")
            if r.operator in ("Gt", "Lt") and (len(r.values) != 1 or parse_int64(r.values[0]) is None):
                raise ValueError(f"{r.operator} needs one integer value (API validation)")
        if not t.requirements:
            return (t.weight, 0, 0)
        return (t.weight,) + tuple(self.id_set(k, [r for r in t.requirements if r.key == self.keys[k]])
                                   for k in (0, 1))

    def term_sets(self, sets: List[List[PreferredTerm]]) -> np.ndarray:
        """uint8 (n, 272) ms_nam_term_set_ext records; set i is term set id i + 1."""
        from ._lib import NAM_TERMS, nam_term_sets_ext_array

        for terms in sets:
            if len(terms) > NAM_TERMS:
                raise UnsupportedTerm(f"more than {NAM_TERMS} preferred terms")
        return nam_term_sets_ext_array([[self.term(t) for t in terms] for terms in sets])


def pod_requests(p: Pod, check_resources: bool = True):
    """(req_cpu, req_mem, nz_cpu, nz_mem).

    req: Fit.computePodResourceRequest — sum of containers, max with each init
    container, plus overhead. nz: NodeInfo.calculateResource's non-zero pair —
    per container GetNonzeroRequests (missing cpu -> 100 m, missing memory ->
    200 MiB, explicit 0 stays 0), max with init containers, plus overhead.
    Raises UnsupportedResource for a request the device cannot evaluate
    (module docstring) unless check_resources is False.
    """
    bad = unsupported_request(p) if check_resources else None
    if bad is not None:
        raise UnsupportedResource(f"pod {p.name} requests {bad!r}: NodeResourcesFit would check it, but the device "
                                  f"records carry {' and '.join(DEVICE_RESOURCES)} only")
    rc = sum(c.requests.get("cpu", 0) for c in p.containers)
    rm = sum(c.requests.get("memory", 0) for c in p.containers)
    nc = sum(c.requests.get("cpu", DEFAULT_MILLI_CPU_REQUEST) for c in p.containers)
    nm = sum(c.requests.get("memory", DEFAULT_MEMORY_REQUEST) for c in p.containers)
    for ic in p.init_containers:
        rc = max(rc, ic.requests.get("cpu", 0))
        rm = max(rm, ic.requests.get("memory", 0))
        nc = max(nc, ic.requests.get("cpu", DEFAULT_MILLI_CPU_REQUEST))
        nm = max(nm, ic.requests.get("memory", DEFAULT_MEMORY_REQUEST))
    if p.overhead:
        rc += p.overhead.get("cpu", 0)
        rm += p.overhead.get("memory", 0)
        nc += p.overhead.get("cpu", 0)
        nm += p.overhead.get("memory", 0)
    return rc, rm, nc, nm


def pod_records(pods: List[Pod], zone_ids: Optional[ZoneIds] = None,
                taint_ids: Optional[TaintIds] = None, check_resources: bool = True) -> np.ndarray:
    """taint_ids (MS_PLUGINS_NU_TT_NN): pref_zone / pref_weight carry the pod's
    tol_hard / tol_soft masks instead of a NodeAffinity term. check_resources:
    refuse requests the device cannot evaluate (pod_requests); a plugin set
    without NodeResourcesFit reads no resources and may pass False."""
    rec = np.zeros(len(pods), dtype=POD_REC)
    for i, p in enumerate(pods):
        if taint_ids is not None:
            if p.preferred_zone is not None:
                raise ValueError("MS_PLUGINS_NU_TT_NN records carry tolerations, not a NodeAffinity term")
            rec[i]["pref_zone"], rec[i]["pref_weight"] = taint_ids.pod_masks(p.tolerations)
        elif p.preferred_zone is not None:
            zone, weight = p.preferred_zone
            if not 1 <= weight <= 100:
                raise ValueError("PreferredSchedulingTerm weight must be in 1..100 (API validation)")
            rec[i]["pref_zone"] = (zone_ids or ZoneIds())(zone)
            rec[i]["pref_weight"] = weight
        rc, rm, nc, nm = pod_requests(p, check_resources)
        rec[i]["ordinal"] = p.ordinal
        rec[i]["name_digit"] = name_digit(p.name)
        rec[i]["tolerates_unschedulable"] = 1 if tolerates_unschedulable(p.tolerations) else 0
        rec[i]["req_milli_cpu"], rec[i]["req_memory"] = rc, rm
        rec[i]["nonzero_milli_cpu"], rec[i]["nonzero_memory"] = nc, nm
    return rec


def node_records(nodes: List[Node], zone_ids: Optional[ZoneIds] = None,
                 taint_ids: Optional[TaintIds] = None) -> np.ndarray:
    rec = np.zeros(len(nodes), dtype=NODE_REC)
    for i, n in enumerate(nodes):
        if taint_ids is not None:
            rec[i]["taints"] = taint_ids.node_bits(n.taints)
        if ZONE_LABEL in n.labels:
            rec[i]["zone"] = (zone_ids or ZoneIds())(n.labels[ZONE_LABEL])
        d = name_digit(n.name)
        rec[i]["unschedulable"] = 1 if n.unschedulable else 0
        rec[i]["name_digit"] = d if d >= 0 else 0xFF
        rec[i]["allowed_pods"] = n.allocatable.get("pods", 110)
        rec[i]["alloc_milli_cpu"] = n.allocatable.get("cpu", 0)
        rec[i]["alloc_memory"] = n.allocatable.get("memory", 0)
    return rec


class DigitOrdinals:
    """Digit-aligned node ordinals (the host mirror's OrdinalAllocator,
    csrc/host/minisched.h): a node whose name ends in digit d
    gets the lowest free ordinal with ordinal % 10 == d, so every 30 consecutive
    ordinals hold at most 3 nodes of one digit whatever the informer Add order
    (the layout K1 pp's fast hash slots cover). Names without a digit, and
    digits whose residue is full up to the capacity, take the lowest free
    ordinal of any residue; so does a digit whose aligned slot lies past
    SPREAD_SLACK + 2 x (live nodes + 1) (skewed name digits would otherwise
    spread the table over up to 10x the ordinals).

    Skew fallback: alignment pays only while the table it
    builds is cheaper to sweep than a dense one. An aligned table spans
    ~10 x (largest digit share) x live rows, all on K1's fast path; a dense one
    spans live rows on the bit-scan path, which costs ~2.6x per row at config C
    (0.68 vs 0.264 ms, profiles/r04x_naming_*.log). So once SKEW_MIN_LIVE nodes
    are live and 10 x the largest digit share of the live nodes (this one
    included) exceeds SKEW_BREAK_EVEN = 2.6 (integer form: 100 x max count >
    26 x live), every allocation takes the lowest free ordinal of any residue.
    release() needs the node's digit to keep the shares current."""

    SPREAD_SLACK = 300
    SKEW_MIN_LIVE = 100
    SKEW_BREAK_EVEN_X10 = 26  # 10 x (10 x largest share) threshold, 2.6 in integers

    def __init__(self, capacity: int):
        import heapq  # noqa: F401  (free lists are min-heaps)

        self.cap = capacity
        self.next = list(range(10))
        self.free: List[List[int]] = [[] for _ in range(10)]
        self.high = 0
        self.live = 0
        self.count = [0] * 10  # live nodes per name digit

    def _lowest_any(self) -> int:
        import heapq

        best, bd = None, None
        for d in range(10):
            o = self.free[d][0] if self.free[d] else self.next[d]
            if o < self.cap and (best is None or o < best):
                best, bd = o, d
        if best is None:
            raise OverflowError("node table full")
        if self.free[bd] and self.free[bd][0] == best:
            heapq.heappop(self.free[bd])
        else:
            self.next[bd] += 10
        return best

    def skewed(self) -> bool:
        """True when the live digit mix makes a dense table cheaper than an aligned one."""
        return self.live >= self.SKEW_MIN_LIVE and 100 * max(self.count) > self.SKEW_BREAK_EVEN_X10 * self.live

    def allocate(self, digit: int) -> int:
        has_digit = 0 <= digit <= 9
        if has_digit:
            self.count[digit] += 1
        self.live += 1
        try:
            o = self._pick(digit, has_digit)
        except OverflowError:  # (full: the shares stay as they were)
            self.live -= 1
            if has_digit:
                self.count[digit] -= 1
            raise
        self.high = max(self.high, o + 1)
        return o

    def _pick(self, digit: int, has_digit: bool) -> int:
        import heapq

        spread = self.SPREAD_SLACK + 2 * self.live
        if self.skewed():
            return self._lowest_any()
        if has_digit and self.free[digit] and self.free[digit][0] < spread:
            return heapq.heappop(self.free[digit])
        if has_digit and self.next[digit] < self.cap and self.next[digit] < spread:
            o = self.next[digit]
            self.next[digit] += 10
            return o
        return self._lowest_any()

    def release(self, ordinal: int, digit: int) -> None:
        """Frees `ordinal`, held by a node whose name digit is `digit` (0..9, or -1)."""
        import heapq

        heapq.heappush(self.free[ordinal % 10], ordinal)
        self.live = max(0, self.live - 1)
        if 0 <= digit <= 9 and self.count[digit]:
            self.count[digit] -= 1
