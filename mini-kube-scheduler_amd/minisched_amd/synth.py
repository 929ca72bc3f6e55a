"""Synthetic clusters for BASELINE.json's configs.

All draws come from splitmix64: the k-th output of stream `s` under seed
`seed` is mix64(state + (k+1) * golden) with state = seed ^ (s * 0xD1B54A32D192ED03),
i.e. one independent splitmix64 sequence per column. Everything is vectorised
numpy uint64 arithmetic (wrapping), so any prefix/slice can be generated
without the rest.

Nodes  : ordinal i, name "node{i}" -> digit i % 10, unschedulable iff u % 1000 < 100.
Pods   : ordinal j, name "pod{j}"  -> digit j % 10, tolerates iff u % 1000 < 20.
Config E nodes: alloc cpu {1000,2000,4000,8000} m, memory {2,4,8,16} GiB, 110 pods.
Config E pods : 10 % have no requests (non-zero defaults 100 m / 200 MiB apply),
                the rest cpu 100..2000 m step 100, memory 128..2048 MiB step 128.
"""
from __future__ import annotations

import numpy as np

from ._lib import NODE_REC, POD_REC

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
STREAM_SALT = np.uint64(0xD1B54A32D192ED03)
MiB = 1 << 20
GiB = 1 << 30

# column streams
S_NODE_UNSCHED, S_POD_TOL, S_NODE_CPU, S_NODE_MEM, S_POD_NOREQ, S_POD_CPU, S_POD_MEM = 1, 2, 3, 4, 5, 6, 7
S_NODE_ZONE, S_POD_ZONE, S_POD_ZWEIGHT = 8, 9, 10
S_NODE_HARD, S_NODE_SOFT, S_POD_TOLH, S_POD_TOLS = 11, 12, 13, 14
S_NODE_LABEL2, S_POD_TERMSET, S_TERMSETS = 15, 16, 17
N_ZONES = 8
N_LABEL2 = 4  # second-label value ids 1..4 (MS_PLUGINS_NU_NN_NAM)
# MS_PLUGINS_NU_TT_NN taint universe of the synthetic clusters: 3 NoSchedule /
# NoExecute taint ids (bits 0-2 of ms_node_rec.taints) and 6 PreferNoSchedule
# ids (bits 8-13)
N_HARD_TAINTS, N_SOFT_TAINTS = 3, 6


def _bits(seed: int, stream: int, start: int, n: int, nbits: int, per_mille: int) -> np.ndarray:
    """Per record a mask of nbits independent bits, each set with probability per_mille / 1000."""
    m = np.zeros(n, dtype=np.uint32)
    for b in range(nbits):
        u = stream_u64(seed, stream * 16 + b, start, n)
        m |= ((u % np.uint64(1000)) < np.uint64(per_mille)).astype(np.uint32) << np.uint32(b)
    return m

DEFAULT_MILLI_CPU_REQUEST = 100  # k8s@v1.22.0 pkg/scheduler/util/non_zero.go
DEFAULT_MEMORY_REQUEST = 200 * MiB


def mix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def stream_u64(seed: int, stream: int, start: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        state = np.uint64(seed) ^ (np.uint64(stream) * STREAM_SALT)
        k = np.arange(start, start + n, dtype=np.uint64) + np.uint64(1)
        return mix64(state + k * GOLDEN)


def nodes(n: int, seed: int = 1, start: int = 0, resources: bool = False, zones: bool = False,
          taints: bool = False, labels: bool = False) -> np.ndarray:
    """Node records for ordinals [start, start+n). zones: topology zone labels
    for MS_PLUGINS_NU_NN_NA (value ids 1..8, 5 % of nodes unlabelled). taints:
    for MS_PLUGINS_NU_TT_NN, each NoSchedule taint id on 4 % of nodes and each
    PreferNoSchedule id on 30 %. labels (MS_PLUGINS_NU_NN_NAM): the zone labels
    and a second label (value ids 1..4, 10 % unlabelled)."""
    rec = np.zeros(n, dtype=NODE_REC)
    i = np.arange(start, start + n, dtype=np.int64)
    rec["name_digit"] = (i % 10).astype(np.uint8)
    rec["unschedulable"] = (stream_u64(seed, S_NODE_UNSCHED, start, n) % np.uint64(1000) < np.uint64(100)).astype(
        np.uint8
    )
    rec["allowed_pods"] = 110
    if resources:
        cpu = np.array([1000, 2000, 4000, 8000], dtype=np.int64)
        mem = np.array([2, 4, 8, 16], dtype=np.int64) * GiB
        rec["alloc_milli_cpu"] = cpu[(stream_u64(seed, S_NODE_CPU, start, n) % np.uint64(4)).astype(np.int64)]
        rec["alloc_memory"] = mem[(stream_u64(seed, S_NODE_MEM, start, n) % np.uint64(4)).astype(np.int64)]
    if zones or labels:
        u = stream_u64(seed, S_NODE_ZONE, start, n)
        rec["zone"] = np.where(u % np.uint64(100) < np.uint64(5), 0, 1 + (u >> np.uint64(8)) % np.uint64(N_ZONES))
    if labels:
        u = stream_u64(seed, S_NODE_LABEL2, start, n)
        rec["label2"] = np.where(u % np.uint64(100) < np.uint64(10), 0, 1 + (u >> np.uint64(8)) % np.uint64(N_LABEL2))
    if taints:
        rec["taints"] = _bits(seed, S_NODE_HARD, start, n, N_HARD_TAINTS, 40) | (
            _bits(seed, S_NODE_SOFT, start, n, N_SOFT_TAINTS, 300) << np.uint32(8))
    return rec


def pods(n: int, seed: int = 1, start: int = 0, resources: bool = False, zones: bool = False,
         taints: bool = False, term_sets: int = 0) -> np.ndarray:
    """Pod records for ordinals [start, start+n). zones: 70 % of pods carry one
    preferred zone term (zone 1..8, weight 1..100) for MS_PLUGINS_NU_NN_NA.
    taints: MS_PLUGINS_NU_TT_NN tolerated taint ids (each with probability
    0.3), in the bytes that set shares with the NodeAffinity term
    (tol_hard = pref_zone, tol_soft = pref_weight, minisched_gpu.h).
    term_sets = K > 0 (MS_PLUGINS_NU_NN_NAM): 85 % of pods name one of K term
    sets (id 1..K, synth.nam_term_sets) in pref_zone | pref_weight << 8."""
    rec = np.zeros(n, dtype=POD_REC)
    j = np.arange(start, start + n, dtype=np.int64)
    rec["ordinal"] = j.astype(np.uint32)
    rec["name_digit"] = (j % 10).astype(np.int8)
    rec["tolerates_unschedulable"] = (
        stream_u64(seed, S_POD_TOL, start, n) % np.uint64(1000) < np.uint64(20)
    ).astype(np.uint8)
    if resources:
        noreq = stream_u64(seed, S_POD_NOREQ, start, n) % np.uint64(10) == np.uint64(0)
        cpu = (np.int64(100) * (np.int64(1) + (stream_u64(seed, S_POD_CPU, start, n) % np.uint64(20)).astype(np.int64)))
        mem = np.int64(128 * MiB) * (np.int64(1) + (stream_u64(seed, S_POD_MEM, start, n) % np.uint64(16)).astype(np.int64))
        rec["req_milli_cpu"] = np.where(noreq, 0, cpu)
        rec["req_memory"] = np.where(noreq, 0, mem)
        rec["nonzero_milli_cpu"] = np.where(noreq, DEFAULT_MILLI_CPU_REQUEST, cpu)
        rec["nonzero_memory"] = np.where(noreq, DEFAULT_MEMORY_REQUEST, mem)
    if zones:
        u = stream_u64(seed, S_POD_ZONE, start, n)
        w = stream_u64(seed, S_POD_ZWEIGHT, start, n)
        rec["pref_zone"] = np.where(u % np.uint64(10) < np.uint64(7), 1 + (u >> np.uint64(8)) % np.uint64(N_ZONES), 0)
        rec["pref_weight"] = np.where(rec["pref_zone"] > 0, 1 + w % np.uint64(100), 0)
    if taints:
        set_tolerations(rec, _bits(seed, S_POD_TOLH, start, n, N_HARD_TAINTS, 300),
                        _bits(seed, S_POD_TOLS, start, n, N_SOFT_TAINTS, 300))
    if term_sets:
        u = stream_u64(seed, S_POD_TERMSET, start, n)
        sid = np.where(u % np.uint64(100) < np.uint64(85), 1 + (u >> np.uint64(8)) % np.uint64(term_sets), 0)
        rec["pref_zone"] = (sid & np.uint64(0xFF)).astype(np.uint8)
        rec["pref_weight"] = (sid >> np.uint64(8)).astype(np.uint8)
    return rec


def nam_term_sets(k: int, seed: int = 1) -> np.ndarray:
    """K random MS_PLUGINS_NU_NN_NAM term sets (uint8 (K, 16), ms_nam_term_set):
    1..4 terms each on the zone label (key 0, values 1..8) or the second label
    (key 1, values 1..4), 1 in 8 of them Exists (0xFF), weights 1..100 — so a
    node matching several terms scores above 100 and the in-loop hook rescales."""
    from ._lib import nam_term_sets_array

    u = stream_u64(seed, S_TERMSETS, 0, 16 * k).reshape(k, 16)
    sets = []
    for i in range(k):
        nt = 1 + int(u[i, 0] % np.uint64(4))
        terms = []
        for t in range(nt):
            x = int(u[i, 1 + t])
            key = x & 1
            value = 0xFF if (x >> 1) % 8 == 0 else 1 + (x >> 4) % (N_ZONES if key == 0 else N_LABEL2)
            terms.append((key, value, 1 + (x >> 12) % 100))
        sets.append(terms)
    return nam_term_sets_array(sets)


def nam_term_sets_ext(k: int, seed: int = 1, n_zone: int = N_ZONES, n_label2: int = N_LABEL2) -> np.ndarray:
    """K random term sets in general form (uint8 (K, 272), ms_nam_term_set_ext): 1..4
    terms with requirements on one or both keys, each In (1-3 ids), NotIn (all
    but 1-3 ids, the absent label included), Exists, DoesNotExist, or Gt / Lt
    (the ids above / below a threshold, as a shim whose value ids follow the
    numeric label values would give them); about 1 term in 16 has no requirement
    (matches nothing); weights 1..100. Value ids up to 255 (id 255 appears)."""
    from ._lib import nam_term_sets_ext_array

    rng = np.random.default_rng(int(seed) * 7919 + k)
    top = {0: n_zone, 1: n_label2}

    def ids(kk):
        pool = list(range(1, top[kk] + 1)) + [255]
        return [int(x) for x in rng.choice(pool, size=int(rng.integers(1, 4)), replace=False)]

    def req_mask(kk):
        op = int(rng.integers(0, 6))
        full = (1 << 256) - 1
        if op == 0:  # In
            return sum(1 << v for v in set(ids(kk)))
        if op == 1:  # NotIn
            return full & ~sum(1 << v for v in set(ids(kk)))
        if op == 2:  # Exists
            return full & ~1
        if op == 3:  # DoesNotExist
            return 1
        t = int(rng.integers(0, top[kk] + 1))
        return sum(1 << v for v in range(t + 1, 256)) if op == 4 else sum(1 << v for v in range(1, t))

    sets = []
    for _ in range(k):
        terms = []
        for _ in range(int(rng.integers(1, 5))):
            w = int(rng.integers(1, 101))
            if rng.integers(0, 16) == 0:
                terms.append((w, 0, 0))
                continue
            which = int(rng.integers(0, 3))  # 0: zone only, 1: label2 only, 2: both
            zm = req_mask(0) if which in (0, 2) else (1 << 256) - 1
            lm = req_mask(1) if which in (1, 2) else (1 << 256) - 1
            if which == 2 and rng.integers(0, 3) == 0:
                zm &= req_mask(0)  # two requirements on one key: ANDed
            terms.append((w, zm, lm))
        sets.append(terms)
    return nam_term_sets_ext_array(sets)


def set_tolerations(rec: np.ndarray, tol_hard, tol_soft) -> None:
    """MS_PLUGINS_NU_TT_NN: bit t of tol_hard / tol_soft = some toleration of the
    pod tolerates NoSchedule / PreferNoSchedule taint id t (ms_pod_rec.tol_hard,
    .tol_soft: the bytes of the NodeAffinity term)."""
    rec["pref_zone"] = np.asarray(tol_hard, dtype=np.uint8)
    rec["pref_weight"] = np.asarray(tol_soft, dtype=np.uint8)


# BASELINE.md §3
CONFIGS = {
    "A": dict(nodes=10, pods=1, plugins="NU+NN", mode="sequential"),
    "B": dict(nodes=5_000, pods=10_000, plugins="NU+NN", mode="sequential"),
    "C": dict(nodes=100_000, pods=100_000, plugins="NU+NN", mode="batched-node-sharded"),
    "D": dict(nodes=50_000, pods=1_000_000, plugins="NU+NN", mode="batched"),
    "E": dict(nodes=50_000, pods=200_000, plugins="NU+NRF+NN+LA", mode="sequential"),
}


def readme_scenario():
    """sched.go:70-140: node0..node8 unschedulable, pod1; later node10 (schedulable).

    Returns (first_nodes, node10, pod1) as records; ordinals 0..8 for node0..8
    and 9 for node10 (ordinal assignment is the caller's, names carry the digit).
    """
    first = np.zeros(9, dtype=NODE_REC)
    first["unschedulable"] = 1
    first["name_digit"] = np.arange(9, dtype=np.uint8)
    first["allowed_pods"] = 110
    node10 = np.zeros(1, dtype=NODE_REC)
    node10["name_digit"] = 0  # "node10"[-1] == '0'
    node10["allowed_pods"] = 110
    pod1 = np.zeros(1, dtype=POD_REC)
    pod1["ordinal"] = 1
    pod1["name_digit"] = 1
    return first, node10, pod1
