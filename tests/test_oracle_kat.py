"""Known-answer tests pinning the CPU oracle (runs without a GPU).

KAT sources:
  * README scenario — sched.go:70-140 (the reference's only executable answer).
  * NodeNumber digit rules — nodenumber.go:50-95.
  * selectHost / filter-first-failure / FitError — minisched.go:115-151,304-325.
  * LeastAllocated / fitsRequest arithmetic — upstream k8s v1.22.0 (restated,
    weights pinned by scheduler/plugin/plugins_test.go:839-858).
"""
import random

import numpy as np
import pytest

import _pyref
from minisched_amd import encode, synth
from minisched_amd.encode import Container, Node, Pod, Toleration


def recs_from(nodes, pods):
    return encode.node_records(nodes), encode.pod_records(pods)


def run(oracle, nodes, pods, **kw):
    nr, pr = recs_from(nodes, pods)
    return oracle.schedule(nr, pr, **kw)


def test_readme_scenario(oracle):
    # node0..node8 all Spec.Unschedulable (sched.go:74-85), pod1 (sched.go:91-101)
    nodes = [Node(f"node{i}", unschedulable=True) for i in range(9)]
    pod1 = [Pod("pod1", 1, containers=[Container()])]
    o = run(oracle, nodes, pod1)
    assert o["code"][0] == 2 and o["mask"][0] == 1 and o["node"][0] == -1  # FitError{NodeUnschedulable}
    # node10 added (sched.go:121-129) -> pod1 bound to node10 (ordinal 9), NodeNumber 1 != 0 -> score 0
    nodes.append(Node("node10"))
    o = run(oracle, nodes, pod1)
    assert (o["code"][0], o["node"][0], o["score"][0], o["mask"][0]) == (0, 9, 0, 0)
    # the pure restatement agrees
    assert _pyref.schedule(nodes, pod1) == [(0, 9, 0, 0)]


def test_readme_scenario_via_synth_helper(oracle):
    first, node10, pod1 = synth.readme_scenario()
    o = oracle.schedule(first, pod1)
    assert (o["code"][0], o["mask"][0]) == (2, 1)
    o = oracle.schedule(np.concatenate([first, node10]), pod1)
    assert (o["code"][0], o["node"][0], o["score"][0]) == (0, 9, 0)


def test_nodenumber_digit_rules(oracle):
    # nodenumber.go:21,81-95: only the LAST char counts; node17 and node7 match pod7, nodeA scores 0
    nodes = [Node("node17"), Node("node7"), Node("nodeA"), Node("node8")]
    pod = [Pod("pod7", 7)]
    for seed in range(1, 20):
        o = run(oracle, nodes, pod, seed=seed)
        assert o["code"][0] == 0 and o["score"][0] == 10 and o["node"][0] in (0, 1)
    # only nodeA present -> score 0, success
    o = run(oracle, [Node("nodeA")], pod)
    assert (o["code"][0], o["node"][0], o["score"][0]) == (0, 0, 0)
    assert encode.name_digit("node10") == 0 and encode.name_digit("nodeA") == -1 and encode.name_digit("x-9") == 9


def test_nondigit_pod_is_score_error(oracle):
    # PreScore writes no state (nodenumber.go:53-56) -> Score fails -> framework.Error
    o = run(oracle, [Node("node1")], [Pod("podX", 0)])
    assert (o["code"][0], o["node"][0], o["mask"][0]) == (1, -1, 0)
    # ...but with no feasible node the FitError comes first (minisched.go:50-55)
    o = run(oracle, [Node("node1", unschedulable=True)], [Pod("podX", 0)])
    assert (o["code"][0], o["mask"][0]) == (2, 1)


def test_empty_cluster_fit_error_empty_mask(oracle):
    o = run(oracle, [], [Pod("pod1", 1)])
    assert (o["code"][0], o["mask"][0], o["node"][0]) == (2, 0, -1)


@pytest.mark.parametrize(
    "tol,expect",
    [
        (Toleration(key="node.kubernetes.io/unschedulable", operator="Exists", effect="NoSchedule"), True),
        (Toleration(key="node.kubernetes.io/unschedulable", operator="Exists"), True),  # empty effect = all
        (Toleration(operator="Exists"), True),  # empty key + Exists tolerates everything
        (Toleration(key="node.kubernetes.io/unschedulable", effect="NoSchedule"), True),  # Equal, value ""
        (Toleration(key="node.kubernetes.io/unschedulable", value="x", effect="NoSchedule"), False),
        (Toleration(key="node.kubernetes.io/unschedulable", operator="Exists", effect="NoExecute"), False),
        (Toleration(key="other", operator="Exists"), False),
        (Toleration(key="node.kubernetes.io/unschedulable", operator="Bogus"), False),
    ],
)
def test_toleration_matching(oracle, tol, expect):
    assert encode.tolerates_unschedulable([tol]) is expect
    o = run(oracle, [Node("node3", unschedulable=True)], [Pod("pod3", 3, tolerations=[tol])])
    if expect:
        assert (o["code"][0], o["node"][0], o["score"][0]) == (0, 0, 10)
    else:
        assert (o["code"][0], o["mask"][0]) == (2, 1)


@pytest.mark.parametrize(
    "req,cap,expect",
    [(0, 0, 0), (5, 0, 0), (4001, 4000, 0), (1000, 4000, 75), (0, 4000, 100), (4000, 4000, 0), (1, 3, 66)],
)
def test_least_requested_kat(oracle, req, cap, expect):
    assert oracle.lib().msor_least_requested(req, cap) == expect
    assert _pyref.least_requested(req, cap) == expect


def test_fit_and_least_allocated_kat(oracle):
    GiB = 1 << 30
    nodes = [Node("node0", allocatable={"cpu": 4000, "memory": 8 * GiB, "pods": 110})]
    # 1000m / 2GiB on an empty 4000m / 8GiB node: cpu 75, mem 75 -> 75; NN pod0 vs node0 -> +10
    pod = Pod("pod0", 0, containers=[Container({"cpu": 1000, "memory": 2 * GiB})])
    o = run(oracle, nodes, [pod], plugin_set=1)
    assert (o["code"][0], o["score"][0]) == (0, 85)
    # request-less pod: filter sees 0/0 (only the pod-count check), score uses 100m/200MiB
    bare = Pod("pod1", 1, containers=[Container()])
    rc, rm, nc, nm = encode.pod_requests(bare)
    assert (rc, rm, nc, nm) == (0, 0, 100, 200 * 1024 * 1024)
    o = run(oracle, nodes, [bare], plugin_set=1)
    s_cpu = (4000 - 100) * 100 // 4000
    s_mem = (8 * GiB - 200 * 1024 * 1024) * 100 // (8 * GiB)
    assert (o["code"][0], o["score"][0]) == (0, (s_cpu + s_mem) // 2)
    # explicit zero stays zero for the non-zero pair
    z = Pod("pod2", 2, containers=[Container({"cpu": 0, "memory": 0})])
    assert encode.pod_requests(z) == (0, 0, 0, 0)
    # Insufficient cpu -> FitError{NodeResourcesFit}
    big = Pod("pod3", 3, containers=[Container({"cpu": 5000})])
    o = run(oracle, nodes, [big], plugin_set=1)
    assert (o["code"][0], o["mask"][0]) == (2, 2)
    # Too many pods: allowed 1, one pod already assumed -> second is rejected even with zero requests
    one = [Node("node0", allocatable={"cpu": 4000, "memory": 8 * GiB, "pods": 1})]
    o = run(oracle, one, [bare, bare], plugin_set=1, mode=1)
    assert list(o["code"]) == [0, 2] and o["mask"][1] == 2
    # NU rejection is charged to NU only (first failing plugin, minisched.go:130-137)
    two = [Node("node0", unschedulable=True, allocatable={"cpu": 10, "memory": 10, "pods": 110})]
    o = run(oracle, two, [big], plugin_set=1)
    assert (o["code"][0], o["mask"][0]) == (2, 1)
    # init containers: max with the container sum; overhead added
    ic = Pod("pod4", 4, containers=[Container({"cpu": 100})], init_containers=[Container({"cpu": 700})],
             overhead={"cpu": 50})
    assert encode.pod_requests(ic)[0] == 750


@pytest.mark.parametrize("where", ["containers", "init_containers", "overhead"])
@pytest.mark.parametrize("name,qty", [("amd.com/gpu", 1), ("ephemeral-storage", 1 << 30),
                                      ("hugepages-2Mi", 2 << 20), ("amd.com/gpu", 0)])
def test_unsupported_requests_are_refused(where, name, qty):
    # upstream fitsRequest also checks ephemeral-storage and every scalar resource
    # the pod requests (k8s@v1.22.0 noderesources/fit.go); ms_pod_rec carries cpu and memory only, so
    # a pod requesting anything else (an explicit 0 included: it defeats the "all requests are 0"
    # early return) must be refused, never encoded as a request-less pod that passes Fit everywhere
    GiB = 1 << 30
    kw = {"containers": [Container({"cpu": 100})]}
    if where == "overhead":
        kw["overhead"] = {name: qty}
    else:
        kw[where] = kw.get(where, []) + [Container({name: qty})]
    p = Pod("pod1", 1, **kw)
    assert encode.unsupported_request(p) == name
    with pytest.raises(encode.UnsupportedResource, match=name):
        encode.pod_requests(p)
    with pytest.raises(encode.UnsupportedResource):
        encode.pod_records([Pod("pod0", 0), p])
    # a plugin set without NodeResourcesFit reads no resources: the cpu / memory fields still encode
    rec = encode.pod_records([p], check_resources=False)[0]
    assert rec["req_milli_cpu"] == 100
    # node-side allocatable of other names is accepted and ignored (no admitted pod requests them)
    nr = encode.node_records([Node("node0", allocatable={"cpu": 4000, "memory": 8 * GiB, "pods": 110,
                                                         "ephemeral-storage": 100 * GiB, "amd.com/gpu": 8})])
    assert (nr[0]["alloc_milli_cpu"], nr[0]["alloc_memory"]) == (4000, 8 * GiB)


def _random_objects(rng, n_nodes, n_pods, resources):
    GiB = 1 << 30
    nodes = []
    for i in range(n_nodes):
        name = f"node{i}" if rng.random() > 0.1 else f"node-{chr(97 + i % 26)}"
        alloc = {"pods": rng.choice([1, 2, 110])}
        if resources:
            alloc.update(cpu=rng.choice([0, 500, 1000, 4000]), memory=rng.choice([0, 1, 2, 8]) * GiB)
        nodes.append(Node(name, unschedulable=rng.random() < 0.3, allocatable=alloc))
    pods = []
    for j in range(n_pods):
        name = f"pod{j}" if rng.random() > 0.1 else f"pod-{chr(97 + j % 26)}"
        tols = [Toleration(operator="Exists")] if rng.random() < 0.2 else []
        reqs = {}
        if resources and rng.random() < 0.8:
            if rng.random() < 0.9:
                reqs["cpu"] = rng.choice([0, 100, 300, 1500])
            if rng.random() < 0.9:
                reqs["memory"] = rng.choice([0, 128, 512, 3000]) * (1 << 20)
        pods.append(Pod(name, j * 7 + 3, tolerations=tols, containers=[Container(reqs)]))
    return nodes, pods


@pytest.mark.parametrize("resources", [False, True])
@pytest.mark.parametrize("sequential", [False, True])
def test_oracle_matches_python_restatement(oracle, resources, sequential):
    rng = random.Random(1234 + resources * 2 + sequential)
    for trial in range(25):
        nodes, pods = _random_objects(rng, rng.randint(0, 40), rng.randint(1, 30), resources)
        seed = rng.randint(0, 2**64 - 1)
        want = _pyref.schedule(nodes, pods, resources=resources, sequential=sequential, seed=seed)
        o = run(oracle, nodes, pods, plugin_set=int(resources), mode=int(sequential), seed=seed)
        got = list(zip(o["code"].tolist(), o["node"].tolist(), o["score"].tolist(), o["mask"].tolist()))
        assert got == want, f"trial {trial}"


def test_faithful_names_form_matches_soa(oracle):
    rng = np.random.default_rng(7)
    n, p = 300, 200
    node_names = [f"node{i}" if i % 13 else f"node-x{i}a" for i in range(n)]
    flags = (rng.random(n) < 0.2).astype(np.uint8)
    pod_names = [f"pod{j}" if j % 17 else f"pod-{j}z" for j in range(p)]
    tol = (rng.random(p) < 0.05).astype(np.uint8)
    ords = np.arange(p, dtype=np.uint32) * 3 + 1
    a = oracle.schedule_nunn_names(node_names, flags, pod_names, tol, ords, seed=5)
    nodes = [Node(nm, unschedulable=bool(f)) for nm, f in zip(node_names, flags)]
    pods = [Pod(nm, int(o), tolerations=[Toleration(operator="Exists")] if t else []) for nm, o, t in zip(pod_names, ords, tol)]
    b = run(oracle, nodes, pods, seed=5)
    for k in ("node", "score", "code", "mask"):
        assert np.array_equal(a[k], b[k]), k


def test_omp_matches_serial(oracle):
    nr = synth.nodes(3000, seed=2)
    pr = synth.pods(500, seed=2)
    a = oracle.schedule(nr, pr, seed=2)
    b = oracle.schedule_nunn_omp(nr, pr, seed=2, threads=4)
    for k in ("node", "score", "code", "mask", "key"):
        assert np.array_equal(a[k], b[k]), k


def test_tiebreak_is_order_independent_and_spread(oracle):
    # the winner is a pure function of (seed, pod, node): permuting the LIST
    # order (while keeping ordinals) cannot change it, and among T tied nodes
    # every node wins for some pods.
    T = 8
    nodes = [Node(f"node{10 * i + 3}") for i in range(T)]  # all digit 3 -> all tie at 10
    pods = [Pod(f"pod{10 * j + 3}", j) for j in range(4000)]
    o = run(oracle, nodes, pods, seed=99)
    counts = np.bincount(o["node"], minlength=T)
    assert counts.min() > 4000 / T * 0.8 and counts.max() < 4000 / T * 1.2
    for j in range(0, 4000, 97):
        best = max(range(T), key=lambda i: _pyref.key(10, _pyref.h32(99, j, i), i))
        assert o["node"][j] == best


def test_sequential_equals_batched_for_nunn(oracle):
    # NU+NN never read mutable NodeInfo state, so queue order cannot change placements
    nr = synth.nodes(2000, seed=3)
    pr = synth.pods(3000, seed=3)
    a = oracle.schedule(nr, pr, mode=0, seed=3)
    b = oracle.schedule(nr, pr, mode=1, seed=3)
    for k in ("node", "score", "code", "mask"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("T,stride", [(2, 1), (3, 1), (10, 1), (64, 1), (16, 10), (32, 1000)])
def test_tiebreak_uniform_over_tied_nodes(T, stride):
    # Rule r3 (minisched_gpu.h) stands in for selectHost's reservoir choice
    # (minisched.go:316-321): over many pods each of T tied nodes must win
    # about 1/T of the time, also for consecutive ordinals (the additive
    # node term's weakest case). Chi-square against uniform, 5-sigma bound.
    P = 20000
    ords = np.arange(T, dtype=np.uint64) * stride
    wins = np.zeros(T, dtype=np.int64)
    for seed in (1, 7):
        for j in range(seed * 1000003, seed * 1000003 + P // 2):  # disjoint pod ordinals per seed
            hs = [_pyref.key(10, _pyref.h32(seed, j, int(o)), int(o)) for o in ords]
            wins[int(np.argmax(hs))] += 1
    exp = P / T
    chi2 = float(((wins - exp) ** 2 / exp).sum())
    dof = T - 1
    assert chi2 < dof + 5 * np.sqrt(2 * dof), (chi2, wins.tolist())


def test_tiebreak_hash_is_invertible():
    # Rule r3: for one pod the hash is a bijection of the node ordinal, so hashes never
    # tie and K1 recovers the winning row from its hash alone (ms_internal.h tb_unhash,
    # same constants: the inverses of 0xc2b2ae35, 0x85ebca6b and 0x9E3779 mod 2^32)
    rng = np.random.default_rng(5)
    M = 0xFFFFFFFF

    def unhash(a, h):
        h = (h * 0x7ED1B41D) & M
        h ^= h >> 16
        h = (h * 0xA5CB9243) & M
        h ^= h >> 16
        return ((h - a) * 0xF2B382C9) & M

    for _ in range(2000):
        seed, pod, node = int(rng.integers(0, 2**63)), int(rng.integers(0, 2**32)), int(rng.integers(0, 0xFFFFF))
        a = _pyref.fmix32(_pyref.seed32(seed) ^ pod)
        assert unhash(a, _pyref.h32(seed, pod, node)) == node
    hs = {_pyref.h32(9, 4242, n) for n in range(20000)}
    assert len(hs) == 20000


def test_digit_ordinals_allocator():
    # encode.DigitOrdinals == the host mirror's OrdinalAllocator (tests/cpp/test_host.cpp
    # checks the same sequence): ordinal % 10 == name digit, holes reused, no-digit names
    # fill the lowest free ordinal, at most 3 of one digit per 30 consecutive ordinals
    from minisched_amd import encode

    a = encode.DigitOrdinals(100)
    got = [a.allocate(d) for d in (7, 7, 7, 3, -1, 0, 7, -1, 9, 3)]
    assert got == [7, 17, 27, 3, 0, 10, 37, 1, 9, 13]
    a.release(17, 7)
    assert a.allocate(7) == 17
    a.release(27, 7)
    assert a.allocate(-1) == 2
    rng = np.random.default_rng(5)
    b = encode.DigitOrdinals(12_000)
    dig = np.full(12_000, -2)
    for d in rng.integers(0, 10, 10_000):
        dig[b.allocate(int(d))] = d
    for g in range(0, 12_000, 30):
        w = dig[g:g + 30]
        assert max((w == d).sum() for d in range(10)) <= 3
    assert b.high <= 12_000
    full = encode.DigitOrdinals(12)
    assert sorted(full.allocate(5) for _ in range(12)) == list(range(12))
    with pytest.raises(OverflowError):
        full.allocate(5)
    # skewed digits (every name ends in 0): aligned slots only within the spread
    # bound, then dense; the sweep extent stays ~2x the node count, not 10x
    sk = encode.DigitOrdinals(100_000)
    got = [sk.allocate(0) for _ in range(5000)]
    assert len(set(got)) == 5000 and sk.high <= 2 * 5000 + sk.SPREAD_SLACK + 2
    assert got[:30] == list(range(0, 300, 10))  # aligned while within the bound
    # ... and dense once SKEW_MIN_LIVE nodes are live
    assert sk.skewed() and sk.high <= 5000 + sk.SPREAD_SLACK


def test_digit_ordinals_skew_fallback():
    # the switch: 10 x the largest live digit share above 2.6 (integer form
    # 100 x max count > 26 x live) once SKEW_MIN_LIVE nodes are live -> dense ordinals
    from minisched_amd import encode

    rng = np.random.default_rng(9)
    n = 50_000
    # i.i.d. uniform digits stay aligned: every 30 ordinals hold <= 3 of a digit
    iid = encode.DigitOrdinals(n + n // 10)
    dig = np.full(n + n // 10, -2)
    for d in rng.integers(0, 10, n):
        dig[iid.allocate(int(d))] = d
    assert not iid.skewed()
    w = dig[: (iid.high // 30) * 30].reshape(-1, 30)
    assert max(int((w == d).sum(1).max()) for d in range(10)) <= 3
    # 70 % of the names end in 0: dense after the first SKEW_MIN_LIVE nodes, so the
    # table spans ~n rows, not the bounded spread's ~2n (profiles/r04x_naming_layouts.log)
    sk = encode.DigitOrdinals(2 * n)
    digits = np.where(rng.random(n) < 0.7, 0, rng.integers(0, 10, n))
    ords = [sk.allocate(int(d)) for d in digits]
    assert sk.skewed() and len(set(ords)) == n and sk.high <= n + sk.SPREAD_SLACK
    # the threshold itself: 26 % of one digit among 100 live nodes is not skewed, 27 % is
    t = encode.DigitOrdinals(10_000)
    for i in range(100):
        t.allocate(0 if i < 26 else 1 + i % 9)
    assert max(t.count) == 26 and not t.skewed()
    t.allocate(0)
    assert 100 * 27 > 26 * 101 and t.skewed()
    # releasing skewed nodes brings alignment back
    for o, d in zip(ords, digits):
        if d == 0:
            sk.release(o, 0)
    assert not sk.skewed()
    o = sk.allocate(3)
    assert o % 10 == 3
