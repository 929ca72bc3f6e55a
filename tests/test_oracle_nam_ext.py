"""MS_PLUGINS_NU_NN_NAM in general form (ABI 7, VERDICT r5 missing 6): preferred
terms whose NodeSelectorTerms hold any In / NotIn / Exists / DoesNotExist / Gt /
Lt requirements (several per term, ANDed) on the two encoded label keys, carried
as per-key value-id sets (ms_nam_term_set_ext). Pinned three ways on the CPU:
hand KATs of the requirement semantics (k8s.io/apimachinery labels.Requirement,
restated), the encoder's id sets against tests/_pyref.py's independent matcher on
label strings, and the oracle's general form against _pyref's literal loop on
v1-style objects (minisched.go:164-199 as written) and against its 16-B form.
"""
import numpy as np
import pytest

import _pyref
from minisched_amd import _lib, encode, synth
from minisched_amd.encode import Node, NodeSelectorRequirement as Req, Pod, PreferredTerm, ZONE_LABEL

L2 = "node.kubernetes.io/instance-type"


@pytest.mark.parametrize("op,values,label,expect", [
    ("In", ("a", "b"), "a", True), ("In", ("a",), None, False), ("In", ("a",), "c", False),
    ("NotIn", ("a",), "a", False), ("NotIn", ("a",), "c", True), ("NotIn", ("a",), None, True),
    ("Exists", (), "x", True), ("Exists", (), None, False),
    ("DoesNotExist", (), None, True), ("DoesNotExist", (), "", False),
    ("Gt", ("5",), "6", True), ("Gt", ("5",), "5", False), ("Gt", ("5",), "x6", False), ("Gt", ("5",), None, False),
    ("Gt", ("-3",), "-2", True), ("Gt", ("5",), "+7", True), ("Lt", ("5",), "4", True), ("Lt", ("5",), "05", False),
    ("Lt", ("0",), "-9223372036854775808", True), ("Lt", ("0",), "-9223372036854775809", False),
])
def test_requirement_semantics_kat(op, values, label, expect):
    labels = {} if label is None else {"k": label}
    r = Req("k", op, values)
    assert _pyref.requirement_matches(r, labels) is expect
    assert encode.requirement_holds(r, labels.get("k")) is expect


def test_empty_term_matches_nothing_and_unsupported_keys_refused():
    z, l2 = encode.ZoneIds(), encode.ZoneIds()
    nt = encode.NamTerms(L2, z, l2)
    assert nt.term(PreferredTerm(7, [])) == (7, 0, 0)
    assert not _pyref.term_matches(PreferredTerm(7, []), {ZONE_LABEL: "a"})
    with pytest.raises(encode.UnsupportedTerm):
        nt.term(PreferredTerm(7, [Req("kubernetes.io/hostname", "In", ("n1",))]))
    with pytest.raises(encode.UnsupportedTerm):
        nt.term_sets([[PreferredTerm(1, [Req(ZONE_LABEL, "Exists")])] * 5])
    with pytest.raises(ValueError):
        nt.term(PreferredTerm(7, [Req(ZONE_LABEL, "Gt", ("x",))]))
    with pytest.raises(ValueError):
        nt.term(PreferredTerm(101, [Req(ZONE_LABEL, "Exists")]))


def _universe(rng):
    zones = [f"z{i}" for i in range(5)]
    l2 = ["3", "10", "-4", "+8", "x7", "007", "12"]
    return zones, l2


def _random_req(rng, zones, l2):
    key = ZONE_LABEL if rng.random() < 0.5 else L2
    vals = zones if key == ZONE_LABEL else l2
    op = encode.NAM_OPERATORS[int(rng.integers(0, 6))]
    if op in ("In", "NotIn"):
        pool = vals + ["unseen"]
        return Req(key, op, tuple(rng.choice(pool, size=int(rng.integers(1, 3)), replace=False)))
    if op in ("Gt", "Lt"):
        return Req(key, op, (str(int(rng.integers(-6, 14))),))
    return Req(key, op)


def _random_labels(rng, zones, l2):
    lab = {}
    if rng.random() < 0.85:
        lab[ZONE_LABEL] = str(rng.choice(zones))
    if rng.random() < 0.8:
        lab[L2] = str(rng.choice(l2))
    return lab


def _bit(m, v):
    return (m >> v) & 1


@pytest.mark.parametrize("seed", range(6))
def test_id_sets_equal_the_requirements(seed):
    rng = np.random.default_rng(seed)
    zones, l2 = _universe(rng)
    zid, lid = encode.ZoneIds(), encode.ZoneIds()
    labels = [_random_labels(rng, zones, l2) for _ in range(60)]
    for lab in labels:  # the node records' value ids
        zid(lab.get(ZONE_LABEL))
        lid(lab.get(L2))
    nt = encode.NamTerms(L2, zid, lid)
    for _ in range(200):
        reqs = [_random_req(rng, zones, l2) for _ in range(int(rng.integers(0, 4)))]
        t = PreferredTerm(int(rng.integers(1, 101)), reqs)
        w, zm, lm = nt.term(t)
        for lab in labels:
            a, b = zid(lab.get(ZONE_LABEL)), lid(lab.get(L2))
            assert bool(_bit(zm, a) and _bit(lm, b)) == _pyref.term_matches(t, lab), (t, lab)


def _objects(rng, n_nodes, n_pods):
    zones, l2 = _universe(rng)
    nodes = []
    for i in range(n_nodes):
        name = f"node{i}" if rng.random() > 0.1 else f"node{i}q"
        nodes.append(Node(name, unschedulable=bool(rng.random() < 0.15), labels=_random_labels(rng, zones, l2)))
    pod_terms = []
    for _ in range(n_pods):
        terms = []
        for _ in range(int(rng.integers(0, 5))):
            reqs = [_random_req(rng, zones, l2) for _ in range(int(rng.integers(1, 3)))]
            if rng.random() < 0.05:
                reqs = []
            terms.append(PreferredTerm(int(rng.integers(1, 101)), reqs))
        pod_terms.append(terms)
    tol = encode.Toleration(key="node.kubernetes.io/unschedulable", operator="Exists")
    pods = [Pod(f"pod{j}" if rng.random() > 0.05 else f"pod{j}x", j,
                tolerations=[tol] if rng.random() < 0.2 else []) for j in range(n_pods)]
    return nodes, pods, pod_terms


def _records(nodes, pods, pod_terms):
    zid, lid = encode.ZoneIds(), encode.ZoneIds()
    nr = encode.node_records(nodes, zid)
    for i, n in enumerate(nodes):
        nr[i]["label2"] = lid(n.labels.get(L2))
    pr = encode.pod_records(pods, check_resources=False)
    ts = encode.NamTerms(L2, zid, lid).term_sets([t for t in pod_terms])
    sid = np.arange(1, len(pods) + 1)
    pr["pref_zone"], pr["pref_weight"] = sid & 0xFF, sid >> 8
    return nr, pr, ts


@pytest.mark.parametrize("seed,n_nodes,n_pods,weights", [(1, 1, 8, (1, 1)), (2, 9, 40, (1, 1)), (3, 40, 60, (1, 1)),
                                                         (4, 60, 40, (3, 2)), (5, 120, 30, (1, 1))])
def test_oracle_ext_equals_the_literal_loop_on_objects(oracle, seed, n_nodes, n_pods, weights):
    rng = np.random.default_rng(100 + seed)
    nodes, pods, pod_terms = _objects(rng, n_nodes, n_pods)
    nr, pr, ts = _records(nodes, pods, pod_terms)
    want = _pyref.schedule_nam(nodes, pods, pod_terms, weights=weights, seed=seed)
    for literal in (True, False):
        o = oracle.schedule_nam_ext(nr, pr, ts, weights=weights, literal=literal, seed=seed)
        got = list(zip(o["code"].tolist(), o["node"].tolist(), o["score"].tolist(), o["mask"].tolist()))
        assert got == want


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_16b_sets_equal_their_ext_form(oracle, seed):
    nr = synth.nodes(700, seed=seed, labels=True)
    nr["zone"][::97] = 255  # (id 255 is a labelled node)
    pr = synth.pods(300, seed=seed, term_sets=24)
    ts = synth.nam_term_sets(24, seed=seed)
    a = oracle.schedule_nam(nr, pr, ts, literal=False, seed=seed)
    b = oracle.schedule_nam_ext(nr, pr, _lib.nam_term_sets_to_ext(ts), literal=False, seed=seed)
    for k in ("node", "code", "score", "mask"):
        assert np.array_equal(a[k], b[k])


def test_random_ext_sets_generator_covers_the_operators():
    ts = synth.nam_term_sets_ext(64, seed=5)
    assert ts.shape == (64, _lib.NAM_SET_EXT_BYTES)
    w = ts.reshape(64, 4, 68)[:, :, 64]
    assert (w > 0).sum() > 64 and w.max() <= 100


def test_rescale_multiply_high_is_exact():
    # ms_affinity.hip f_r: floor(100 v / r) as umulhi(100 v, floor((2^32 - 1) / r) + 1) for the
    # rescale of every table entry (v <= 100; a rescale has r > 100, raw scores reach 400)
    r = np.arange(101, 65536, dtype=np.uint64)[:, None]
    v = np.arange(0, 101, dtype=np.uint64)[None, :]
    m = np.uint64(0xFFFFFFFF) // r + np.uint64(1)
    assert np.array_equal((np.uint64(100) * v * m) >> np.uint64(32), (np.uint64(100) * v) // r)
