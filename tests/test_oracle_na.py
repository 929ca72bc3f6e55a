"""MS_PLUGINS_NU_NN_NA on the CPU: NodeNumber + a normalising NodeAffinity score
plugin, with weights.

RunScorePlugins runs NodeAffinity's NormalizeScore (upstream
DefaultNormalizeScore(MaxNodeScore, reverse=false)) on the WHOLE, partially
filled list after every node (minisched.go:164-185). The oracle restates that
loop as written (literal, O(F^2) per pod) and in closed form (raw scores <= 100:
every entry keeps its raw score except the first feasible node in LIST order
with a non-zero raw score, which ends at 100); both must agree with each other
and with the pure-Python restatement on v1-style objects. Parity unpinned by
reference outputs: the reference registers no normalising plugin.
"""
import numpy as np
import pytest

import _pyref
from minisched_amd import encode, synth


def test_default_normalize_score_kats(oracle):
    assert oracle.default_normalize([0, 30, 50]).tolist() == [0, 60, 100]
    assert oracle.default_normalize([0, 0, 0]).tolist() == [0, 0, 0]
    assert oracle.default_normalize([0, 0], reverse=True).tolist() == [100, 100]
    assert oracle.default_normalize([200, 100]).tolist() == [100, 50]
    assert oracle.default_normalize([10, 40], reverse=True).tolist() == [75, 0]
    s = [0, 30, 50]
    _pyref.default_normalize_score(100, False, s)
    assert s == [0, 60, 100]


def test_in_loop_normalise_quirk_kat(oracle):
    # three feasible nodes, NodeAffinity raw scores [0, 50, 50] (node1, node2 in zone a,
    # the pod prefers a with weight 50), NodeNumber 0 everywhere (pod digit 9). The hook
    # after node1 lifts its 50 to 100; after node2 the list max is 100, so node2's 50
    # stays 50: node1 wins with 100 although both raw scores tie.
    zid = encode.ZoneIds()
    nodes = [encode.Node("node0"), encode.Node("node1", labels={encode.ZONE_LABEL: "a"}),
             encode.Node("node2", labels={encode.ZONE_LABEL: "a"})]
    pods = [encode.Pod("pod9", 9, preferred_zone=("a", 50))]
    assert _pyref.schedule_na(nodes, pods) == [(0, 1, 100, 0)]
    nr, pr = encode.node_records(nodes, zid), encode.pod_records(pods, zid)
    for literal in (True, False):
        o = oracle.schedule_na(nr, pr, literal=literal)
        assert (o["code"][0], o["node"][0], o["score"][0]) == (0, 1, 100)


def test_first_anchor_skips_infeasible_and_zero_nodes(oracle):
    # the anchor is the first FEASIBLE node with a non-zero raw score: an unschedulable
    # zone match before it does not count, a tolerating pod sees it
    zid = encode.ZoneIds()
    nodes = [encode.Node("node0", unschedulable=True, labels={encode.ZONE_LABEL: "a"}),
             encode.Node("node1"), encode.Node("node2", labels={encode.ZONE_LABEL: "a"}),
             encode.Node("node3", labels={encode.ZONE_LABEL: "a"})]
    tol = [encode.Toleration(key=encode.TAINT_NODE_UNSCHEDULABLE, operator="Exists")]
    pods = [encode.Pod("pod7", 7, preferred_zone=("a", 40)), encode.Pod("pod8", 8, tolerations=tol, preferred_zone=("a", 40))]
    want = _pyref.schedule_na(nodes, pods)
    assert want[0][1] == 2 and want[0][2] == 100  # node2 is pod7's anchor
    assert want[1][1] == 0 and want[1][2] == 100  # node0 is pod8's anchor (it tolerates)
    nr, pr = encode.node_records(nodes, zid), encode.pod_records(pods, zid)
    for literal in (True, False):
        o = oracle.schedule_na(nr, pr, literal=literal)
        assert [(int(c), int(n), int(s), int(m)) for c, n, s, m in zip(o["code"], o["node"], o["score"], o["mask"])] == want


@pytest.mark.parametrize("weights", [(1, 1), (2, 1), (3, 7), (10, 10)])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_literal_closed_form_and_pyref_agree(oracle, weights, seed):
    rng = np.random.default_rng(seed)
    n_nodes, n_pods = 120, 90
    nr = synth.nodes(n_nodes, seed=seed, zones=True)
    pr = synth.pods(n_pods, seed=seed, zones=True)
    pr["tolerates_unschedulable"][::7] = 1
    pr["name_digit"][::13] = -1
    nr["name_digit"][::11] = 0xFF
    nr["unschedulable"][rng.random(n_nodes) < 0.3] = 1
    lit = oracle.schedule_na(nr, pr, weights=weights, literal=True, seed=seed)
    cf = oracle.schedule_na(nr, pr, weights=weights, literal=False, seed=seed)
    for k in ("node", "code", "score", "mask", "key"):
        assert np.array_equal(lit[k], cf[k]), k
    # the v1-object restatement
    zname = {z: f"zone-{z}" for z in range(1, 9)}
    nodes = [encode.Node(f"node{i}" if nr["name_digit"][i] != 0xFF else f"node{i}x",
                         unschedulable=bool(nr["unschedulable"][i]),
                         labels={encode.ZONE_LABEL: zname[int(nr["zone"][i])]} if nr["zone"][i] else {})
             for i in range(n_nodes)]
    tol = [encode.Toleration(key=encode.TAINT_NODE_UNSCHEDULABLE, operator="Exists")]
    pods = [encode.Pod(f"pod{j}" if pr["name_digit"][j] >= 0 else f"pod{j}q", int(pr["ordinal"][j]),
                       tolerations=tol if pr["tolerates_unschedulable"][j] else [],
                       preferred_zone=(zname[int(pr["pref_zone"][j])], int(pr["pref_weight"][j])) if pr["pref_zone"][j] else None)
            for j in range(n_pods)]
    # name digits of the v1 names must match the records' digits
    assert all(encode.name_digit(p.name) == int(pr["name_digit"][j]) for j, p in enumerate(pods))
    got = _pyref.schedule_na(nodes, pods, weights=weights, seed=seed)
    for j, (code, node, score, mask) in enumerate(got):
        assert (code, node, score, mask) == (lit["code"][j], lit["node"][j], lit["score"][j], lit["mask"][j]), j


def test_raw_scores_above_100_break_the_closed_form(oracle):
    # why the ABI requires weights <= 100 (PreferredSchedulingTerm API validation): with a
    # raw score above 100 the hook rescales earlier entries and the closed form is wrong
    s = [0, 150, 0]
    _pyref.default_normalize_score(100, False, s)
    s[2] = 120
    _pyref.default_normalize_score(100, False, s)
    assert s == [0, 83, 100]  # the closed form would say [0, 100, 120]
    with pytest.raises(ValueError):
        encode.pod_records([encode.Pod("pod1", 1, preferred_zone=("a", 101))])


def test_weights_one_one_equal_unweighted_nunn_when_no_preferences(oracle):
    # no preferred terms: NodeAffinity scores 0 everywhere, the set reduces to NU+NN
    nr = synth.nodes(500, seed=4, zones=True)
    pr = synth.pods(300, seed=4)
    a = oracle.schedule_na(nr, pr, literal=False, seed=4)
    b = oracle.schedule(nr, pr, seed=4)
    for k in ("node", "code", "score", "mask"):
        assert np.array_equal(a[k], b[k]), k
