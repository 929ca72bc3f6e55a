"""TaintToleration with RunScorePlugins' in-loop reverse normalise hook (plugin
set MS_PLUGINS_NU_TT_NN) — the oracle on the CPU.

RunScorePlugins (/root/reference/minisched/minisched.go:164-185) writes entry
k of a plugin's NodeScoreList and immediately calls its NormalizeScore on the
WHOLE list, whose later entries are still the zeros of
createPluginToNodeScores (:327-334). TaintToleration's NormalizeScore is
upstream DefaultNormalizeScore(MaxNodeScore, reverse=true)
(k8s@v1.22.0 pkg/scheduler/framework/plugins/tainttoleration/
taint_toleration.go, helper/normalize_score.go; not in the container, restated).
The oracle runs that loop literally (O(F^2) per pod) and as a closed form;
this file checks both against each other and against a transcription of the
loop in Python, and pins hand-derived known answers.
"""
import numpy as np
import pytest

from minisched_amd import _lib, synth


def py_default_normalize(scores, max_priority=100, reverse=False):
    # helper.DefaultNormalizeScore, transcribed
    max_count = max(scores) if scores else 0
    if max_count == 0:
        if reverse:
            for i in range(len(scores)):
                scores[i] = max_priority
        return
    for i in range(len(scores)):
        s = max_priority * scores[i] // max_count
        if reverse:
            s = max_priority - s
        scores[i] = s


def py_inloop(counts):
    # minisched.go:164-185 for one plugin with ScoreExtensions: the list starts as zeros
    lst = [0] * len(counts)
    for k, c in enumerate(counts):
        lst[k] = c
        py_default_normalize(lst, 100, reverse=True)
    return lst


def test_inloop_known_answers(oracle):
    # one node: raw 0 -> maxCount 0 -> 100; raw 2 -> 100 - 100 = 0
    assert list(oracle.tt_inloop([0])) == [100]
    assert list(oracle.tt_inloop([2])) == [0]
    # [1, 0]: step 0 -> [0, 100] (the unscored entry is normalised too), step 1
    # writes 0 -> [0, 0] -> maxCount 0 -> [100, 100]; a two-pass normalise of the
    # final raw list would give [0, 100]: the in-loop quirk changes the winner set
    assert list(oracle.tt_inloop([1, 0])) == [100, 100]
    two_pass = [1, 0]
    py_default_normalize(two_pass, 100, reverse=True)
    assert two_pass == [0, 100]
    # [0, 1]: step 0 -> [100, 100], step 1 -> [100, 1] -> max 100 -> [0, 99]
    assert list(oracle.tt_inloop([0, 1])) == [0, 99]
    # long lists settle into a flip per step: the parity of the distance to the
    # end decides between c and 100 - c
    got = list(oracle.tt_inloop([0, 0, 0, 0, 0, 3, 0, 3, 0]))
    assert got == py_inloop([0, 0, 0, 0, 0, 3, 0, 3, 0])


@pytest.mark.parametrize("seed", range(6))
def test_inloop_closed_form_matches_the_loop(oracle, seed):
    rng = np.random.default_rng(seed)
    for _ in range(400):
        F = int(rng.integers(1, 90))
        p = rng.random()
        c = np.where(rng.random(F) < p, rng.integers(1, 9, F), 0)
        lit = oracle.tt_inloop(c, literal=True)
        closed = oracle.tt_inloop(c, literal=False)
        assert np.array_equal(lit, closed), c.tolist()
        if F <= 30:
            assert lit.tolist() == py_inloop(c.tolist())


def test_inloop_rejects_counts_outside_the_universe(oracle):
    L = oracle.lib()
    c = np.array([0, 9], dtype=np.int64)
    out = np.zeros(2, dtype=np.int64)
    assert L.msor_tt_inloop(oracle._p(c), 2, 0, oracle._p(out)) == -1


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_schedule_tt_literal_equals_closed(oracle, seed):
    nr = synth.nodes(700, seed=seed, taints=True)
    pr = synth.pods(900, seed=seed, taints=True)
    pr["name_digit"][::17] = -1
    nr["allowed_pods"][::29] = -1  # tombstones: not in the LIST
    lit = oracle.schedule_tt(nr, pr, literal=True, seed=seed)
    closed = oracle.schedule_tt(nr, pr, literal=False, seed=seed)
    for k in ("node", "code", "score", "mask", "key"):
        assert np.array_equal(lit[k], closed[k]), k
    assert (lit["code"] == 0).sum() > 0.8 * len(pr)


def test_schedule_tt_filters_and_fit_error_mask(oracle):
    # node 0 unschedulable, node 1 with an untolerated NoSchedule taint, node 2 absent
    nr = np.zeros(3, dtype=_lib.NODE_REC)
    nr["unschedulable"] = [1, 0, 0]
    nr["name_digit"] = [0, 1, 2]
    nr["allowed_pods"] = [110, 110, -1]
    nr["taints"] = [0, 0x1, 0]
    pr = np.zeros(3, dtype=_lib.POD_REC)
    pr["ordinal"] = [0, 1, 2]
    pr["name_digit"] = [1, 1, 1]
    synth.set_tolerations(pr, [0, 0x1, 0x1], [0, 0, 0])
    pr["tolerates_unschedulable"] = [0, 0, 1]
    o = oracle.schedule_tt(nr, pr, seed=1)
    # pod 0: NU rejects node 0, TT rejects node 1 -> FitError {NU, TT}
    assert (o["code"][0], o["mask"][0]) == (2, _lib.MASK_NODE_UNSCHEDULABLE | _lib.MASK_TAINT_TOLERATION)
    # pod 1 tolerates taint 0: node 1 feasible alone -> NN 10 + TT (raw 0 -> 100)
    assert (o["code"][1], o["node"][1], o["score"][1]) == (0, 1, 110)
    # pod 2 tolerates both: nodes 0 and 1 feasible, raw [0, 0] -> [100, 100]; NN picks node 1
    assert (o["code"][2], o["node"][2], o["score"][2]) == (0, 1, 110)
    # an empty LIST: FitError with no plugin
    nr["allowed_pods"] = -1
    o = oracle.schedule_tt(nr, pr, seed=1)
    assert (o["code"] == 2).all() and (o["mask"] == 0).all()


def test_schedule_tt_soft_taints_score_reverse(oracle):
    # two feasible nodes of the pod's digit: raw counts [1, 0] end at [100, 100] (the
    # quirk) -> a tie broken by the hash; counts [0, 1] end at [0, 99] -> node 1 wins
    nr = np.zeros(2, dtype=_lib.NODE_REC)
    nr["name_digit"] = [3, 3]
    nr["allowed_pods"] = 110
    pr = np.zeros(1, dtype=_lib.POD_REC)
    pr["name_digit"] = 3
    nr["taints"] = [0, 1 << 8]
    o = oracle.schedule_tt(nr, pr, seed=7)
    assert (o["node"][0], o["score"][0]) == (1, 10 + 99)
    nr["taints"] = [1 << 8, 0]
    o = oracle.schedule_tt(nr, pr, seed=7)
    assert o["score"][0] == 110
    h = [oracle.lib().msor_h32(7, 0, i) for i in range(2)]
    assert o["node"][0] == int(np.argmax(h))
