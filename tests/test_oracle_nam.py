"""NodeAffinity with several preferred terms (plugin set MS_PLUGINS_NU_NN_NAM,
VERDICT r4 item 7) — the oracle on the CPU.

Upstream NodeAffinity.Score sums the weights of the pod's matching
PreferredSchedulingTerms, so with several terms a raw score reaches 400. Its
ScoreExtensions is DefaultNormalizeScore(MaxNodeScore, reverse=false), which
RunScorePlugins (/root/reference/minisched/minisched.go:164-185) calls on the
WHOLE, partially filled list after every node (k8s@v1.22.0
plugins/nodeaffinity/node_affinity.go, helper/normalize_score.go; not in the
container, restated). The oracle runs that loop literally (O(F^2) per pod) and
as a closed form (the composition of the later rescales applied to each
entry's starting value); this file checks both against each other and against
a transcription of the loop in Python, and pins hand-derived known answers.
"""
import numpy as np
import pytest

from minisched_amd import _lib, synth


def py_default_normalize(scores, max_priority=100):
    # helper.DefaultNormalizeScore(reverse=false), transcribed
    max_count = max(scores) if scores else 0
    if max_count == 0:
        return
    for i in range(len(scores)):
        scores[i] = max_priority * scores[i] // max_count


def py_inloop(raw):
    lst = [0] * len(raw)  # createPluginToNodeScores (minisched.go:327-334)
    for k, r in enumerate(raw):
        lst[k] = int(r)
        py_default_normalize(lst)
    return lst


@pytest.mark.parametrize(
    "raw,final",
    [
        ([70], [100]),                          # the anchor ends at 100 whatever its raw score
        ([0, 0, 30], [0, 0, 100]),
        ([50, 150], [66, 100]),                 # 150 rescales the anchor: floor(100 * 100 / 150)
        ([120, 30], [100, 30]),                 # later entries <= 100: identity steps
        ([30, 120, 250], [33, 40, 100]),        # 100 -> 83 -> 33 and 100 -> 40
        ([100, 101, 101, 101], [97, 98, 99, 100]),
        ([0, 400, 0, 200], [0, 50, 0, 100]),
    ],
)
def test_inloop_known_answers(oracle, raw, final):
    assert py_inloop(raw) == final
    assert list(oracle.nam_inloop(raw, literal=True)) == final
    assert list(oracle.nam_inloop(raw, literal=False)) == final


def test_repeated_rescales_reach_zero(oracle):
    # every rescale by r > 100 maps 1..100 strictly below itself: after 100 of
    # them everything before is 0 (the bounded table of the device form)
    raw = [100] + [101] * 100
    got = oracle.nam_inloop(raw, literal=False)
    assert got[0] == 0 and list(got) == py_inloop(raw)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_closed_form_matches_the_loop(oracle, seed):
    rng = np.random.default_rng(seed)
    for _ in range(600):
        F = int(rng.integers(1, 60))
        raw = rng.integers(0, 401, F) * (rng.random(F) < rng.random())
        lit = oracle.nam_inloop(raw, literal=True)
        assert list(lit) == py_inloop(raw)
        assert np.array_equal(oracle.nam_inloop(raw, literal=False), lit)


def _cluster(n_nodes, n_pods, n_sets, seed):
    nr = synth.nodes(n_nodes, seed=seed, labels=True)
    pr = synth.pods(n_pods, seed=seed, term_sets=n_sets)
    return nr, pr, synth.nam_term_sets(n_sets, seed=seed)


@pytest.mark.parametrize("seed,weights", [(11, (1, 1)), (12, (3, 2)), (13, (1, 5))])
def test_schedule_nam_literal_equals_closed(oracle, seed, weights):
    nr, pr, ts = _cluster(400, 500, 24, seed)
    pr["name_digit"][::31] = -1
    pr["tolerates_unschedulable"][::7] = 1
    nr["allowed_pods"][::41] = -1  # tombstones
    lit = oracle.schedule_nam(nr, pr, ts, weights=weights, literal=True, seed=seed)
    clo = oracle.schedule_nam(nr, pr, ts, weights=weights, literal=False, seed=seed)
    for k in ("node", "code", "score", "mask"):
        assert np.array_equal(lit[k], clo[k]), k
    ok = lit["code"] == 0
    assert ok.sum() > 400 and (lit["code"] == 1).sum() > 0
    # raw scores above 100 really occur (several matching terms)
    assert (lit["score"][ok] > 10 * weights[0] + 0).any()


def test_terms_match_keys_values_and_exists(oracle):
    # one node per label combination; pod with {zone == 3 (w 60), label2 Exists (w 50)}
    nr = np.zeros(4, dtype=_lib.NODE_REC)
    nr["allowed_pods"] = 110
    nr["name_digit"] = [1, 2, 3, 4]
    nr["zone"] = [3, 3, 5, 0]
    nr["label2"] = [0, 2, 2, 0]
    ts = _lib.nam_term_sets_array([[(0, 3, 60), (1, 0xFF, 50)]])
    pr = np.zeros(1, dtype=_lib.POD_REC)
    pr["name_digit"] = 9
    pr["pref_zone"] = 1  # term set 1
    # raw [60, 110, 50, 0]: step0 -> 100, step1 110 > 100 rescales: 100 -> 90, node1 100,
    # node2 50 -> identity: final [90, 100, 50, 0]; node1 wins
    lit = oracle.schedule_nam(nr, pr, ts, literal=True, seed=1)
    assert (lit["code"][0], lit["node"][0], lit["score"][0]) == (0, 1, 100)
    assert list(oracle.nam_inloop([60, 110, 50, 0])) == [90, 100, 50, 0]
    # weights 0 and unused slots never count; set id 0 = no terms
    pr["pref_zone"] = 0
    o = oracle.schedule_nam(nr, pr, ts, literal=True, seed=1)
    assert o["score"][0] == 0


def test_set_id_beyond_the_table_counts_as_no_terms(oracle):
    # minisched_gpu.h ms_nam_term_sets: "ids above n_sets count as no terms" (the device's rule)
    nr, pr, ts = _cluster(20, 5, 2, 3)
    pr["pref_zone"][0] = 7
    a = oracle.schedule_nam(nr, pr, ts)
    pr["pref_zone"][0] = 0
    b = oracle.schedule_nam(nr, pr, ts)
    for k in ("node", "code", "score", "mask"):
        assert np.array_equal(a[k], b[k])


def test_term_set_encoder_validates():
    with pytest.raises(ValueError):
        _lib.nam_term_sets_array([[(2, 1, 10)]])
    with pytest.raises(ValueError):
        _lib.nam_term_sets_array([[(0, 1, 101)]])
    with pytest.raises(ValueError):
        _lib.nam_term_sets_array([[(0, 1, 10)] * 5])
    a = _lib.nam_term_sets_array([[(1, 0xFF, 7), (0, 4, 100)]])
    assert a.shape == (1, 16) and list(a[0, :8]) == [1, 0xFF, 7, 0, 0, 4, 100, 0]


def test_zone_ids_stop_at_254():
    # 0xFF is the Exists marker of a multi-term set, so the shared value-id table never
    # hands it to a label value (an In term could not name it)
    from minisched_amd import encode

    z = encode.ZoneIds()
    ids = [z(f"v{i}") for i in range(254)]
    assert ids == list(range(1, 255)) and z("v0") == 1 and z(None) == 0
    with pytest.raises(ValueError):
        z("one-too-many")
