"""The TaintToleration shard protocol on the CPU: per-segment summaries, their
associative merge and the closed-form finalisation (csrc/ms_taint.hip
k_tt_sweep / tt_merge / tt_finalize), restated in Python and checked against
the oracle's literal in-loop normalisation over random row segmentations —
the property the GPU's row segments and node shards rely on (any split of the
LIST into consecutive pieces gives the same placements).
Reference: /root/reference/minisched/minisched.go:164-185 (the in-loop hook),
:304-325 (selectHost).
"""
import numpy as np
import pytest

from minisched_amd import synth


def tmap(m, v):
    return 100 if m == 0 else 100 - (100 * v) // m


def summarise(entries):
    """entries: [(c, key)] of one segment's feasible nodes in LIST order -> summary."""
    n = len(entries)
    s = {"n": n, "first": entries[:3], "last": entries[-1] if n else None, "cls": {}}
    for j in range(3, n - 1):
        c, key = entries[j]
        k = (c, j & 1)
        s["cls"][k] = max(s["cls"].get(k, key), key)
    return s


def merge(a, b):
    r = {"n": a["n"] + b["n"], "first": list(a["first"]), "last": a["last"], "cls": dict(a["cls"])}
    for (c, q), key in b["cls"].items():
        k = (c, q ^ (a["n"] & 1))
        r["cls"][k] = max(r["cls"].get(k, key), key)

    def place(e, g):
        if g < 3:
            r["first"].append(e)
        if g + 1 == r["n"]:
            r["last"] = e
        if 3 <= g < r["n"] - 1:
            k = (e[0], g & 1)
            r["cls"][k] = max(r["cls"].get(k, e[1]), e[1])

    if a["n"] > 3:
        place(a["last"], a["n"] - 1)
    for i, e in enumerate(b["first"]):
        place(e, a["n"] + i)
    if b["n"] > 3:
        place(b["last"], a["n"] + b["n"] - 1)
    return r


def finalize(s):
    """Max over candidates of (10 * match + final TT score, hash): the winning key."""
    F = s["n"]
    cands = []
    if F <= 4:
        es = s["first"] + ([s["last"]] if F == 4 else [])
        vals = [0] * F
        for k in range(F):
            vals[k] = es[k][0]
            m = max(vals)
            vals = [tmap(m, v) for v in vals]
        cands = [(es[k][1], vals[k]) for k in range(F)]
    else:
        sv, u = [], 0
        for k in range(3):
            sv.append(s["first"][k][0])
            m = max(sv + [u])
            sv = [tmap(m, v) for v in sv]
            u = tmap(m, u)
        p = [100 - v if (F - 4) & 1 else v for v in sv]
        pc = {k: (100 - k[0] if k[1] == (F & 1) else k[0]) for k in s["cls"]}
        m_last = max(p + list(pc.values()) + [s["last"][0]])
        cands = [(s["first"][k][1], tmap(m_last, p[k])) for k in range(3)]
        cands.append((s["last"][1], tmap(m_last, s["last"][0])))
        cands += [(key, tmap(m_last, pc[k])) for k, key in s["cls"].items()]
    # key = (match, hash): total = 10 * match + v, ties by hash
    return max(((10 * key[0] + v, key[1]) for key, v in cands), default=None)


@pytest.mark.parametrize("seed", range(4))
def test_segment_merge_equals_the_literal_loop(oracle, seed):
    rng = np.random.default_rng(seed)
    for _ in range(300):
        F = int(rng.integers(0, 40))
        c = np.where(rng.random(F) < rng.random(), rng.integers(1, 9, F), 0)
        match = rng.integers(0, 2, F)
        h = rng.permutation(1 << 16)[:F]  # distinct hashes, as the bijective tie-break hash gives
        entries = [(int(c[i]), (int(match[i]), int(h[i]))) for i in range(F)]
        want = None
        if F:
            tt = oracle.tt_inloop(c, literal=True)
            want = max((10 * int(match[i]) + int(tt[i]), int(h[i])) for i in range(F))
        # a random split of the LIST into consecutive segments, merged left to right
        cuts = sorted(set(rng.integers(0, F + 1, int(rng.integers(0, 6))).tolist()) | {0, F})
        segs = [summarise(entries[a:b]) for a, b in zip(cuts[:-1], cuts[1:])] or [summarise([])]
        acc = segs[0]
        for sg in segs[1:]:
            acc = merge(acc, sg)
        assert acc["n"] == F
        assert finalize(acc) == want, (c.tolist(), cuts)


def test_merge_is_associative_on_a_cluster(oracle):
    # three-way splits of one synthetic pod's feasible list merged as (a.b).c and a.(b.c)
    nr = synth.nodes(400, seed=3, taints=True)
    pr = synth.pods(1, seed=3, taints=True)
    soft = (nr["taints"] >> 8) & 0xFF
    c = np.array([bin(int(x) & ~int(pr["pref_weight"][0])).count("1") for x in soft])
    entries = [(int(c[i]), (i % 2, (i * 7919) % 65536)) for i in range(len(c))]
    for cut in [(0, 1, 2, 400), (0, 3, 7, 400), (0, 200, 396, 400), (0, 5, 6, 400)]:
        a, b, d = (summarise(entries[x:y]) for x, y in zip(cut[:-1], cut[1:]))
        assert finalize(merge(merge(a, b), d)) == finalize(merge(a, merge(b, d))) == finalize(summarise(entries))
