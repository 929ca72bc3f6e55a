"""MS_PLUGINS_NU_TT_NN on the GPU: TaintToleration's filter
and its score with the in-loop reverse DefaultNormalizeScore, against the
oracle's literal O(F^2) loop (small clusters) and its closed form (larger
ones, the closed form itself checked against the loop in
tests/test_oracle_tt.py), on one context (every host and device entry point)
and over node shards (ms_tt_summaries_device / ms_tt_decode_device).
Reference: /root/reference/minisched/minisched.go:115-151 (filters, first
failure), :164-185 (the in-loop hook), :304-325 (selectHost).
"""
import numpy as np
import pytest

from minisched_amd import _lib, sharded, synth

pytestmark = pytest.mark.gpu

TT = _lib.PLUGINS_NU_TT_NN


def _same(res, o, tag, a=0, b=None):
    b = len(o["node"]) if b is None else b
    for k_res, k_or in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
        got, want = np.asarray(res[k_res]).astype(np.int64), np.asarray(o[k_or][a:b]).astype(np.int64)
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0][:8]
            raise AssertionError(f"{tag} {k_res} differs at {(bad + a).tolist()}: gpu {got[bad].tolist()} "
                                 f"oracle {want[bad].tolist()}")


def _cluster(n_nodes, n_pods, seed, dead_every=0):
    nr = synth.nodes(n_nodes, seed=seed, taints=True)
    pr = synth.pods(n_pods, seed=seed, taints=True)
    pr["name_digit"][::19] = -1
    pr["tolerates_unschedulable"][::7] = 1
    dead = np.arange(0, n_nodes, dead_every) if dead_every else np.arange(0)
    return nr, pr, dead


def _oracle(oracle, nr, pr, seed, dead=(), literal=False):
    nr = nr.copy()
    if len(dead):
        nr["allowed_pods"][np.asarray(dead)] = -1
    return oracle.schedule_tt(nr, pr, literal=literal, seed=seed)


def _engine(nr, seed, lo=0, hi=None, dead=()):
    hi = len(nr) if hi is None else hi
    e = _lib.Engine(max_nodes=max(1, hi - lo), plugin_set=TT, node_base=lo, seed=seed)
    e.upsert(np.arange(lo, hi), nr[lo:hi])
    gone = np.asarray([d for d in dead if lo <= d < hi], dtype=np.uint32)
    if len(gone):
        e.delete(gone)
    e.flush()
    return e


def _device_cycle(e, pr):
    import torch

    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    out = torch.full((len(pr) * 24,), 0xCD, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # (the fill ran on torch's stream, not s)
    e.select_batch_device(len(pr), pods.data_ptr(), out.data_ptr(), s.cuda_stream)
    s.synchronize()
    return out.cpu().numpy().view(_lib.RESULT)


@pytest.mark.parametrize("n_nodes,n_pods,seed", [(1, 40, 1), (5, 200, 2), (300, 500, 3), (2100, 300, 4)])
def test_tt_against_literal_loop(oracle, n_nodes, n_pods, seed):
    # small clusters (F <= 4, the closed-form regime, two row segments) against the
    # loop exactly as RunScorePlugins runs it
    nr, pr, dead = _cluster(n_nodes, n_pods, seed, dead_every=11)
    o = _oracle(oracle, nr, pr, seed, dead, literal=True)
    with _engine(nr, seed, dead=dead) as e:
        _same(_device_cycle(e, pr), o, "device")
        _same(e.schedule(pr, _lib.MODE_BATCHED), o, "host")


@pytest.mark.parametrize("n_nodes,n_pods,seed", [(20_000, 3000, 5), (45_000, 1500, 6)])
def test_tt_many_segments(oracle, n_nodes, n_pods, seed):
    # 10 and 16 row segments per pod merged in LIST order, against the closed form
    nr, pr, dead = _cluster(n_nodes, n_pods, seed, dead_every=101)
    o = _oracle(oracle, nr, pr, seed, dead)
    with _engine(nr, seed, dead=dead) as e:
        _same(_device_cycle(e, pr), o, "device")
    assert (o["code"] == 0).sum() > 0.8 * n_pods


def test_tt_host_modes_compact_and_binds(oracle):
    # ms_schedule_batch batched / sequential (stateless set: equal, binds accumulate)
    # and compact records (the tolerated taint ids travel in the compact bytes)
    seed = 7
    nr, pr, _ = _cluster(3000, 2500, seed)
    o = _oracle(oracle, nr, pr, seed)
    with _engine(nr, seed) as e:
        _same(e.schedule(pr, _lib.MODE_BATCHED), o, "batched")
        _same(e.schedule(pr, _lib.MODE_SEQUENTIAL), o, "sequential")
        r = e.schedule_compact(_lib.compact_pods(pr))
        for k_res, k_or in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
            assert np.array_equal(r[k_res].astype(np.int64), o[k_or].astype(np.int64)), k_res
        placed = np.bincount(o["node"][o["code"] == 0], minlength=3000)
        assert np.array_equal(e.read(0, 3000)["pod_count"], 3 * placed)


def test_tt_fit_error_masks(oracle):
    # every node either unschedulable or carrying an untolerated NoSchedule taint; and
    # an empty LIST (no plugin rejected anything)
    seed = 8
    nr = synth.nodes(500, seed=seed, taints=True)
    nr["taints"] |= np.where(nr["unschedulable"] == 1, 0, 0x4).astype(np.uint32)
    pr = synth.pods(300, seed=seed, taints=True)
    synth.set_tolerations(pr, pr["pref_zone"] & 0x3, pr["pref_weight"])  # nobody tolerates taint id 2
    pr["tolerates_unschedulable"] = 0
    o = _oracle(oracle, nr, pr, seed)
    assert (o["code"] == 2).all()
    with _engine(nr, seed) as e:
        _same(e.schedule(pr), o, "all rejected")
    with _engine(nr, seed, dead=np.arange(500)) as e:
        r = e.schedule(pr)
        assert (r["code"] == 2).all() and (r["plugin_mask"] == 0).all()


@pytest.mark.parametrize("cuts", [(0, 5000, 10_000), (0, 37, 38, 4000, 9000), (0, 3, 6000)])
def test_tt_node_shards(oracle, cuts):
    # node shards (contexts with their own node_base): per-shard summaries, gathered
    # shard-major, merged and decoded on one of them; includes a shard of one node, a
    # shard whose nodes are all deleted, and shards of fewer than 4 feasible nodes
    import torch

    seed = 9 + len(cuts)
    n = cuts[-1]
    nr, pr, _ = _cluster(n, 2000, seed)
    dead = np.arange(cuts[1], cuts[2]) if len(cuts) > 3 else np.arange(0, n, 13)
    o = _oracle(oracle, nr, pr, seed, dead)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    G, P, SB = len(cuts) - 1, len(pr), _lib.TT_SUMMARY_BYTES
    summ = torch.zeros(G * P * SB, dtype=torch.uint8, device=dev)
    outs = [torch.zeros(P * 24, dtype=torch.uint8, device=dev) for _ in range(G)]
    torch.cuda.synchronize()  # (the fills ran on torch's stream, not s)
    engines = [_engine(nr, seed, lo, hi, dead) for lo, hi in zip(cuts[:-1], cuts[1:])]
    try:
        for g, e in enumerate(engines):
            e.tt_summaries_device(P, pods.data_ptr(), summ.data_ptr() + g * P * SB, s.cuda_stream)
        for g, e in enumerate(engines):  # every shard decodes the same merge
            out = outs[g]
            e.tt_decode_device(P, pods.data_ptr(), G, summ.data_ptr(), out.data_ptr(), s.cuda_stream)
            s.synchronize()
            _same(out.cpu().numpy().view(_lib.RESULT), o, f"shards {cuts} decoded on {g}")
        with pytest.raises(_lib.MSError):  # keys do not combine for this set
            kb = torch.zeros(P, dtype=torch.int64, device=dev)
            engines[0].sweep_device(P, pods.data_ptr(), kb.data_ptr(), 0, s.cuda_stream)
    finally:
        for e in engines:
            e.close()
    assert sharded.shard_bounds(n, 0, 1) == (0, n)


def _dense_cluster(n_nodes, n_pods, seed, hard_p=0.03, soft_p=0.35, tol_p=0.3):
    # every one of the 8 NoSchedule and 8 PreferNoSchedule ids in use, so raw
    # counts reach 8 (the bit-sliced census' c3 plane) and classes are sparse
    rng = np.random.default_rng(seed)
    nr = synth.nodes(n_nodes, seed=seed, taints=True)
    hard = (rng.random((n_nodes, 8)) < hard_p) @ (1 << np.arange(8))
    soft = (rng.random((n_nodes, 8)) < soft_p) @ (1 << np.arange(8))
    nr["taints"] = (hard | (soft << 8)).astype(np.uint32)
    nr["taints"][rng.random(n_nodes) < 0.01] |= 0xFF00  # some rows with all 8 soft ids
    pr = synth.pods(n_pods, seed=seed, taints=True)
    synth.set_tolerations(pr, (rng.random((n_pods, 8)) < tol_p) @ (1 << np.arange(8)),
                          (rng.random((n_pods, 8)) < tol_p) @ (1 << np.arange(8)))
    pr["name_digit"][::23] = -1
    pr["tolerates_unschedulable"][::5] = 1
    return nr, pr


@pytest.mark.parametrize("n_nodes,n_pods,seed", [(3, 300, 21), (7, 400, 22), (40, 600, 23), (700, 800, 24),
                                                 (2050, 500, 25)])
def test_tt_dense_taints_literal(oracle, n_nodes, n_pods, seed):
    # the two-pass census / pick: F <= 4, the first-three and last rows inside one
    # word and across words, classes present only without a NodeNumber match (W0)
    nr, pr = _dense_cluster(n_nodes, n_pods, seed)
    dead = np.arange(0, n_nodes, 9)
    o = _oracle(oracle, nr, pr, seed, dead, literal=True)
    with _engine(nr, seed, dead=dead) as e:
        _same(_device_cycle(e, pr), o, "device")
        _same(e.schedule(pr, _lib.MODE_BATCHED), o, "host")


@pytest.mark.parametrize("n_nodes,n_pods,seed", [(9000, 2000, 26), (33_000, 1200, 27)])
def test_tt_dense_taints_segments(oracle, n_nodes, n_pods, seed):
    # several row segments (census merge, global rank parity in the pick) against the
    # closed form; sparse digits make W0 (no matching row in the winning class) common
    nr, pr = _dense_cluster(n_nodes, n_pods, seed, hard_p=0.05, soft_p=0.45)
    rng = np.random.default_rng(seed)
    nr["name_digit"][rng.random(n_nodes) < 0.7] = 255  # most nodes without a digit name
    dead = np.arange(0, n_nodes, 31)
    o = _oracle(oracle, nr, pr, seed, dead)
    with _engine(nr, seed, dead=dead) as e:
        _same(_device_cycle(e, pr), o, "device")
    assert (o["code"] == 0).sum() > 0.5 * n_pods


@pytest.mark.parametrize("cuts,dense", [((0, 5000, 10_000), False), ((0, 37, 38, 4000, 9000), False),
                                        ((0, 3, 6000), False), ((0, 1100, 2600, 7000), True)])
def test_tt_node_shards_two_pass(oracle, cuts, dense):
    # the two-pass form over node shards: censuses gathered shard-major, each shard's
    # keys under the plan of all of them, uint64 MAX, the results on any shard; incl. a
    # one-node shard, an all-deleted shard, shards under 4 feasible nodes, and dense
    # 8 + 8-id taints (the literal loop checks the small one)
    import torch

    seed = 70 + len(cuts) + (5 if dense else 0)
    n = cuts[-1]
    if dense:
        nr, pr = _dense_cluster(n, 1500, seed, hard_p=0.05, soft_p=0.45)
        dead = np.arange(0, n, 17)
    else:
        nr, pr, _ = _cluster(n, 2000, seed)
        dead = np.arange(cuts[1], cuts[2]) if len(cuts) > 3 else np.arange(0, n, 13)
    o = _oracle(oracle, nr, pr, seed, dead)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    G, P, CB = len(cuts) - 1, len(pr), _lib.TT_CENSUS_BYTES
    census = torch.zeros(G * P * CB, dtype=torch.uint8, device=dev)
    keys = torch.zeros((G, P), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()  # (the fills ran on torch's stream, not s)
    engines = [_engine(nr, seed, lo, hi, dead) for lo, hi in zip(cuts[:-1], cuts[1:])]
    try:
        for g, e in enumerate(engines):
            e.tt_census_device(P, pods.data_ptr(), census.data_ptr() + g * P * CB, s.cuda_stream)
        for g, e in enumerate(engines):
            e.tt_pick_device(P, pods.data_ptr(), G, g, census.data_ptr(), keys[g].data_ptr(), s.cuda_stream)
        s.synchronize()
        best = keys.max(dim=0).values.contiguous()  # keys < 2^63: the signed max is the unsigned one
        torch.cuda.synchronize()
        for g, e in enumerate(engines):  # any shard decodes
            out = torch.full((P * 24,), 0xCD, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            e.tt_final_device(P, pods.data_ptr(), G, census.data_ptr(), best.data_ptr(), out.data_ptr(), s.cuda_stream)
            s.synchronize()
            _same(out.cpu().numpy().view(_lib.RESULT), o, f"two-pass shards {cuts} decoded on {g}")
    finally:
        for e in engines:
            e.close()
