"""Bit-exact parity of the HIP path (through the C ABI) with the CPU oracle.

Every comparison is on the same seeded inputs: (node, code, score, mask) per
pod must be identical, and after sequential/bind work the node table read
back from the device must equal the oracle's columns.
"""
import numpy as np
import pytest

from minisched_amd import _lib, synth
from minisched_amd._lib import (
    MODE_BATCHED,
    MODE_SEQUENTIAL,
    PLUGINS_NU_NN,
    PLUGINS_NU_NRF_NN_LA,
    Engine,
)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    _lib.load()
    if _lib.device_count() == 0:
        pytest.fail("gpu test collected on a host without a visible device")


def engine_with(node_recs, plugin_set=PLUGINS_NU_NN, seed=1, node_base=0, cap=None, max_batch=1 << 16):
    e = Engine(max_nodes=cap or max(1, len(node_recs)), plugin_set=plugin_set, node_base=node_base, seed=seed,
               max_batch=max_batch)
    if len(node_recs):
        e.upsert(np.arange(node_base, node_base + len(node_recs)), node_recs)
    return e


def assert_same(res, o, idx=None):
    sel = slice(None) if idx is None else idx
    for k_res, k_or in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
        a = res[k_res][sel]
        b = o[k_or][sel]
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0][:10]
            raise AssertionError(f"{k_res} differs at {bad.tolist()}: gpu {a[bad].tolist()} oracle {b[bad].tolist()}")


def assert_table_equal(e, cols, n, base=0):
    t = e.read(base, n)
    for k_dev, k_or in (
        ("pod_count", "pod_count"),
        ("req_milli_cpu", "req_cpu"),
        ("req_memory", "req_mem"),
        ("nonzero_milli_cpu", "nz_cpu"),
        ("nonzero_memory", "nz_mem"),
    ):
        assert np.array_equal(t[k_dev], getattr(cols, k_or)), k_dev


def test_readme_scenario_gpu(oracle):
    first, node10, pod1 = synth.readme_scenario()
    with Engine(max_nodes=16) as e:
        e.upsert(np.arange(9), first)
        r = e.schedule(pod1, MODE_SEQUENTIAL)
        assert (r["code"][0], r["plugin_mask"][0], r["node"][0]) == (2, 1, -1)
        e.upsert(np.array([9]), node10)  # informer Add of node10
        r = e.schedule(pod1, MODE_SEQUENTIAL)
        assert (r["code"][0], r["node"][0], r["score"][0], r["plugin_mask"][0]) == (0, 9, 0, 0)
        assert e.read(9, 1)["pod_count"][0] == 1  # assume-on-select


@pytest.fixture(params=["pp", "v7", "v7w2", "v7w4", "v7w4-gen", "v8", "v0"])
def k1_variant(request, monkeypatch):
    # every NU+NN sweep form stays bit-exact: pp (the per-pair bit-sliced production kernel),
    # the class-indexed v7 with 1, 2 or 4 waves per workgroup sharing one tile build (and with
    # tolerating pods on the general path: -gen), the persistent v8, and v0 (hash every pair),
    # the plain cross-check
    v = request.param
    monkeypatch.setenv("MINISCHED_K1", v[:2])
    monkeypatch.setenv("MINISCHED_K1_WAVES", v[3] if "w" in v else "1")
    monkeypatch.setenv("MINISCHED_K1_TOL", "0" if v.endswith("-gen") else "1")
    return v


@pytest.mark.parametrize("n_nodes", [1, 15, 16, 17, 1000, 2047, 2048, 2049, 4096, 8193, 12345])
@pytest.mark.parametrize("n_pods", [1, 63, 64, 65, 700])
def test_nunn_random_sizes(oracle, k1_variant, n_nodes, n_pods):
    seed = 1000 + n_nodes * 7 + n_pods
    nr = synth.nodes(n_nodes, seed=seed)
    pr = synth.pods(n_pods, seed=seed)
    pr["tolerates_unschedulable"][::5] = 1
    pr["name_digit"][::11] = -1  # non-digit pod names -> Error when F > 0
    nr["name_digit"][::7] = 0xFF  # non-digit node names
    o = oracle.schedule(nr, pr, seed=seed)
    with engine_with(nr, seed=seed) as e:
        assert_same(e.schedule(pr, MODE_BATCHED), o)


@pytest.mark.parametrize("rpl", [None, "1", "7", "20", "21", "28", "29", "30", "31", "32"])
@pytest.mark.parametrize("n_nodes,node_base", [(12_500, 37_500), (25_000, 0), (3001, 99_000)])
def test_nunn_rows_per_lane(oracle, monkeypatch, k1_variant, rpl, n_nodes, node_base):
    # K1's row geometry (rows per lane, balanced waves over a shard, byte/dword/vector
    # tile loads) and the global-ordinal arithmetic of a shard that starts at node_base
    if rpl is not None:
        monkeypatch.setenv("MINISCHED_K1_RPL", rpl)
    seed = 77 + n_nodes
    nr = synth.nodes(n_nodes, seed=seed, start=node_base)
    pr = synth.pods(1000, seed=seed)
    pr["tolerates_unschedulable"][::9] = 1
    nr["name_digit"][::13] = 0xFF
    o = oracle.schedule(nr, pr, seed=seed, node_base=node_base)
    with engine_with(nr, seed=seed, node_base=node_base) as e:
        assert_same(e.schedule(pr, MODE_BATCHED), o)


@pytest.mark.parametrize("n_nodes,node_base", [(100_000, 0), (76_800, 12_345), (50_000, 50_000)])
def test_nunn_default_kernel_large_shards(oracle, monkeypatch, n_nodes, node_base):
    # the default K1 choice (persistent v8 from 40 node columns up, v7 below) at shard sizes
    # on both sides of the switch
    monkeypatch.delenv("MINISCHED_K1", raising=False)
    seed = 5 + n_nodes
    nr = synth.nodes(n_nodes, seed=seed, start=node_base)
    pr = synth.pods(2000, seed=seed)
    pr["tolerates_unschedulable"][::7] = 1
    pr["name_digit"][::97] = -1
    o = oracle.schedule(nr, pr, seed=seed, node_base=node_base)
    with engine_with(nr, seed=seed, node_base=node_base) as e:
        assert_same(e.schedule(pr, MODE_BATCHED), o)


@pytest.mark.parametrize("layout", ["runs", "skewed", "single"])
def test_nunn_uneven_digits(oracle, layout):
    # K1 v7 keeps at most K rows per (lane, digit) in its class lists; clusters whose
    # name digits do not cycle overflow them and take the general path for that class
    # (runs of equal digits, a skewed digit mix, every name ending in the same digit)
    n_nodes = 9000
    seed = {"runs": 11, "skewed": 12, "single": 13}[layout]
    rng = np.random.default_rng(seed)
    nr = synth.nodes(n_nodes, seed=seed)
    if layout == "runs":
        nr["name_digit"] = (np.arange(n_nodes) // 37) % 10
    elif layout == "skewed":
        nr["name_digit"] = np.where(rng.random(n_nodes) < 0.6, 3, rng.integers(0, 10, n_nodes))
    else:
        nr["name_digit"] = 7
    pr = synth.pods(777, seed=seed)
    pr["tolerates_unschedulable"][::6] = 1
    o = oracle.schedule(nr, pr, seed=seed)
    with engine_with(nr, seed=seed) as e:
        assert_same(e.schedule(pr, MODE_BATCHED), o)


def test_nunn_edge_cases(oracle, k1_variant):
    pr = synth.pods(130, seed=4)
    # empty table: FitError with an empty mask
    with Engine(max_nodes=64) as e:
        r = e.schedule(pr)
        assert np.all(r["code"] == 2) and np.all(r["plugin_mask"] == 0)
    # every node unschedulable: FitError{NU} unless the pod tolerates
    nr = synth.nodes(300, seed=4)
    nr["unschedulable"] = 1
    o = oracle.schedule(nr, pr, seed=4)
    with engine_with(nr, seed=4) as e:
        assert_same(e.schedule(pr), o)
    # tombstones: deleted nodes vanish from the LIST
    nr = synth.nodes(5000, seed=5)
    with engine_with(nr, seed=5) as e:
        dead = np.arange(0, 5000, 3)
        e.delete(dead)
        keep = nr.copy()
        keep["allowed_pods"][dead] = -1  # oracle: absent
        o = oracle.schedule(keep, pr, seed=5)
        assert_same(e.schedule(pr), o)
        # re-adding restores them, updates overwrite
        nr2 = nr.copy()
        nr2["unschedulable"] = 1 - nr2["unschedulable"]
        e.upsert(np.arange(5000), nr2)
        assert_same(e.schedule(pr), oracle.schedule(nr2, pr, seed=5))
        assert e.info().present_nodes == 5000


def test_config_b_exact_sequential(oracle, k1_variant):
    # BASELINE config B: 5k nodes x 10k pods, NU+NN, exact sequential
    nr = synth.nodes(5000, seed=1)
    pr = synth.pods(10000, seed=1)
    o = oracle.schedule(nr, pr, mode=1, seed=1)
    with engine_with(nr, seed=1) as e:
        res = e.schedule(pr, MODE_SEQUENTIAL)
        assert_same(res, o)
        assert_table_equal(e, o["cols"], 5000)


def test_config_c_shape_prefix(oracle, k1_variant):
    # config C nodes (100k) against a 1k-pod prefix, plus a 20k-pod run
    # checked on a strided sample
    nr = synth.nodes(100_000, seed=1)
    pr = synth.pods(20_000, seed=1)
    with engine_with(nr, seed=1) as e:
        res = e.schedule(pr)
    sample = np.arange(0, 20_000, 20)
    o = oracle.schedule_nunn_omp(nr, pr[sample], seed=1)
    assert_same(res[sample], o)


def test_node_sharded_combine_equals_single(oracle):
    # two contexts own disjoint ordinal ranges (what each rank of bench.py does);
    # the element-wise max of their keys decodes to the single-context result
    import torch

    n, p = 20_000, 3000
    nr = synth.nodes(n, seed=8)
    pr = synth.pods(p, seed=8)
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(device=dev)  # all work ordered on one real stream
    sp = stream.cuda_stream
    engines = []
    with torch.cuda.stream(stream):
        pods_d = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
        keys = []
        cuts = [0, 7777, n]
        for a, b in zip(cuts[:-1], cuts[1:]):
            e = engine_with(nr[a:b], seed=8, node_base=a)
            engines.append(e)
            k = torch.empty(p, dtype=torch.int64, device=dev)
            e.sweep_device(p, pods_d.data_ptr(), k.data_ptr(), 0, sp)
            keys.append(k)
        comb = torch.maximum(keys[0], keys[1])
        res_d = torch.empty(p * 24, dtype=torch.uint8, device=dev)
        engines[0].decode_device(p, pods_d.data_ptr(), comb.data_ptr(), 0, n, res_d.data_ptr(), sp)
    stream.synchronize()
    res = res_d.cpu().numpy().view(_lib.RESULT)
    o = oracle.schedule(nr, pr, seed=8)
    assert_same(res, o)
    assert np.array_equal(comb.cpu().numpy().view(np.uint64), o["key"])
    for e in engines:
        e.close()


@pytest.mark.parametrize("n_nodes,n_pods", [(37, 50), (1000, 700), (3000, 2500)])
def test_resource_batched(oracle, n_nodes, n_pods):
    seed = n_nodes + n_pods
    nr = synth.nodes(n_nodes, seed=seed, resources=True)
    pr = synth.pods(n_pods, seed=seed, resources=True)
    # pre-load some nodes so filters bite
    nr["req_milli_cpu"] = nr["alloc_milli_cpu"] // 2
    nr["nonzero_milli_cpu"] = nr["req_milli_cpu"]
    nr["pod_count"][::9] = 110
    nr["alloc_memory"][::13] = 0
    o = oracle.schedule_batched_commit(nr, pr, 1, seed=seed)
    with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=seed) as e:
        assert_same(e.schedule(pr, MODE_BATCHED), o)
        assert_table_equal(e, o["cols"], n_nodes)


@pytest.mark.parametrize("n_nodes,n_pods", [(1, 5), (50, 400), (700, 5000), (3000, 12000)])
def test_resource_exact_sequential(oracle, n_nodes, n_pods):
    seed = 3 * n_nodes + n_pods
    nr = synth.nodes(n_nodes, seed=seed, resources=True)
    pr = synth.pods(n_pods, seed=seed, resources=True)
    pr["name_digit"][::29] = -1
    o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=seed)
    assert (o["code"] == 2).sum() > 0 or n_pods < 1000  # saturation reached in the big cases
    with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=seed) as e:
        res = e.schedule(pr, MODE_SEQUENTIAL)
        assert_same(res, o)
        assert_table_equal(e, o["cols"], n_nodes)
        assert e.info()._pad == 0  # validator capacity / hand-off flags


def test_config_e_prefix(oracle):
    # config E shape (50k nodes) with the first 20k pods of the queue: exact
    nr = synth.nodes(50_000, seed=1, resources=True)
    pr = synth.pods(20_000, seed=1, resources=True)
    o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=1)
    with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=1) as e:
        assert_same(e.schedule(pr, MODE_SEQUENTIAL), o)
        assert_table_equal(e, o["cols"], 50_000)
        assert e.info()._pad == 0


def test_commit_uncommit(oracle):
    nr = synth.nodes(10, seed=2, resources=True)
    pr = synth.pods(1, seed=2, resources=True)
    with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=2) as e:
        e.commit_bind(4, pr[0])
        t = e.read(4, 1)
        assert t["pod_count"][0] == 1 and t["req_milli_cpu"][0] == pr["req_milli_cpu"][0]
        e.uncommit_bind(4, pr[0])
        t = e.read(4, 1)
        assert t["pod_count"][0] == 0 and t["req_milli_cpu"][0] == 0
        with pytest.raises(_lib.MSError):
            e.commit_bind(99, pr[0])


def test_chunked_batches(oracle):
    # more pods than max_batch: internal chunks must preserve queue order
    nr = synth.nodes(2000, seed=6, resources=True)
    pr = synth.pods(3000, seed=6, resources=True)
    o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=6)
    with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=6, max_batch=700) as e:
        assert_same(e.schedule(pr, MODE_SEQUENTIAL), o)


@pytest.mark.parametrize("pipe", ["1", "0"])
@pytest.mark.parametrize("batch", ["1", "7", "64", "256"])
def test_resource_sequential_batch_sizes(oracle, monkeypatch, batch, pipe):
    # speculative batch boundaries must not change placements: 50 nodes (one
    # tile, heavy re-sweeps) and 2500 nodes (lists rarely exhausted); with and
    # without the next batch's speculation overlapping validation
    monkeypatch.setenv("MINISCHED_SEQ_BATCH", batch)
    monkeypatch.setenv("MINISCHED_SEQ_PIPE", pipe)
    for n_nodes, n_pods in ((50, 600), (2500, 3000)):
        seed = 11 * n_nodes + int(batch)
        nr = synth.nodes(n_nodes, seed=seed, resources=True)
        pr = synth.pods(n_pods, seed=seed, resources=True)
        o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=seed)
        with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=seed) as e:
            assert_same(e.schedule(pr, MODE_SEQUENTIAL), o)
            assert_table_equal(e, o["cols"], n_nodes)
            assert e.info()._pad == 0


@pytest.mark.parametrize("n_nodes", [20_000, 100_000, 140_000])
def test_resource_sequential_tile_counts(oracle, n_nodes):
    # validator register layouts for 79, 391 and 547 tiles (2, 8 and 16 lists per lane)
    nr = synth.nodes(n_nodes, seed=5, resources=True)
    pr = synth.pods(1500, seed=5, resources=True)
    o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=5)
    with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=5) as e:
        assert_same(e.schedule(pr, MODE_SEQUENTIAL), o)
        assert_table_equal(e, o["cols"], n_nodes)
