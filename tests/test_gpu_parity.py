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


@pytest.mark.parametrize("n_nodes", [1, 15, 16, 17, 1000, 2047, 2048, 2049, 4096, 8193, 12345])
@pytest.mark.parametrize("n_pods", [1, 63, 64, 65, 700])
def test_nunn_random_sizes(oracle, n_nodes, n_pods):
    seed = 1000 + n_nodes * 7 + n_pods
    nr = synth.nodes(n_nodes, seed=seed)
    pr = synth.pods(n_pods, seed=seed)
    pr["tolerates_unschedulable"][::5] = 1
    pr["name_digit"][::11] = -1  # non-digit pod names -> Error when F > 0
    nr["name_digit"][::7] = 0xFF  # non-digit node names
    o = oracle.schedule(nr, pr, seed=seed)
    with engine_with(nr, seed=seed) as e:
        assert_same(e.schedule(pr, MODE_BATCHED), o)


@pytest.mark.parametrize("waves", [None, "1", "2", "4", "16"])
@pytest.mark.parametrize("n_nodes,node_base", [(12_500, 37_500), (25_000, 0), (3001, 99_000)])
def test_nunn_shard_geometry(oracle, monkeypatch, waves, n_nodes, node_base):
    # K1 pp's workgroup geometry (waves per workgroup holding a shard's groups, the
    # round-robin deal of groups over waves) and the global-ordinal arithmetic of a
    # shard that starts at node_base
    if waves is not None:
        monkeypatch.setenv("MINISCHED_PP_WAVES", waves)
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
    # K1 pp at shard sizes around one 16-wave workgroup's 122,880 rows and a shard
    # that starts at a non-zero ordinal
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
    # K1 pp's three fast slots cover at most 3 rows of one digit per 30-row group; clusters
    # whose name digits do not cycle set the group's "over" plane and take the bit-scan
    # path (runs of equal digits, a skewed digit mix, every name ending in the same digit)
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


def test_nunn_edge_cases(oracle):
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


@pytest.mark.parametrize("node_base", [0, 7, 33_333, 999_990])
@pytest.mark.parametrize("layout", ["aligned", "one_misaligned", "names", "sparse"])
def test_fixed_slot_form(oracle, node_base, layout):
    # K1's fixed-slot form (ms_sweep_pp.hip word_fix): waves whose groups are
    # digit-aligned (digit == ordinal mod 10 for every present digit-named row)
    # take three known slots per pod; a single misaligned group sends its wave
    # back to the slot search. Shard offsets not divisible by 10 move the slots
    # (node_base mod 10), non-digit node names and pods, unschedulable rows,
    # tolerations and tombstones keep their meaning; every layout equals the oracle.
    n = 40_000 if node_base < 999_000 else 1_000
    nr = synth.nodes(n, seed=11, start=node_base)
    pr = synth.pods(3001, seed=11)
    pr["name_digit"][::13] = -1
    pr["tolerates_unschedulable"][::5] = 1
    rng = np.random.default_rng(node_base + len(layout))
    if layout == "one_misaligned":
        nr["name_digit"][12_345 % n] = (nr["name_digit"][12_345 % n] + 1) % 10
    elif layout == "names":  # non-digit names stay aligned (they never match)
        nr["name_digit"][rng.integers(0, n, n // 7)] = 0xFF
    elif layout == "sparse":  # most rows deleted: groups with one or two present rows
        nr["allowed_pods"][rng.random(n) < 0.9] = -1
    o = oracle.schedule(nr, pr, seed=11, node_base=node_base)
    with engine_with(nr, seed=11, node_base=node_base) as e:
        if layout == "sparse":
            gone = np.flatnonzero(nr["allowed_pods"] < 0) + node_base
            e.delete(gone.astype(np.uint32))
        assert_same(e.schedule(pr, MODE_BATCHED), o)
    assert (o["code"] == 0).sum() > 0


@pytest.mark.parametrize("n_nodes,layout", [(7_711, "aligned"), (12_500, "aligned"), (15_360, "aligned"),
                                             (12_500, "misaligned"), (12_500, "overfull")])
def test_two_wave_shards(oracle, n_nodes, layout):
    # 257..512 row groups take 2-wave workgroups (ms_sweep_pp.hip geometry): the
    # G = 8 shard of config C (12,500 rows) and the bounds of the range, with the
    # fixed-slot form, the slot search (one misaligned row) and the bit-scan
    # loop (more than 3 rows of a digit in a group).
    nr = synth.nodes(n_nodes, seed=21, start=87_500)
    if layout == "misaligned":
        nr["name_digit"][6_001] = (nr["name_digit"][6_001] + 3) % 10
    elif layout == "overfull":
        nr["name_digit"][3_000:3_030] = 4
    pr = synth.pods(20_000, seed=21)
    pr["name_digit"][::11] = -1
    o = oracle.schedule(nr, pr, seed=21, node_base=87_500)
    with engine_with(nr, seed=21, node_base=87_500) as e:
        assert_same(e.schedule(pr, MODE_BATCHED), o)


def test_config_b_exact_sequential(oracle):
    # BASELINE config B: 5k nodes x 10k pods, NU+NN, exact sequential
    nr = synth.nodes(5000, seed=1)
    pr = synth.pods(10000, seed=1)
    o = oracle.schedule(nr, pr, mode=1, seed=1)
    with engine_with(nr, seed=1) as e:
        res = e.schedule(pr, MODE_SEQUENTIAL)
        assert_same(res, o)
        assert_table_equal(e, o["cols"], 5000)


def test_config_c_shape_prefix(oracle):
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
    k = comb.cpu().numpy().view(np.uint64)
    # no feasible node: key 1 (the shards list nodes), real keys equal the oracle's
    assert np.array_equal(np.where(k <= 1, 0, k), o["key"]) and np.array_equal(k == 1, o["key"] == 0)
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


@pytest.mark.parametrize("max_batch", [1 << 16, 8192])
def test_resource_batched_large_call(oracle, max_batch):
    # a MODE_BATCHED call of the resource-aware set decides every pod on
    # the same node state, whatever the call size: 40k pods used to be split into chunks
    # whose binds landed before the next chunk was swept (and max_batch chunks likewise)
    nr = synth.nodes(3000, seed=91, resources=True)
    pr = synth.pods(40_000, seed=91, resources=True)
    nr["req_milli_cpu"] = nr["alloc_milli_cpu"] // 3
    nr["nonzero_milli_cpu"] = nr["req_milli_cpu"]
    o = oracle.schedule_batched_commit(nr, pr, 1, seed=91)
    with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=91, max_batch=max_batch) as e:
        assert_same(e.schedule(pr, MODE_BATCHED), o)
        assert_table_equal(e, o["cols"], 3000)


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


@pytest.mark.parametrize("plugin_set", [PLUGINS_NU_NN, _lib.PLUGINS_NU_NN_NA])
@pytest.mark.parametrize("n_pods", [1, 777, 40_000])
def test_compact_records(oracle, plugin_set, n_pods):
    # ms_schedule_batch_compact: 8 B pods in, 8 B results out, the same outcomes and binds
    # (pod_count) as the full records
    seed = 300 + n_pods + plugin_set
    zones = plugin_set == _lib.PLUGINS_NU_NN_NA
    nr = synth.nodes(6000, seed=seed, zones=zones)
    pr = synth.pods(n_pods, seed=seed, zones=zones)
    pr["name_digit"][::13] = -1
    pr["tolerates_unschedulable"][::7] = 1
    o = oracle.schedule_na(nr, pr, seed=seed, literal=False) if zones else oracle.schedule(nr, pr, seed=seed)
    with engine_with(nr, plugin_set=plugin_set, seed=seed) as e:
        r = e.schedule_compact(_lib.compact_pods(pr))
        for k_res, k_or in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
            assert np.array_equal(r[k_res].astype(np.int64), o[k_or].astype(np.int64)), k_res
        placed = np.bincount(o["node"][o["code"] == 0], minlength=6000)
        assert np.array_equal(e.read(0, 6000)["pod_count"], placed)
    with engine_with(synth.nodes(10, seed=1, resources=True), plugin_set=PLUGINS_NU_NRF_NN_LA) as e:
        with pytest.raises(_lib.MSError):  # the resource-aware set needs the full records
            e.schedule_compact(_lib.compact_pods(pr[:3]))


def test_compact_repeated_calls(oracle):
    # successive compact calls on one context with different pods (the pinned staging is
    # reused, and regrown for a larger call): every call equals the oracle, binds accumulate
    nr = synth.nodes(7000, seed=41)
    total = np.zeros(7000, dtype=np.int64)
    with engine_with(nr, seed=41) as e:
        for k, n in enumerate((5000, 1200, 30_000, 3)):
            pr = synth.pods(n, seed=41, start=k * 100_000)
            pr["tolerates_unschedulable"][::9] = 1
            o = oracle.schedule(nr, pr, seed=41)
            r = e.schedule_compact(_lib.compact_pods(pr))
            for k_res, k_or in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
                assert np.array_equal(r[k_res].astype(np.int64), o[k_or].astype(np.int64)), (n, k_res)
            total += np.bincount(o["node"][o["code"] == 0], minlength=7000)
        assert np.array_equal(e.read(0, 7000)["pod_count"], total)


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


@pytest.mark.parametrize("max_batch", [8300, 8320, 8384])
def test_chunked_warm_runs(oracle, max_batch):
    # every chunk of a call is a sequential run that opens with warm-up batches of
    # 64 (its first 8,192 pods), so only pods 0..63 of a list set are rewritten
    # until its first full-size batch; cells left over from the previous chunk
    # must never pass for swept ones (the 2-bit list tag repeats every third
    # step: three chunk sizes, three tag phases), nor across two calls
    seed = max_batch
    nr = synth.nodes(3000, seed=seed, resources=True)
    pr = synth.pods(3 * max_batch + 77, seed=seed, resources=True)
    o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=seed)
    half = len(pr) // 2
    with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=seed, max_batch=max_batch) as e:
        a = e.schedule(pr[:half], MODE_SEQUENTIAL)
        b = e.schedule(pr[half:], MODE_SEQUENTIAL)
        assert_same(np.concatenate([a, b]), o)
        assert_table_equal(e, o["cols"], 3000)


@pytest.mark.parametrize("batch", ["1", "7", "64", "128", "256"])
def test_resource_sequential_batch_sizes(oracle, monkeypatch, batch):
    # speculative batch boundaries must not change placements: 50 nodes (one
    # tile, heavy re-sweeps) and 2500 nodes (lists rarely exhausted); single-stream
    # steps (validation k beside the sweep of k+1 and its in-step merge); 256 is
    # clamped to the validator's 128
    monkeypatch.setenv("MINISCHED_SEQ_BATCH", batch)
    for n_nodes, n_pods in ((50, 600), (2500, 3000)):
        seed = 11 * n_nodes + int(batch)
        nr = synth.nodes(n_nodes, seed=seed, resources=True)
        pr = synth.pods(n_pods, seed=seed, resources=True)
        o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=seed)
        with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=seed) as e:
            assert_same(e.schedule(pr, MODE_SEQUENTIAL), o)
            assert_table_equal(e, o["cols"], n_nodes)
            assert e.info()._pad == 0


@pytest.mark.parametrize("merge", ["launch", "fallback"])
@pytest.mark.parametrize("batch", ["1", "7", "64", "256"])
def test_resource_sequential_merge_forms(oracle, monkeypatch, batch, merge):
    # batch k+1's top-4 merge inside step k (the sweep workgroups merge once all
    # have written its tile lists), and the fallback where every in-step worker
    # skips and each validation merges its own batch first
    monkeypatch.setenv("MINISCHED_SEQ_BATCH", batch)
    monkeypatch.setenv("MINISCHED_SEQ_MERGE", merge)
    for n_nodes, n_pods in ((50, 600), (2500, 3000)):
        seed = 13 * n_nodes + int(batch)
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


@pytest.mark.parametrize("fast", ["1", "0"])
@pytest.mark.parametrize("n_nodes,n_pods", [(3000, 4000), (40_000, 1500)])
def test_resource_sequential_capacity_forms(oracle, monkeypatch, fast, n_nodes, n_pods):
    # the sweep's binary64 LeastAllocated form (exact for Allocatable < 2^41,
    # NonZeroRequested >= 0, pod requests < 2^53) beside tiles that must take the
    # general form: 5 TiB and 2^60 capacities, zero capacities, overcommitted
    # nodes, pods with non-zero requests >= 2^53; MINISCHED_SEQ_FAST=0 forces the
    # general form everywhere. Placements and tables equal the oracle either way.
    monkeypatch.setenv("MINISCHED_SEQ_FAST", fast)
    seed = n_nodes + 17
    nr = synth.nodes(n_nodes, seed=seed, resources=True)
    pr = synth.pods(n_pods, seed=seed, resources=True)
    nr["alloc_memory"][5::997] = 5 << 40
    nr["alloc_memory"][7::2113] = 1 << 60
    nr["alloc_milli_cpu"][3::89] = 0
    over = slice(11, None, 53)
    nr["nonzero_milli_cpu"][over] = nr["alloc_milli_cpu"][over] * 2 + 1
    nr["req_milli_cpu"][over] = nr["alloc_milli_cpu"][over] // 4
    pr["nonzero_memory"][13::701] = 1 << 54
    pr["req_memory"][13::701] = 0
    pr["req_milli_cpu"][13::701] = 0
    o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=seed)
    with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=seed) as e:
        assert_same(e.schedule(pr, MODE_SEQUENTIAL), o)
        assert_table_equal(e, o["cols"], n_nodes)
        assert e.info()._pad == 0


def test_resource_sequential_with_deltas(oracle):
    # the sequential engine across calls with node deltas in between: binds
    # carried over, a fifth of the nodes deleted (tombstones), half of those
    # re-added with fresh records; the derived rows of the binary64 sweep are
    # rebuilt at every call from the table (tests the rebuild, not only the
    # validator's write-back)
    n, seed = 3000, 21
    nr = synth.nodes(n, seed=seed, resources=True)
    pr = synth.pods(4500, seed=seed, resources=True)
    with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=seed) as e:
        o1 = oracle.schedule(nr, pr[:1500], plugin_set=1, mode=1, seed=seed)
        assert_same(e.schedule(pr[:1500], MODE_SEQUENTIAL), o1)
        cols = o1["cols"]
        dead = np.arange(7, n, 5)
        e.delete(dead)
        cols.flags[dead] |= 0x80
        o2 = oracle.schedule(nr, pr[1500:3000], plugin_set=1, mode=1, seed=seed, cols=cols)
        assert_same(e.schedule(pr[1500:3000], MODE_SEQUENTIAL), o2)
        back = dead[::2]
        e.upsert(back, nr[back])
        cols.flags[back] = nr["unschedulable"][back] & 1
        for c, f in (("pod_count", "pod_count"), ("req_cpu", "req_milli_cpu"), ("req_mem", "req_memory"),
                     ("nz_cpu", "nonzero_milli_cpu"), ("nz_mem", "nonzero_memory")):
            getattr(cols, c)[back] = nr[f][back]
        o3 = oracle.schedule(nr, pr[3000:], plugin_set=1, mode=1, seed=seed, cols=cols)
        assert_same(e.schedule(pr[3000:], MODE_SEQUENTIAL), o3)
        t = e.read(0, n)
        live = (cols.flags & 0x80) == 0
        for k_dev, k_or in (("pod_count", "pod_count"), ("req_milli_cpu", "req_cpu"), ("req_memory", "req_mem"),
                            ("nonzero_milli_cpu", "nz_cpu"), ("nonzero_memory", "nz_mem")):
            assert np.array_equal(t[k_dev][live], getattr(cols, k_or)[live]), k_dev
        assert e.info()._pad == 0


def _pods_with_zero_hash(seed, n_nodes, want=4):
    # pods j for which some node ordinal r < n_nodes has tie-break hash exactly 0:
    # mix32(A + r * kG24) == 0 <=> A + r * kG24 == 0 (mix32 is a bijection fixing 0),
    # so r = -A * kG24^-1 mod 2^32 (ms_internal.h tb_unhash(A, 0)); distinct digits r % 10
    import _pyref

    M = np.uint64(0xFFFFFFFF)

    def fmix32(h):
        h = h ^ (h >> np.uint64(16))
        h = (h * np.uint64(0x85EBCA6B)) & M
        h = h ^ (h >> np.uint64(13))
        h = (h * np.uint64(0xC2B2AE35)) & M
        return h ^ (h >> np.uint64(16))

    out, digits, j = [], set(), 0
    with np.errstate(over="ignore"):
        while len(out) < want:
            js = np.arange(j, j + 1 << 20, dtype=np.uint64)
            j += 1 << 20
            a = fmix32(js ^ np.uint64(_pyref.seed32(seed)))
            r = (((M + np.uint64(1) - a) & M) * np.uint64(0xF2B382C9)) & M
            for x in np.nonzero(r < np.uint64(n_nodes))[0]:
                rr = int(r[x])
                if rr % 10 not in digits and len(out) < want:
                    assert _pyref.h32(seed, int(js[x]), rr) == 0
                    digits.add(rr % 10)
                    out.append((int(js[x]), rr))
    return out


@pytest.mark.parametrize("rows", [99_870, 25_020, 130, 50_010])
@pytest.mark.parametrize("layout", ["cycle", "iid"])
def test_pp_packed_last_word(oracle, rows, layout):
    # K1 pp packs a workgroup's last lane word of <= 8 groups (8 pods per evaluation,
    # shared by up to 4 waves) where that lowers the busiest SIMD's load: 99,870 rows
    # (16 waves, 1 group left over), 25,020 (4 waves), 130 (one wave, one word);
    # 50,010 rows stay unpacked. i.i.d. digits take the bit-scan form, non-digit pods
    # and tiny clusters the exact slow path, both over the packed word.
    seed = 31 if layout == "cycle" else 32
    rng = np.random.default_rng(seed)
    nr = synth.nodes(rows, seed=seed)
    if layout == "iid":
        nr["name_digit"] = rng.integers(0, 10, rows)
    pr = synth.pods(2_500, seed=seed)
    pr["tolerates_unschedulable"][::5] = 1
    pr["name_digit"][::97] = -1
    o = oracle.schedule_nunn_omp(nr, pr, seed=seed) if rows > 1000 else oracle.schedule(nr, pr, seed=seed)
    with engine_with(nr, seed=seed) as e:
        assert_same(e.schedule(pr, MODE_BATCHED), o)


def test_pp_zero_hash_winner(oracle):
    # K1 pp treats a wave maximum of 0 as "no score-10 row here" and redoes the pod
    # exactly: a pod whose only feasible score-10 node hashes to exactly 0 must still
    # land on it, and with other score-10 nodes present the 0 must lose
    seed, n = 4, 1 << 15
    cases = _pods_with_zero_hash(seed, n, want=4)
    nr = synth.nodes(n, seed=seed)
    nr["unschedulable"] = 0
    pr = synth.pods(len(cases) * 2, seed=seed)
    for k, (j, r) in enumerate(cases):
        for t in (0, 1):
            p = pr[2 * k + t]
            p["ordinal"] = j
            p["name_digit"] = r % 10
            p["tolerates_unschedulable"] = t
    lone = nr.copy()
    for j, r in cases:  # every other node of that digit unschedulable
        same = (np.arange(n) % 10 == r % 10) & (np.arange(n) != r)
        lone["unschedulable"][same] = 1
    for table, tag in ((lone, "lone"), (nr, "crowded")):
        o = oracle.schedule(table, pr, seed=seed)
        with engine_with(table, seed=seed) as e:
            res = e.schedule(pr, MODE_BATCHED)
        assert_same(res, o)
        if tag == "lone":
            for k, (j, r) in enumerate(cases):
                assert res["node"][2 * k] == r and res["score"][2 * k] == 10, (j, r)


def test_stream_ordering_deltas_binds_reads(oracle):
    # work queued on a caller stream and the context stream's delta /
    # bind / read-back work must be ordered both ways. Rounds of select + bind
    # commit on a caller stream with informer upserts in between and no host sync:
    # each round must see exactly the table its call found, and the read-back at
    # the end must include every bind.
    import torch

    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    n, p, rounds = 40_000, 4000, 5
    nr = synth.nodes(n, seed=12)
    pr = synth.pods(p, seed=12)
    pods_d = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    outs = [torch.empty(p * 24, dtype=torch.uint8, device=dev) for _ in range(rounds)]
    tables, touched = [], np.zeros(n, dtype=bool)
    rng = np.random.default_rng(3)
    with engine_with(nr, seed=12) as e:
        cur = nr.copy()
        for k in range(rounds):
            tables.append(cur.copy())
            e.select_batch_device(p, pods_d.data_ptr(), outs[k].data_ptr(), s.cuda_stream)
            e.apply_binds_device(p, pods_d.data_ptr(), outs[k].data_ptr(), s.cuda_stream)
            idx = rng.choice(n, 3000, replace=False)  # an informer Update, mid-flight
            cur["unschedulable"][idx] = 1 - cur["unschedulable"][idx]
            e.upsert(idx, cur[idx])
            touched[idx] = True
        t = e.read(0, n)  # context stream: after every caller-stream bind
        s.synchronize()
    placed = np.zeros(n, dtype=np.int64)
    for k in range(rounds):
        res = outs[k].cpu().numpy().view(_lib.RESULT)
        assert_same(res, oracle.schedule(tables[k], pr, seed=12))
        ok = res["code"] == 0
        placed += np.bincount(res["node"][ok], minlength=n)
    # rows an upsert never replaced carry every round's binds
    keep = ~touched
    assert np.array_equal(t["pod_count"][keep], placed[keep])


@pytest.mark.parametrize("weights", [(1, 1), (2, 3), (10, 10)])
@pytest.mark.parametrize("n_nodes,n_pods", [(1, 5), (17, 64), (300, 200), (5000, 700), (40_000, 300)])
def test_na_batched(oracle, weights, n_nodes, n_pods):
    seed = n_nodes + 3 * n_pods + weights[1]
    nr = synth.nodes(n_nodes, seed=seed, zones=True)
    pr = synth.pods(n_pods, seed=seed, zones=True)
    pr["tolerates_unschedulable"][::6] = 1
    pr["name_digit"][::17] = -1
    nr["name_digit"][::9] = 0xFF
    literal = n_nodes <= 300  # the loop as written is O(F^2) per pod
    o = oracle.schedule_na(nr, pr, weights=weights, literal=literal, seed=seed)
    with Engine(max_nodes=n_nodes, plugin_set=_lib.PLUGINS_NU_NN_NA, seed=seed, score_weights=weights) as e:
        e.upsert(np.arange(n_nodes), nr)
        assert_same(e.schedule(pr, MODE_BATCHED), o)
        assert_same(e.schedule(pr, MODE_SEQUENTIAL), o)  # no mutable state: queue order changes nothing


def test_na_two_shards_combine(oracle):
    # node-sharded NA: keys combine with a u64 MAX and the normalise anchors with a u32 MAX
    import torch

    n, p, seed = 9000, 800, 21
    nr = synth.nodes(n, seed=seed, zones=True)
    pr = synth.pods(p, seed=seed, zones=True)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    pods_d = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    keys, anchors, engines = [], [], []
    for a, b in ((0, 4321), (4321, n)):
        e = Engine(max_nodes=b - a, plugin_set=_lib.PLUGINS_NU_NN_NA, node_base=a, seed=seed, score_weights=(2, 1))
        e.upsert(np.arange(a, b), nr[a:b])
        k = torch.empty(p, dtype=torch.int64, device=dev)
        f = torch.empty(p, dtype=torch.int32, device=dev)
        e.sweep_device(p, pods_d.data_ptr(), k.data_ptr(), f.data_ptr(), s.cuda_stream)
        keys.append(k)
        anchors.append(f)
        engines.append(e)
    with torch.cuda.stream(s):
        kc = torch.maximum(keys[0], keys[1])
        fc = torch.maximum(anchors[0], anchors[1])  # anchors < 2^21: the int32 max is the u32 max
    res = torch.empty(p * 24, dtype=torch.uint8, device=dev)
    engines[0].decode_device(p, pods_d.data_ptr(), kc.data_ptr(), fc.data_ptr(), n, res.data_ptr(), s.cuda_stream)
    s.synchronize()
    assert_same(res.cpu().numpy().view(_lib.RESULT), oracle.schedule_na(nr, pr, weights=(2, 1), literal=False, seed=seed))
    for e in engines:
        e.close()


def test_na_weight_validation():
    with pytest.raises(_lib.MSError):
        Engine(max_nodes=4, plugin_set=_lib.PLUGINS_NU_NN_NA, score_weights=(5, 20))  # 5*10 + 20*100 >= 2048
    with pytest.raises(_lib.MSError):
        Engine(max_nodes=4, plugin_set=PLUGINS_NU_NN, score_weights=(2, 1))  # weights are NA-only


@pytest.mark.parametrize("n_pods", [1, 60_000, 100_000, 50_000 * 3 + 5, 50_000 * 4 + 9, 500_003])
def test_host_arrays_zero_copy_chunks(oracle, n_pods):
    # ms_schedule_batch / _compact on a single NU+NN shard: the host narrows (or copies)
    # each chunk of pods into pinned memory, one compact cycle launch per chunk (binds
    # included), results widened (or copied) chunk by chunk while the next chunk runs;
    # 1, 2, 3 and 4 chunks, both record forms, both modes, binds accumulating across calls
    seed = 900 + n_pods % 97
    nr = synth.nodes(20_000, seed=seed)
    pr = synth.pods(n_pods, seed=seed, start=3)
    pr["name_digit"][::11] = -1
    pr["tolerates_unschedulable"][::5] = 1
    o = oracle.schedule(nr, pr, seed=seed)
    placed = np.bincount(o["node"][o["code"] == 0], minlength=20_000)
    with engine_with(nr, seed=seed) as e:
        assert_same(e.schedule(pr, MODE_BATCHED), o)
        prof = e.last_call_profile()
        assert prof["chunks"] == max(1, min(4, n_pods // 50_000)) and prof["total"] > 0  # (ms_capi.cpp kZcMinChunk)
        assert_same(e.schedule(pr, MODE_SEQUENTIAL), o)
        r = e.schedule_compact(_lib.compact_pods(pr))
        for k_res, k_or in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
            assert np.array_equal(r[k_res].astype(np.int64), o[k_or].astype(np.int64)), k_res
        assert np.array_equal(e.read(0, 20_000)["pod_count"], 3 * placed)
