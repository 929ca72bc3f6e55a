"""The library's OWN world > 1 node-sharded code, run on one GPU.

RCCL refuses two ranks of one communicator on the same GPU, so these tests load
the test-only build `libminisched_gpu_loopback.so` (`make comm-loopback`): the
same objects as the product library except that ms_comm.cpp's RCCL calls go to
an in-process rendezvous (csrc/ms_comm_loopback.h). G contexts, one per node
shard, are driven by G host threads (one thread per rank, SURVEY §8(b)
"Threading") and joined with ms_comm_init(rank, G). Everything else is the
product code path an 8-GPU driver run times: ms_sharded_submit / drain (slice
offsets, padded combine buffers, the pipelined grouped reduce-scatter, the slice
decodes), ms_schedule_batch on joined contexts (slices all-gathered, binds
committed per shard), and ms_schedule_sequential_device (the device-cursor
windows, the G-way candidate all-gather, the replicated validator, owner-only
write-back). Every result is compared with the oracle over the WHOLE cluster
(or the committed config-E fixture), and every shard's node table after the
binds with the oracle's columns. Reference: minisched/minisched.go:124-141
(the node loop that is sharded), :304-325 (selectHost over the union).
"""
import hashlib
import os
import threading
import traceback

import numpy as np
import pytest

from minisched_amd import _lib, sharded, synth
from minisched_amd.hostinfo import cpu_threads

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def lb():
    if not os.path.exists(_lib.LOOPBACK_LIB_PATH):
        pytest.fail("libminisched_gpu_loopback.so is missing: `make -C mini-kube-scheduler_amd comm-loopback`")
    return _lib.load(_lib.LOOPBACK_LIB_PATH)


def _same(res, o, a, b, tag):
    for k_res, k_or in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
        got, want = np.asarray(res[k_res]).astype(np.int64), np.asarray(o[k_or][a:b]).astype(np.int64)
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0][:8]
            raise AssertionError(f"{tag} {k_res} differs at {(bad + a).tolist()}: "
                                 f"gpu {got[bad].tolist()} oracle {want[bad].tolist()}")


def run_ranks(G, fn, timeout=900):
    """fn(rank) on G threads (ctypes releases the GIL inside every library call);
    returns the per-rank results, failing on any rank's exception or a hang."""
    out, errs = [None] * G, [None] * G

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException:  # reported below
            errs[r] = traceback.format_exc()

    ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(G)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout)
    assert not any(t.is_alive() for t in ts), "a rank thread did not finish"
    bad = [e for e in errs if e]
    assert not bad, "\n".join(bad)
    return out


def _cuts(n, G, uneven=False):
    if not uneven:
        return [sharded.shard_bounds(n, r, G) for r in range(G)]
    # very uneven shards: rank r gets weight r + 1 (the last shard is the largest)
    w = np.arange(1, G + 1, dtype=np.float64)
    edges = np.concatenate([[0], np.floor(np.cumsum(w) / w.sum() * n)]).astype(np.int64)
    edges[-1] = n
    return [(int(edges[r]), int(edges[r + 1])) for r in range(G)]


def _joined(lib, cid, rank, G, nr, lo, hi, plugin_set, seed, dead=()):
    e = _lib.Engine(max_nodes=hi - lo, plugin_set=plugin_set, node_base=lo, seed=seed, lib=lib)
    e.upsert(np.arange(lo, hi), nr[lo:hi])
    e.flush()
    gone = np.asarray([d for d in dead if lo <= d < hi], dtype=np.uint32)
    if len(gone):
        e.delete(gone)
        e.flush()
    e.comm_init(cid, rank, G)
    info = e.info()
    assert (info.comm_rank, info.comm_world) == (rank, G)
    return e


def _sharded_cycle(lib, nr, pr, G, plugin_set, seed, steps=6, uneven=False, dead=(), caller_stream=True):
    """ms_sharded_submit x steps + ms_sharded_drain on G joined contexts; returns
    [(first, count, results)] per rank."""
    import torch

    cuts = _cuts(len(nr), G, uneven)
    cid = _lib.comm_id_create(lib)
    dev = torch.device("cuda:0")
    host_pods = pr.view(np.uint8).copy()

    def rank_fn(r):
        lo, hi = cuts[r]
        e = _joined(lib, cid, r, G, nr, lo, hi, plugin_set, seed, dead)
        try:
            first, count = e.sharded_slice(len(pr))
            assert (first, first + count) == sharded.pod_slice(len(pr), r, G)
            pods = torch.from_numpy(host_pods).to(dev)
            res = torch.full((max(1, count) * 24,), 0xAB, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()  # (the copy and the fill ran on torch's stream, not the library's)
            s = torch.cuda.Stream(device=dev) if caller_stream else None
            sp = s.cuda_stream if s is not None else 0
            for _ in range(steps):  # more than the pipeline depth: slots are reused after their decodes
                e.sharded_submit(len(pr), pods.data_ptr(), res.data_ptr(), sp)
            e.sharded_drain(sp)
            if s is not None:
                s.synchronize()
            torch.cuda.synchronize()
            return first, count, res.cpu().numpy().view(_lib.RESULT)[:count].copy()
        finally:
            e.close()

    return run_ranks(G, rank_fn)


def _oracle_for(oracle, nr, pr, plugin_set, seed, dead=()):
    nr = nr.copy()
    if len(dead):
        nr["allowed_pods"][np.asarray(dead)] = -1  # oracle: absent from the node list
    if plugin_set == _lib.PLUGINS_NU_NN_NA:
        return oracle.schedule_na(nr, pr, seed=seed, literal=False)
    if plugin_set == _lib.PLUGINS_NU_TT_NN:
        return oracle.schedule_tt(nr, pr, seed=seed, literal=False)
    if plugin_set == _lib.PLUGINS_NU_NN:
        return oracle.schedule_nunn_omp(nr, pr, seed=seed, threads=cpu_threads())
    return oracle.schedule(nr, pr, plugin_set=plugin_set, seed=seed)


@pytest.mark.parametrize("plugin_set", [0, 1, 2, 3])
@pytest.mark.parametrize("G,uneven", [(2, False), (3, True), (4, False), (8, True)])
def test_loopback_sharded_cycle(lb, oracle, plugin_set, G, uneven):
    # every plugin set's combine (keys; filter bytes; NodeAffinity anchors; TaintToleration
    # summaries through the all-to-all) at world G,
    # pods not divisible by G (3001), uneven shards, deleted nodes on one shard and a
    # shard with every node deleted (it contributes key 0 / empty flags)
    seed = 300 + 10 * G + plugin_set
    res_set, zones, taints = plugin_set == 1, plugin_set == 2, plugin_set == 3
    n = 9000
    nr = synth.nodes(n, seed=seed, resources=res_set, zones=zones, taints=taints)
    pr = synth.pods(3001, seed=seed, resources=res_set, zones=zones, taints=taints)
    pr["name_digit"][::17] = -1
    cuts = _cuts(n, G, uneven)
    dead = list(range(cuts[0][0], cuts[0][1])) + list(range(cuts[-1][0], cuts[-1][1], 3))
    o = _oracle_for(oracle, nr, pr, plugin_set, seed, dead)
    before = lb.lb_collectives_issued()
    got = _sharded_cycle(lb, nr, pr, G, plugin_set, seed, uneven=uneven, dead=dead)
    assert lb.lb_collectives_issued() - before >= 6  # the reduce-scatters really ran at world G
    covered = 0
    for r, (first, count, res) in enumerate(got):
        _same(res, o, first, first + count, f"G={G} rank {r}")
        covered += count
    assert covered == len(pr)


@pytest.mark.parametrize("mode", ["two_sweep_streams", "alternating_caller_streams"])
def test_loopback_tt_distinct_batches_concurrent_streams(lb, oracle, monkeypatch, mode):
    # TaintToleration submits share the context's segment-summary
    # scratch. With two sweep streams (MINISCHED_SHARD_STREAMS=2), or consecutive
    # submits on different caller streams, two batches' sweeps could run at once on
    # it; each submit here carries a DIFFERENT pod batch into its own result buffer,
    # so an unordered overlap shows up as a wrong result
    import torch

    if mode == "two_sweep_streams":
        monkeypatch.setenv("MINISCHED_SHARD_STREAMS", "2")
    G, seed, n, nb, steps = 2, 707, 6000, 1500, 6
    nr = synth.nodes(n, seed=seed, taints=True)
    pr = synth.pods(nb * steps, seed=seed, taints=True)
    o = _oracle_for(oracle, nr, pr, _lib.PLUGINS_NU_TT_NN, seed)
    cuts = _cuts(n, G)
    cid = _lib.comm_id_create(lb)
    dev = torch.device("cuda:0")
    host_pods = pr.view(np.uint8).copy()

    def rank_fn(r):
        lo, hi = cuts[r]
        e = _joined(lb, cid, r, G, nr, lo, hi, _lib.PLUGINS_NU_TT_NN, seed)
        try:
            first, count = e.sharded_slice(nb)
            pods = torch.from_numpy(host_pods).to(dev)
            res = [torch.full((max(1, count) * 24,), 0xAB, dtype=torch.uint8, device=dev) for _ in range(steps)]
            torch.cuda.synchronize()
            ss = [torch.cuda.Stream(device=dev) for _ in range(2)]
            for k in range(steps):
                s = ss[k % 2] if mode == "alternating_caller_streams" else ss[0]
                e.sharded_submit(nb, pods.data_ptr() + 40 * nb * k, res[k].data_ptr(), s.cuda_stream)
            for s in ss:
                e.sharded_drain(s.cuda_stream)
            torch.cuda.synchronize()
            return first, count, [x.cpu().numpy().view(_lib.RESULT)[:count].copy() for x in res]
        finally:
            e.close()

    got = run_ranks(G, rank_fn)
    for r, (first, count, res) in enumerate(got):
        for k in range(steps):
            _same(res[k], o, nb * k + first, nb * k + first + count, f"TT {mode} rank {r} batch {k}")


@pytest.mark.parametrize("G", [2, 4, 8])
def test_loopback_config_c_full(lb, oracle, G):
    # config C at full size (100k nodes x 100k pods) through the library's pipelined
    # world-G path, against the OpenMP oracle over the whole cluster
    nr = synth.nodes(100_000, seed=1)
    pr = synth.pods(100_000, seed=1)
    o = oracle.schedule_nunn_omp(nr, pr, seed=1, threads=cpu_threads())
    got = _sharded_cycle(lb, nr, pr, G, 0, 1, steps=5)
    for r, (first, count, res) in enumerate(got):
        _same(res, o, first, first + count, f"C G={G} rank {r}")
    assert sum(c for _, c, _ in got) == 100_000


def test_loopback_config_c_weak_full(lb, oracle):
    # weak scaling at G = 8: 800k pods against 100k nodes, every rank's 12.5k-row shard
    # sweeps all of them, the reduce-scatter leaves each rank 100k pods to decode
    nr = synth.nodes(100_000, seed=1)
    pr = synth.pods(800_000, seed=1)
    o = oracle.schedule_nunn_omp(nr, pr, seed=1, threads=cpu_threads())
    got = _sharded_cycle(lb, nr, pr, 8, 0, 1, steps=2)
    for r, (first, count, res) in enumerate(got):
        assert count == 100_000
        _same(res, o, first, first + count, f"weak rank {r}")


def _schedule_ranks(lb, nr, pr, G, plugin_set, mode, seed, uneven=True, compact=False):
    cuts = _cuts(len(nr), G, uneven)
    cid = _lib.comm_id_create(lb)

    def rank_fn(r):
        lo, hi = cuts[r]
        e = _joined(lb, cid, r, G, nr, lo, hi, plugin_set, seed)
        try:
            if compact:
                res = e.schedule_compact(_lib.compact_pods(pr), mode)
            else:
                res = e.schedule(pr, mode)
            return res.copy(), e.read(lo, hi - lo)
        finally:
            e.close()

    return cuts, run_ranks(G, rank_fn)


def _check_tables(cuts, got, cols, tag):
    t = np.concatenate([tab for _, tab in got])
    for k_dev, k_or in (("pod_count", "pod_count"), ("req_milli_cpu", "req_cpu"), ("req_memory", "req_mem"),
                        ("nonzero_milli_cpu", "nz_cpu"), ("nonzero_memory", "nz_mem")):
        if not np.array_equal(t[k_dev], getattr(cols, k_or)):
            raise AssertionError(f"{tag}: node table column {k_dev} differs after the binds")


@pytest.mark.parametrize("plugin_set,mode", [(0, 0), (0, 1), (1, 0), (1, 1), (2, 0), (2, 1), (3, 0), (3, 1)])
def test_loopback_schedule_batch(lb, oracle, plugin_set, mode):
    # ms_schedule_batch on joined contexts (world 3, uneven shards): every rank returns
    # every pod's result (the all-gather of the slices / the replicated validator), and
    # each shard commits only its own nodes' binds
    G, seed = 3, 400 + 2 * plugin_set + mode
    res_set, zones, taints = plugin_set == 1, plugin_set == 2, plugin_set == 3
    n_nodes, n_pods = (1200, 7001) if res_set else (5000, 4001)
    nr = synth.nodes(n_nodes, seed=seed, resources=res_set, zones=zones, taints=taints)
    pr = synth.pods(n_pods, seed=seed, resources=res_set, zones=zones, taints=taints)
    pr["name_digit"][::23] = -1
    if plugin_set == 1:
        o = (oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=seed) if mode == 1
             else oracle.schedule_batched_commit(nr, pr, 1, seed=seed))
        if mode == 1:
            assert (o["code"] == 2).sum() > 0  # saturation reached
    else:
        o = _oracle_for(oracle, nr, pr, plugin_set, seed)
        cols = oracle.NodeCols(nr)  # binds of a stateless set: AddPod on each winner
        for j in np.nonzero(o["code"] == 0)[0]:
            i = int(o["node"][j])
            cols.pod_count[i] += 1
            cols.req_cpu[i] += pr["req_milli_cpu"][j]
            cols.req_mem[i] += pr["req_memory"][j]
            cols.nz_cpu[i] += pr["nonzero_milli_cpu"][j]
            cols.nz_mem[i] += pr["nonzero_memory"][j]
        o["cols"] = cols
    cuts, got = _schedule_ranks(lb, nr, pr, G, plugin_set, mode, seed)
    for r, (res, _tab) in enumerate(got):
        _same(res, o, 0, len(pr), f"set {plugin_set} mode {mode} rank {r}")
    _check_tables(cuts, got, o["cols"], f"set {plugin_set} mode {mode}")


def test_loopback_schedule_batch_compact(lb, oracle):
    # ms_schedule_batch_compact on joined contexts (the staged form; world 4)
    G, seed = 4, 470
    nr = synth.nodes(6000, seed=seed)
    pr = synth.pods(5003, seed=seed)
    o = oracle.schedule(nr, pr, seed=seed)
    _cuts_, got = _schedule_ranks(lb, nr, pr, G, 0, 0, seed, compact=True)
    for r, (res, _tab) in enumerate(got):
        for k_res, k_or in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
            assert np.array_equal(res[k_res].astype(np.int64), o[k_or].astype(np.int64)), f"rank {r} {k_res}"


def _sequential_ranks(lb, nr, pr, G, seed, uneven=False):
    import torch

    cuts = _cuts(len(nr), G, uneven)
    cid = _lib.comm_id_create(lb)
    dev = torch.device("cuda:0")
    host_pods = pr.view(np.uint8).copy()

    def rank_fn(r):
        lo, hi = cuts[r]
        e = _joined(lb, cid, r, G, nr, lo, hi, _lib.PLUGINS_NU_NRF_NN_LA, seed)
        try:
            pods = torch.from_numpy(host_pods).to(dev)
            res = torch.zeros(len(pr) * 24, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()  # (the copy and the fill ran on torch's stream, not s)
            s = torch.cuda.Stream(device=dev)
            e.schedule_sequential_device(len(pr), pods.data_ptr(), res.data_ptr(), s.cuda_stream)
            s.synchronize()
            return res.cpu().numpy().view(_lib.RESULT).copy(), e.read(lo, hi - lo)
        finally:
            e.close()

    return cuts, run_ranks(G, rank_fn)


@pytest.mark.parametrize("G,window,uneven", [(2, "128", False), (3, "7", True), (4, "256", True), (5, "1", False)])
def test_loopback_sequential_device(lb, oracle, monkeypatch, G, window, uneven):
    # ms_schedule_sequential_device at world G: device-cursor windows, the G-way grouped
    # all-gather of candidates + flags, the replicated validator, owner-only write-back
    monkeypatch.setenv("MINISCHED_SHARD_SEQ_BATCH", window)
    seed = 500 + G
    nr = synth.nodes(1500, seed=seed, resources=True)
    pr = synth.pods(4000 if window != "1" else 900, seed=seed, resources=True)
    pr["name_digit"][::29] = -1
    o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=seed)
    cuts, got = _sequential_ranks(lb, nr, pr, G, seed, uneven)
    for r, (res, _tab) in enumerate(got):
        _same(res, o, 0, len(pr), f"seq G={G} W={window} rank {r}")
    _check_tables(cuts, got, o["cols"], f"seq G={G}")


def test_loopback_config_e_full_four_ranks(lb):
    # config E at full size (50k nodes x 200k pods, exact sequential) at world 4 through
    # ms_schedule_sequential_device, against the committed fixture and its table digest
    fx = np.load(os.path.join(HERE, "golden", "config_e_full_seed1.npz"))
    nr = synth.nodes(50_000, seed=1, resources=True)
    pr = synth.pods(200_000, seed=1, resources=True)
    cuts, got = _sequential_ranks(lb, nr, pr, 4, 1)
    o = {k: fx[k] for k in ("node", "code", "score", "mask")}
    for r, (res, _tab) in enumerate(got):
        _same(res, o, 0, len(pr), f"E rank {r}")
    t = np.concatenate([tab for _, tab in got])
    h = hashlib.sha256()
    for k in ("pod_count", "req_milli_cpu", "req_memory", "nonzero_milli_cpu", "nonzero_memory"):
        h.update(np.ascontiguousarray(t[k], dtype=np.int64).tobytes())
    assert h.hexdigest() == str(fx["table_sha256"])


def test_loopback_mismatched_collectives_fail_cleanly(lb):
    # ranks that issue different collectives (different batch sizes) get MS_E_RCCL back,
    # not a hang; the contexts still close
    G, seed = 2, 610
    nr = synth.nodes(2000, seed=seed)
    cuts = _cuts(2000, G)
    cid = _lib.comm_id_create(lb)

    def rank_fn(r):
        import torch

        lo, hi = cuts[r]
        e = _joined(lb, cid, r, G, nr, lo, hi, 0, seed)
        try:
            n = 1000 if r == 0 else 2000
            pr = synth.pods(n, seed=seed)
            dev = torch.device("cuda:0")
            pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
            res = torch.zeros(n * 24, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            with pytest.raises(_lib.MSError) as ei:
                e.sharded_submit(n, pods.data_ptr(), res.data_ptr(), 0)
                e.sharded_drain(0)
            assert ei.value.code == _lib.MS_E_RCCL
            torch.cuda.synchronize()
        finally:
            e.close()

    run_ranks(G, rank_fn, timeout=300)


@pytest.mark.parametrize("G,r", [(4, 2), (8, 7)])
def test_solo_rank_probe_mode(lb, oracle, monkeypatch, G, r):
    # MS_LB_SOLO=1 (tools/step_probe_rank.py): ONE rank of a G-rank
    # communicator on its own -- its shard sweep, its ceil(P/G)-pod slice, a G-way MAX
    # reduce-scatter over G copies of its own keys, the slice decode -- the per-rank work
    # of the driver's G-GPU run. Its slice therefore holds the best over ITS shard only:
    # the oracle over that shard's rows equals it
    import torch

    monkeypatch.setenv("MS_LB_SOLO", "1")
    N, P, seed = 24_000, 9_001, 5
    lo, hi = sharded.shard_bounds(N, r, G)
    nr, pr = synth.nodes(N, seed=seed), synth.pods(P, seed=seed)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    e = _lib.Engine(max_nodes=hi - lo, node_base=lo, seed=seed, lib=lb)
    try:
        e.upsert(np.arange(lo, hi), nr[lo:hi])
        e.flush()
        e.comm_init(_lib.comm_id_create(lb), r, G)
        cyc = sharded.ShardedCycle(e, N, P, pods, s)
        assert cyc.library and (cyc.a, cyc.b) == (r * -(-P // G), min(P, (r + 1) * -(-P // G)))
        for _ in range(3):  # (pipelined submits, then the drain)
            cyc.step()
        cyc.finish()
        s.synchronize()
        got = cyc.results.cpu().numpy().view(_lib.RESULT)[: cyc.b - cyc.a]
    finally:
        e.close()
    o = oracle.schedule(nr[lo:hi], pr[cyc.a:cyc.b], seed=seed, node_base=lo)
    _same(got, {k: np.concatenate([np.zeros(cyc.a, v.dtype), v]) for k, v in o.items() if k != "cols"},
          cyc.a, cyc.b, f"solo rank {r} of {G}")
