"""N > 1 bench path on one GPU: two ranks (gloo, both on cuda:0) run
sharded.ShardedCycle exactly as bench.py does — the HIP sweep of each node
shard, the cross-shard MAX reduce-scatter, the decode of each rank's pod
slice (pipelined at depth 1 and 2), and the pod-split replicas — and every
rank's decoded slice must equal the oracle's over the whole cluster. A 1-rank
RCCL group drives the same pipeline through torch's "nccl" backend
(reduce_scatter_tensor, ordered drains, grouped decodes).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from minisched_amd import synth

pytestmark = pytest.mark.gpu

N_NODES, N_PODS, SEED = 30_000, 5_001, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _same(res, o, a, b, tag):
    for k_res, k_or in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
        assert np.array_equal(res[k_res], o[k_or][a:b]), f"{tag} {k_res}"


def _dead(kind):
    """Global ordinals deleted before the cycle (the FitError mask must use the
    cluster's present count; with every node gone the reference reports an empty plugin set)."""
    if kind == "third":
        return np.arange(0, N_NODES, 3)
    if kind == "all":
        return np.arange(N_NODES)
    return np.arange(0)


def _worker(rank, world, port, split, depth, group, q, dead=None):
    import torch
    import torch.distributed as dist

    from minisched_amd import _lib, sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lo, hi = sharded.shard_bounds(N_NODES, rank, world) if split == "nodes" else (0, N_NODES)
        eng = _lib.Engine(max_nodes=hi - lo, plugin_set=_lib.PLUGINS_NU_NN, node_base=lo, seed=SEED)
        eng.upsert(np.arange(lo, hi, dtype=np.uint32), synth.nodes(hi - lo, seed=SEED, start=lo))
        eng.flush()
        gone = _dead(dead)
        gone = gone[(gone >= lo) & (gone < hi)]
        if len(gone):
            eng.delete(gone.astype(np.uint32))
            eng.flush()
        present = sharded.present_total(eng) if split == "nodes" else None
        pods = torch.from_numpy(synth.pods(N_PODS, seed=SEED).view(np.uint8).copy()).to(dev)
        stream = torch.cuda.Stream(device=dev)
        torch.cuda.set_stream(stream)
        cyc = sharded.ShardedCycle(eng, N_NODES, N_PODS, pods, stream, split=split, depth=depth,
                                   drain_group=group, rank=rank, world=world, present_total=present)
        for _ in range(5):  # key buffers reused after their decodes
            cyc.step()
        cyc.finish()
        torch.cuda.synchronize()
        res = cyc.results.cpu().numpy().view(_lib.RESULT)[: cyc.b - cyc.a].copy()
        eng.close()
        dist.destroy_process_group()
        q.put((rank, cyc.a, cyc.b, res, present, None))
    except Exception as e:  # reported to the parent, which fails the test
        q.put((rank, 0, 0, None, None, repr(e)))


@pytest.mark.parametrize("split,depth,group,dead", [("nodes", 1, 1, None), ("nodes", 2, 2, None), ("nodes", 3, 1, None),
                                                    ("pods", 1, 1, None), ("nodes", 1, 1, "third"),
                                                    ("nodes", 1, 1, "all"), ("pods", 1, 1, "third")])
def test_two_rank_cycle_on_gpu(oracle, split, depth, group, dead):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, split, depth, group, q, dead)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=110) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [e for *_, e in got if e]
    assert not errs, errs
    nr = synth.nodes(N_NODES, seed=SEED)
    nr["allowed_pods"][_dead(dead)] = -1  # oracle: absent from the node list
    o = oracle.schedule(nr, synth.pods(N_PODS, seed=SEED), seed=SEED)
    covered = 0
    for rank, a, b, res, present, _ in got:
        _same(res, o, a, b, f"rank {rank}")
        covered += b - a
        if split == "nodes":
            assert present == N_NODES - len(_dead(dead))  # summed over the shards
    if dead == "all":
        assert (o["mask"] == 0).all() and (o["code"] != 0).all()
    assert covered == N_PODS


def _rccl_worker(port, depth, group, q):
    import torch
    import torch.distributed as dist

    from minisched_amd import _lib, sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        eng = _lib.Engine(max_nodes=N_NODES, plugin_set=_lib.PLUGINS_NU_NN, node_base=0, seed=SEED)
        eng.upsert(np.arange(N_NODES, dtype=np.uint32), synth.nodes(N_NODES, seed=SEED))
        eng.flush()
        pods = torch.from_numpy(synth.pods(N_PODS, seed=SEED).view(np.uint8).copy()).to(dev)
        stream = torch.cuda.Stream(device=dev)
        torch.cuda.set_stream(stream)
        cyc = sharded.ShardedCycle(eng, N_NODES, N_PODS, pods, stream, depth=depth, drain_group=group,
                                   collective=True, present_total=sharded.present_total(eng))
        ordered = cyc._pipe.ordered
        for _ in range(7):  # the world > 1 form: RCCL reduce-scatter per step, grouped drains
            cyc.step()
        cyc.finish()
        torch.cuda.synchronize()
        res = cyc.results.cpu().numpy().view(_lib.RESULT).copy()
        eng.close()
        dist.destroy_process_group()
        q.put((ordered, res, None))
    except Exception as e:
        q.put((None, None, repr(e)))


@pytest.mark.parametrize("depth,group", [(2, 2), (4, 4), (3, 1)])
def test_rccl_pipeline(oracle, depth, group):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), depth, group, q))
    p.start()
    ordered, res, err = q.get(timeout=110)
    p.join(timeout=60)
    assert err is None, err
    assert ordered
    o = oracle.schedule(synth.nodes(N_NODES, seed=SEED), synth.pods(N_PODS, seed=SEED), seed=SEED)
    _same(res, o, 0, N_PODS, "rccl")


def test_decode_device_jobs_matches_oracle(oracle):
    # ms_decode_device_jobs: three batches of different sizes swept into their own
    # key buffers, decoded in one launch, each equal to the oracle
    import torch

    from minisched_amd import _lib

    dev = torch.device("cuda:0")
    n_nodes = 7_000
    eng = _lib.Engine(max_nodes=n_nodes, plugin_set=_lib.PLUGINS_NU_NN, node_base=0, seed=SEED)
    try:
        nr = synth.nodes(n_nodes, seed=SEED)
        eng.upsert(np.arange(n_nodes, dtype=np.uint32), nr)
        eng.flush()
        stream = torch.cuda.Stream(device=dev)
        sizes = [1000, 333, 2049]
        batches, jobs = [], []
        for k, n in enumerate(sizes):
            pr = synth.pods(n, seed=40 + k)
            pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
            keys = torch.empty(n, dtype=torch.int64, device=dev)
            res = torch.full((n * 24,), 0xAB, dtype=torch.uint8, device=dev)
            eng.sweep_device(n, pods.data_ptr(), keys.data_ptr(), 0, stream.cuda_stream)
            batches.append((pr, pods, keys, res))
            jobs.append((n, pods.data_ptr(), keys.data_ptr(), 0, res.data_ptr()))
        eng.decode_device_jobs(jobs, n_nodes, stream.cuda_stream)
        torch.cuda.synchronize()
        for k, (pr, _pods, _keys, res) in enumerate(batches):
            got = res.cpu().numpy().view(_lib.RESULT)
            o = oracle.schedule(nr, pr, seed=SEED)
            _same(got, o, 0, len(pr), f"batch {k}")
        with pytest.raises(RuntimeError):
            eng.decode_device_jobs(jobs * 3, n_nodes, stream.cuda_stream)  # > MS_DECODE_MAX_JOBS
    finally:
        eng.close()


@pytest.mark.parametrize("cuts,n_pods,batch", [((0, 23, 60), 700, 64), ((0, 700, 1400, 2000), 12_000, 128),
                                              ((0, 9000, 20_000), 30_000, 256), ((0, 3, 7), 300, 16)])
def test_node_sharded_sequential_contexts(oracle, cuts, n_pods, batch):
    # config E over node shards on one GPU: one context per shard, the all-gather done by
    # concatenation; every shard's replicated validation must agree, the results equal the
    # 1-context sequential oracle, and the shards' tables after the binds its columns
    import torch

    from minisched_amd import _lib

    n_nodes = cuts[-1]
    seed = 40 + n_nodes
    nr = synth.nodes(n_nodes, seed=seed, resources=True)
    pr = synth.pods(n_pods, seed=seed, resources=True)
    pr["name_digit"][::19] = -1
    o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=seed)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    sp = s.cuda_stream
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    G = len(cuts) - 1
    engines = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        e = _lib.Engine(max_nodes=b - a, plugin_set=_lib.PLUGINS_NU_NRF_NN_LA, node_base=a, seed=seed)
        e.upsert(np.arange(a, b), nr[a:b])
        engines.append(e)
    cb = _lib.SEQ_CAND.itemsize * _lib.SEQ_TOPK
    cands = [torch.zeros(batch * cb, dtype=torch.uint8, device=dev) for _ in range(G)]
    flags = [torch.zeros(batch, dtype=torch.int32, device=dev) for _ in range(G)]
    res = [torch.zeros(n_pods * 24, dtype=torch.uint8, device=dev) for _ in range(G)]
    done = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in range(G)]
    a, batches = 0, 0
    try:
        while a < n_pods:
            nb = min(batch, n_pods - a)
            for g, e in enumerate(engines):
                e.seq_candidates_device(nb, pods.data_ptr() + 40 * a, cands[g].data_ptr(), flags[g].data_ptr(), sp)
            with torch.cuda.stream(s):
                call = torch.cat([c[: nb * cb] for c in cands])
                fall = torch.cat([f[:nb] for f in flags])
            for g, e in enumerate(engines):
                e.seq_validate_device(nb, pods.data_ptr() + 40 * a, G, call.data_ptr(), fall.data_ptr(),
                                      res[g].data_ptr() + 24 * a, done[g].data_ptr(), sp)
            s.synchronize()
            nd = [int(d.item()) for d in done]
            assert len(set(nd)) == 1 and nd[0] >= 1, nd
            a += nd[0]
            batches += 1
        tables = [e.read(lo, hi - lo) for e, lo, hi in zip(engines, cuts[:-1], cuts[1:])]
    finally:
        for e in engines:
            e.close()
    for g in range(G):
        _same(res[g].cpu().numpy().view(_lib.RESULT), o, 0, n_pods, f"shard {g}")
    t = np.concatenate(tables)
    cols = o["cols"]
    for k_dev, k_or in (("pod_count", "pod_count"), ("req_milli_cpu", "req_cpu"), ("req_memory", "req_mem"),
                        ("nonzero_milli_cpu", "nz_cpu"), ("nonzero_memory", "nz_mem")):
        assert np.array_equal(t[k_dev], getattr(cols, k_or)), k_dev
    assert batches >= (n_pods + batch - 1) // batch


def _seq_rccl_worker(port, q):
    import torch
    import torch.distributed as dist

    from minisched_amd import _lib, sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        n, p = 3000, 9000
        eng = _lib.Engine(max_nodes=n, plugin_set=_lib.PLUGINS_NU_NRF_NN_LA, seed=5)
        eng.upsert(np.arange(n), synth.nodes(n, seed=5, resources=True))
        pods = torch.from_numpy(synth.pods(p, seed=5, resources=True).view(np.uint8).copy()).to(dev)
        stream = torch.cuda.Stream(device=dev)
        torch.cuda.set_stream(stream)
        cyc = sharded.ShardedSequential(eng, p, pods, stream, batch=128)
        res = cyc.run().cpu().numpy().view(_lib.RESULT).copy()
        t = eng.read(0, n)
        eng.close()
        dist.destroy_process_group()
        q.put((res, t["pod_count"].copy(), None))
    except Exception as e:
        q.put((None, None, repr(e)))


def test_sharded_sequential_class_rccl(oracle):
    # sharded.ShardedSequential through a 1-rank RCCL group (the world-1 gather path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr_ = ctx.Process(target=_seq_rccl_worker, args=(_free_port(), q))
    pr_.start()
    res, cnt, err = q.get(timeout=110)
    pr_.join(timeout=60)
    assert err is None, err
    o = oracle.schedule(synth.nodes(3000, seed=5, resources=True), synth.pods(9000, seed=5, resources=True),
                        plugin_set=1, mode=1, seed=5)
    _same(res, o, 0, 9000, "rccl seq")
    assert np.array_equal(cnt, o["cols"].pod_count)


# ---- multi-GPU inside the library (ms_comm_*): a 1-rank RCCL communicator -----
# RCCL refuses two ranks of one communicator on the same GPU ("Duplicate GPU
# detected", tools/probe_rccl_dup.py), so on a 1-GPU box the in-library path
# runs as a 1-rank communicator: the same submit / grouped reduce-scatter /
# slice decode / all-gather code with G = 1. The G > 1 slicing and combine
# arithmetic is checked at full size by the multi-context tests below.

def _comm_engine(nr, plugin_set, seed, node_base=0, **kw):
    from minisched_amd import _lib, sharded

    e = _lib.Engine(max_nodes=len(nr), plugin_set=plugin_set, node_base=node_base, seed=seed, **kw)
    e.upsert(np.arange(node_base, node_base + len(nr)), nr)
    e.flush()
    sharded.init_comm(e)  # no process group: a 1-rank communicator
    info = e.info()
    assert (info.comm_rank, info.comm_world) == (0, 1)
    return e


@pytest.mark.parametrize("plugin_set", [0, 1, 2])
def test_library_sharded_cycle_1rank(oracle, plugin_set):
    # ShardedCycle on a communicator: ms_sharded_submit / ms_sharded_drain, pipelined
    # (more steps than the depth), every plugin set's combine (keys, filter bytes,
    # NodeAffinity anchors, the listed-node flag)
    import torch

    from minisched_amd import _lib, sharded

    seed = 60 + plugin_set
    res_set, zones = plugin_set == 1, plugin_set == 2
    nr = synth.nodes(9000, seed=seed, resources=res_set, zones=zones)
    pr = synth.pods(3001, seed=seed, resources=res_set, zones=zones)
    pr["name_digit"][::17] = -1
    if plugin_set == 2:
        o = oracle.schedule_na(nr, pr, seed=seed, literal=False)
    else:
        o = oracle.schedule(nr, pr, plugin_set=plugin_set, seed=seed)
    dev = torch.device("cuda:0")
    e = _comm_engine(nr, plugin_set, seed)
    try:
        stream = torch.cuda.Stream(device=dev)
        pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
        cyc = sharded.ShardedCycle(e, len(nr), len(pr), pods, stream)
        assert cyc.library and (cyc.a, cyc.b) == (0, len(pr))
        for _ in range(7):
            cyc.step()
        cyc.finish()
        stream.synchronize()
        res = cyc.results.cpu().numpy().view(_lib.RESULT)
        with pytest.raises(_lib.MSError):  # single-shard call on a sharded context
            e.select_batch_device(len(pr), pods.data_ptr(), cyc.results.data_ptr(), stream.cuda_stream)
    finally:
        e.close()
    _same(res, o, 0, len(pr), "library cycle")


@pytest.mark.parametrize("coalesce,words,prof", [("1", "", "1"), ("0", "", ""), ("1", "8", ""), ("1", "4", "")])
def test_library_submit_coalescing(oracle, monkeypatch, capfd, coalesce, words, prof):
    # Consecutive NU+NN submits share one K1 launch (ms_comm.cpp submit_locked's
    # stash): distinct pod batches of distinct sizes, an odd count (the last one
    # swept alone at the drain), and a node delta between two submits (the
    # stashed sweep must read the table BEFORE the delta, as submitted). Both
    # K1 forms for small shards (MINISCHED_PP_WORDS: 8 = one wave holds every
    # row, chosen above 1024 pods per CU; 4) under the two-batch launch.
    import torch

    from minisched_amd import _lib

    monkeypatch.setenv("MINISCHED_SHARD_COALESCE", coalesce)
    if words:
        monkeypatch.setenv("MINISCHED_PP_WORDS", words)
    if prof:  # the per-submit host clocks (tools/step_probe_lib.py reads them), printed at teardown
        monkeypatch.setenv("MINISCHED_HOST_PROF", prof)
    nr = synth.nodes(5000, seed=81)
    batches = [synth.pods(n, seed=81 + i) for i, n in enumerate((700, 1200, 333, 2048, 901))]
    nr2 = nr.copy()
    nr2["unschedulable"][::5] ^= 1  # the delta: NodeUnschedulable flips, NodeNumber digits move
    nr2["name_digit"][::7] = (nr2["name_digit"][::7] + 3) % 10
    want = [oracle.schedule(nr if i < 3 else nr2, p, seed=81) for i, p in enumerate(batches)]
    dev = torch.device("cuda:0")
    e = _comm_engine(nr, 0, 81)
    try:
        s = torch.cuda.Stream(device=dev)
        pods = [torch.from_numpy(p.view(np.uint8).copy()).to(dev) for p in batches]
        res = [torch.zeros(len(p) * _lib.RESULT.itemsize, dtype=torch.uint8, device=dev) for p in batches]
        torch.cuda.synchronize()
        for i in range(5):
            if i == 3:  # (batch 2 is stashed here when coalescing: 0+1 shared a launch)
                e.upsert(np.arange(5000), nr2)
                e.flush()
            e.sharded_submit(len(batches[i]), pods[i].data_ptr(), res[i].data_ptr(), s.cuda_stream)
        e.sharded_drain(s.cuda_stream)
        s.synchronize()
        for i in range(5):
            _same(res[i].cpu().numpy().view(_lib.RESULT), want[i], 0, len(batches[i]), f"batch {i}")
    finally:
        e.close()
    if prof:
        assert "MS_HOST_PROF submits=5 " in capfd.readouterr().err


def test_library_schedule_batch_1rank(oracle):
    # ms_schedule_batch on a communicator: every pod's result on every rank (all-gather of
    # the slices), binds committed on the rank's own shard; NU+NN batched and sequential,
    # the resource-aware set batched (one state for the whole call) and exact sequential
    # (the device-cursor windows), the node tables after the binds
    from minisched_amd import _lib

    nr = synth.nodes(4000, seed=71)
    pr = synth.pods(5000, seed=71)
    e = _comm_engine(nr, 0, 71)
    try:
        _same(e.schedule(pr, _lib.MODE_BATCHED), oracle.schedule(nr, pr, seed=71), 0, len(pr), "NU+NN batched")
        _same(e.schedule(pr, _lib.MODE_SEQUENTIAL), oracle.schedule(nr, pr, seed=71), 0, len(pr), "NU+NN seq")
        assert e.read(0, 4000)["pod_count"].sum() == 2 * (oracle.schedule(nr, pr, seed=71)["code"] == 0).sum()
    finally:
        e.close()
    nr = synth.nodes(1000, seed=72, resources=True)
    pr = synth.pods(9000, seed=72, resources=True)
    pr["name_digit"][::23] = -1
    ob = oracle.schedule_batched_commit(nr, pr, 1, seed=72)
    e = _comm_engine(nr, 1, 72)
    try:
        _same(e.schedule(pr, _lib.MODE_BATCHED), ob, 0, len(pr), "NRF batched")
        t = e.read(0, 1000)
        assert np.array_equal(t["pod_count"], ob["cols"].pod_count)
    finally:
        e.close()
    os_ = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=72)
    assert (os_["code"] == 2).sum() > 0  # saturation reached
    e = _comm_engine(nr, 1, 72)
    try:
        _same(e.schedule(pr, _lib.MODE_SEQUENTIAL), os_, 0, len(pr), "NRF sequential")
        t = e.read(0, 1000)
        for k_dev, k_or in (("pod_count", "pod_count"), ("req_milli_cpu", "req_cpu"), ("nonzero_memory", "nz_mem")):
            assert np.array_equal(t[k_dev], getattr(os_["cols"], k_or)), k_dev
    finally:
        e.close()


@pytest.mark.parametrize("window", ["1", "7", "128", "256"])
def test_library_sequential_device_cursor(oracle, monkeypatch, window):
    # ms_schedule_sequential_device on a communicator: windows of W pods issued back to
    # back with the queue cursor on the device (window 1: every pod its own window;
    # windows that stop early at an undecidable pod make the host loop run more rounds)
    import torch

    from minisched_amd import _lib, sharded

    monkeypatch.setenv("MINISCHED_SHARD_SEQ_BATCH", window)
    seed = 80 + int(window)
    nr = synth.nodes(700, seed=seed, resources=True)
    pr = synth.pods(2600, seed=seed, resources=True)
    pr["name_digit"][::31] = -1
    o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=seed)
    dev = torch.device("cuda:0")
    e = _comm_engine(nr, 1, seed)
    try:
        stream = torch.cuda.Stream(device=dev)
        pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
        seq = sharded.ShardedSequential(e, len(pr), pods, stream)
        assert seq.library
        res = seq.run()
        stream.synchronize()
        res = res.cpu().numpy().view(_lib.RESULT)
        t = e.read(0, len(nr))
    finally:
        e.close()
    _same(res, o, 0, len(pr), f"window {window}")
    assert np.array_equal(t["pod_count"], o["cols"].pod_count)


# ---- full-size node-sharded parity: the bench's N > 1 shard shapes ----------
# One context per rank on one GPU: each sweeps ALL pods against its node shard
# (ms_sweep_device, K1 pp) into a key buffer padded to G * ceil(P/G); the
# reduce-scatter (uint64 MAX) is emulated with torch; each rank decodes its own
# pod slice (ms_decode_device, the cluster's present count). Every pod must equal
# the OpenMP oracle over the whole cluster (config C's shard shapes).

def _sharded_c(oracle, n_nodes, n_pods, G, seed=1):
    import torch

    from minisched_amd import _lib, sharded

    nr = synth.nodes(n_nodes, seed=seed)
    pr = synth.pods(n_pods, seed=seed)
    from minisched_amd.hostinfo import cpu_threads

    o = oracle.schedule_nunn_omp(nr, pr, seed=seed, threads=cpu_threads())
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    sp = s.cuda_stream
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    pp = sharded.padded_pods(n_pods, G)
    per = pp // G
    keys = []
    for r in range(G):
        lo, hi = sharded.shard_bounds(n_nodes, r, G)
        with _lib.Engine(max_nodes=hi - lo, node_base=lo, seed=seed) as e:
            e.upsert(np.arange(lo, hi), nr[lo:hi])
            e.flush()
            k = torch.zeros(pp, dtype=torch.int64, device=dev)
            e.sweep_device(n_pods, pods.data_ptr(), k.data_ptr(), 0, sp)
            s.synchronize()
            keys.append(k)
    with torch.cuda.stream(s):
        comb = torch.stack(keys).max(0).values  # the reduce-scatter's MAX, all slices at once
    for r in range(G):
        a, b = sharded.pod_slice(n_pods, r, G)
        lo, hi = sharded.shard_bounds(n_nodes, r, G)
        with _lib.Engine(max_nodes=hi - lo, node_base=lo, seed=seed) as e:
            res = torch.empty(max(1, b - a) * 24, dtype=torch.uint8, device=dev)
            if b > a:
                e.decode_device(b - a, pods.data_ptr() + 40 * a, comb.data_ptr() + 8 * r * per, 0, n_nodes,
                                res.data_ptr(), sp)
            s.synchronize()
            _same(res.cpu().numpy().view(_lib.RESULT)[: b - a], o, a, b, f"G={G} rank {r}")
    k = comb[:n_pods].cpu().numpy().view(np.uint64)
    # no feasible node: key 1 (every shard lists nodes); real keys equal the oracle's
    assert np.array_equal(np.where(k <= 1, 0, k), o["key"]) and np.array_equal(k == 1, o["key"] == 0)


@pytest.mark.parametrize("G", [2, 4, 8])
def test_config_c_node_sharded_full(oracle, G):
    # strong scaling: 100k nodes x 100k pods split over G node shards
    _sharded_c(oracle, 100_000, 100_000, G)


def test_config_c_weak_shard_full(oracle):
    # weak scaling at G = 8: every rank sweeps 800k pods against its 12.5k-row shard
    _sharded_c(oracle, 100_000, 800_000, 8)


def test_config_e_four_contexts_full():
    # config E (50k nodes x 200k pods, exact sequential) over 4 node shards through
    # ms_seq_candidates_device / ms_seq_validate_device, against the committed fixture
    import hashlib

    import torch

    from minisched_amd import _lib, sharded

    here = os.path.dirname(os.path.abspath(__file__))
    fx = np.load(os.path.join(here, "golden", "config_e_full_seed1.npz"))
    N, P, G, B = 50_000, 200_000, 4, 128
    nr = synth.nodes(N, seed=1, resources=True)
    pr = synth.pods(P, seed=1, resources=True)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    sp = s.cuda_stream
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    engines, cuts = [], [sharded.shard_bounds(N, r, G) for r in range(G)]
    for lo, hi in cuts:
        e = _lib.Engine(max_nodes=hi - lo, plugin_set=_lib.PLUGINS_NU_NRF_NN_LA, node_base=lo, seed=1)
        e.upsert(np.arange(lo, hi), nr[lo:hi])
        engines.append(e)
    cb = _lib.SEQ_CAND.itemsize * _lib.SEQ_TOPK
    cands = [torch.zeros(B * cb, dtype=torch.uint8, device=dev) for _ in range(G)]
    flags = [torch.zeros(B, dtype=torch.int32, device=dev) for _ in range(G)]
    res = [torch.zeros(P * 24, dtype=torch.uint8, device=dev) for _ in range(G)]
    done = torch.zeros(G, dtype=torch.int32, device=dev)
    a = 0
    try:
        while a < P:
            nb = min(B, P - a)
            for g, e in enumerate(engines):
                e.seq_candidates_device(nb, pods.data_ptr() + 40 * a, cands[g].data_ptr(), flags[g].data_ptr(), sp)
            with torch.cuda.stream(s):
                call = torch.cat([c[: nb * cb] for c in cands])
                fall = torch.cat([f[:nb] for f in flags])
            for g, e in enumerate(engines):
                e.seq_validate_device(nb, pods.data_ptr() + 40 * a, G, call.data_ptr(), fall.data_ptr(),
                                      res[g].data_ptr() + 24 * a, done.data_ptr() + 4 * g, sp)
            s.synchronize()
            nd = done.cpu().numpy()
            assert (nd == nd[0]).all() and nd[0] >= 1, nd
            a += int(nd[0])
        tables = np.concatenate([e.read(lo, hi - lo) for e, (lo, hi) in zip(engines, cuts)])
    finally:
        for e in engines:
            e.close()
    o = {k: fx[k] for k in ("node", "code", "score", "mask")}
    for g in range(G):
        _same(res[g].cpu().numpy().view(_lib.RESULT), o, 0, P, f"E shard {g}")
    h = hashlib.sha256()
    for k in ("pod_count", "req_milli_cpu", "req_memory", "nonzero_milli_cpu", "nonzero_memory"):
        h.update(np.ascontiguousarray(tables[k], dtype=np.int64).tobytes())
    assert h.hexdigest() == str(fx["table_sha256"])
