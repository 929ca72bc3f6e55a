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
