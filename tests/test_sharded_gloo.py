"""N > 1 path on CPU: node-sharded shards combined over torch.distributed (gloo).

Each rank evaluates its own node shard with the oracle (standing in for the
HIP sweep, which needs a GPU), then the product's combine_scatter_
reduce-scatters the packed keys and filter flags (MAX); every rank must end
with exactly the keys and FitError masks of the single-process run over the
whole cluster for its own pod slice. The pod-split partition (replicas, no
collective) is checked the same way.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from minisched_amd import sharded, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _decode_mask(keys, flags):
    return np.where(keys == 0, (flags & 0xFF != 0) * 1 | ((flags >> 8) & 0xFF != 0) * 2, 0)


def _worker(rank, world, port, n_nodes, n_pods, plugin_set, q, chunks=1):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "mini-kube-scheduler_amd"))
    import _oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = plugin_set == 1
    nr = synth.nodes(n_nodes, seed=11, resources=res)
    pr = synth.pods(n_pods, seed=11, resources=res)
    if res:
        nr["req_milli_cpu"] = nr["alloc_milli_cpu"] * 3 // 4  # make NRF bite
        nr["pod_count"][::5] = 110
    lo, hi = sharded.shard_bounds(n_nodes, rank, world)
    o = _oracle.schedule(nr[lo:hi], pr, plugin_set=plugin_set, seed=11, node_base=lo)
    pp = sharded.padded_pods(n_pods, world)
    keys = torch.zeros(pp, dtype=torch.int64)
    keys[:n_pods] = torch.from_numpy(o["key"].view(np.int64).copy())
    # per-shard flags: a shard with no feasible node reports its own FitError mask
    m = o["mask"].astype(np.uint32)
    flags = torch.zeros(pp, dtype=torch.int32)
    flags[:n_pods] = torch.from_numpy(((m & 1) | ((m >> 1) & 1) << 8).astype(np.int32))
    kout = torch.zeros(pp // world, dtype=torch.int64)
    fout = torch.zeros(pp // world, dtype=torch.int32)
    if chunks == 1:
        sharded.combine_scatter_(keys, kout, flags if plugin_set == 1 else None, fout if plugin_set == 1 else None)
    else:  # async form used by the pipelined step: wait later
        works = sharded.combine_scatter_(keys, kout, flags if plugin_set == 1 else None,
                                         fout if plugin_set == 1 else None, async_op=True)
        for w in works:
            w.wait()
    a, b = sharded.pod_slice(n_pods, rank, world)
    q.put((rank, a, b, kout.numpy().view(np.uint64)[: b - a].copy(), fout.numpy().astype(np.uint32)[: b - a].copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 1), (2, 3)])
@pytest.mark.parametrize("plugin_set", [0, 1])
def test_node_sharded_reduce_scatter_gloo(oracle, world, chunks, plugin_set):
    n_nodes, n_pods = 997, 300
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [
        ctx.Process(target=_worker, args=(r, world, port, n_nodes, n_pods, plugin_set, q, chunks))
        for r in range(world)
    ]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = plugin_set == 1
    nr = synth.nodes(n_nodes, seed=11, resources=res)
    pr = synth.pods(n_pods, seed=11, resources=res)
    if res:
        nr["req_milli_cpu"] = nr["alloc_milli_cpu"] * 3 // 4
        nr["pod_count"][::5] = 110
    full = oracle.schedule(nr, pr, plugin_set=plugin_set, seed=11)
    covered = np.zeros(n_pods, dtype=bool)
    for rank, a, b, keys, flags in got:
        assert np.array_equal(keys, full["key"][a:b]), f"rank {rank}"
        covered[a:b] = True
        if plugin_set == 1:
            assert np.array_equal(_decode_mask(keys, flags), full["mask"][a:b]), f"rank {rank}"
        # decoded winners: the global ordinal sits in the low 20 bits of the key
        won = full["code"][a:b] == 0
        assert np.array_equal((0xFFFFF - (keys[won] & 0xFFFFF)).astype(np.int64),
                              full["node"][a:b][won].astype(np.int64))
        assert np.array_equal((keys[won] >> 52).astype(np.int64), full["score"][a:b][won])
    assert covered.all()


def _podsplit_worker(rank, world, port, n_nodes, n_pods, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import _oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nr = synth.nodes(n_nodes, seed=13)  # every rank holds the whole table (replica)
    pr = synth.pods(n_pods, seed=13)
    a, b = sharded.pod_slice(n_pods, rank, world)
    o = _oracle.schedule(nr, pr[a:b], seed=13)  # stands in for ms_select_batch_device on the slice
    # gather the slices to rank 0 the way a caller would (not part of the step: no collective there)
    parts = [None] * world
    dist.all_gather_object(parts, (a, b, o["key"].copy()))
    q.put((rank, parts))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_pod_split_replicas_gloo(oracle, world):
    # config D's pod split: replicated nodes, disjoint pod slices, no combine; the union of
    # the slices equals the single-process run (the tie-break hash depends on the pod's
    # ordinal, not its position in the batch)
    n_nodes, n_pods = 1200, 401
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_podsplit_worker, args=(r, world, port, n_nodes, n_pods, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = oracle.schedule(synth.nodes(n_nodes, seed=13), synth.pods(n_pods, seed=13), seed=13)
    for rank, parts in got:
        keys = np.concatenate([k for _a, _b, k in sorted(parts, key=lambda t: t[0])])
        assert np.array_equal(keys, full["key"]), f"rank {rank}"


def test_pod_slices_cover_everything():
    for n in (0, 1, 7, 100_000, 1_000_000):
        for w in (1, 2, 3, 8):
            spans = [sharded.pod_slice(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            per = (n + w - 1) // w
            assert all(b - a <= per for a, b in spans)
            assert sharded.padded_pods(n, w) == per * w


def test_shard_bounds_cover_everything():
    for n in (0, 1, 7, 100_000):
        for w in (1, 2, 3, 8):
            spans = [sharded.shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
    with pytest.raises(ValueError):
        sharded.shard_bounds(10, 3, 3)


def _pipe_worker(rank, world, port, n_nodes, batches, depth, group, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "mini-kube-scheduler_amd"))
    import _oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nr = synth.nodes(n_nodes, seed=21)
    lo, hi = sharded.shard_bounds(n_nodes, rank, world)
    pp = sharded.padded_pods(max(batches), world)
    keys = [torch.zeros(pp, dtype=torch.int64) for _ in range(depth + 1)]
    mine = [torch.zeros(pp // world, dtype=torch.int64) for _ in range(depth + 1)]
    out = {}

    def sweep(buf, k):  # this rank's shard of batch k (the oracle stands in for the HIP sweep)
        pr = synth.pods(batches[k], seed=100 + k)
        o = _oracle.schedule(nr[lo:hi], pr, seed=21, node_base=lo)
        keys[buf].zero_()
        keys[buf][: batches[k]] = torch.from_numpy(o["key"].view(np.int64).copy())

    def combine(buf):
        return sharded.combine_scatter_(keys[buf], mine[buf], async_op=True)

    def decode(buf, k):
        a, b = sharded.pod_slice(pp, rank, world)
        out[k] = (a, mine[buf].numpy().view(np.uint64).copy())

    pipe = sharded.CrossStepPipeline(sweep, combine, decode, depth=depth, group=group)
    for k in range(len(batches)):
        pipe.step(k)
        assert len(out) == k + 1 - len(pipe._pending)  # decoded in order, at most `depth` in flight
        assert len(pipe._pending) <= depth
    pipe.finish()
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("depth,group", [(1, 1), (2, 1), (2, 2), (3, 3)])
def test_cross_step_pipeline_gloo(oracle, depth, group):
    # bench.py's N > 1 step: batch k's all-reduce overlaps the next `depth` sweeps,
    # depth + 1 key buffers rotate; every batch must decode to the single-process result
    world, n_nodes, batches = 2, 1500, [256, 200, 256, 131, 256]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, n_nodes, batches, depth, group, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nr = synth.nodes(n_nodes, seed=21)
    for k, n in enumerate(batches):
        full = oracle.schedule(nr, synth.pods(n, seed=100 + k), seed=21)
        ref = np.zeros(sharded.padded_pods(max(batches), world), dtype=np.uint64)
        ref[:n] = full["key"]
        for rank, out in got:
            a, keys = out[k]
            assert np.array_equal(keys, ref[a:a + len(keys)]), f"rank {rank} batch {k}"


def _seqshard_worker(rank, world, port, n_nodes, n_pods, batch, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import _seq_shard_ref as ref

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nr = synth.nodes(n_nodes, seed=31, resources=True)
    pr = synth.pods(n_pods, seed=31, resources=True)
    pr["name_digit"][::23] = -1
    lo, hi = sharded.shard_bounds(n_nodes, rank, world)
    shard = ref.Shard(nr[lo:hi], lo)
    results, a, batches = [], 0, 0
    while a < n_pods:
        nb = min(batch, n_pods - a)
        c, f = shard.candidates(pr[a:a + nb], seed=31)
        call = torch.zeros((world,) + c.shape, dtype=torch.int64)
        fall = torch.zeros((world, nb), dtype=torch.int64)
        dist.all_gather_into_tensor(call, torch.from_numpy(c).unsqueeze(0))  # shard-major, like the GPU path
        dist.all_gather_into_tensor(fall, torch.from_numpy(f).unsqueeze(0))
        done, out, live = ref.validate(pr[a:a + nb], call.numpy(), fall.numpy(), seed=31)
        assert done >= 1
        results += out
        for o, rec in live.items():  # every bind reaches its owner and no other shard
            shard.commit(o, (rec[3], rec[4], rec[5], rec[6], rec[8]))
        a += done
        batches += 1
    q.put((rank, results, batches, shard.cnt.copy(), shard.req_cpu.copy(), shard.nz_mem.copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_nodes,n_pods,batch", [(2, 60, 700, 64), (3, 200, 1200, 128), (2, 7, 300, 16)])
def test_node_sharded_sequential_protocol_gloo(oracle, world, n_nodes, n_pods, batch):
    # config E over node shards: per-shard top-4 + records, all-gather,
    # replicated in-order validation with truncation, binds to their owner only. Every
    # rank's results and the shards' tables after the binds equal the 1-process oracle.
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seqshard_worker, args=(r, world, port, n_nodes, n_pods, batch, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nr = synth.nodes(n_nodes, seed=31, resources=True)
    pr = synth.pods(n_pods, seed=31, resources=True)
    pr["name_digit"][::23] = -1
    o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=31)
    assert (o["code"] == 2).sum() > 0  # saturated: FitErrors and re-evaluations happen
    for rank, results, batches, *_ in got:
        codes = np.array([r[0] for r in results])
        nodes = np.array([r[1] for r in results])
        scores = np.array([r[2] for r in results])
        masks = np.array([r[3] for r in results])
        assert np.array_equal(codes, o["code"]), rank
        assert np.array_equal(nodes, o["node"]), rank
        assert np.array_equal(scores, o["score"]), rank
        assert np.array_equal(masks, o["mask"]), rank
        assert batches >= (n_pods + batch - 1) // batch
    cols = o["cols"]
    cnt = np.concatenate([g[3] for g in got])
    req = np.concatenate([g[4] for g in got])
    nzm = np.concatenate([g[5] for g in got])
    assert np.array_equal(cnt, cols.pod_count) and np.array_equal(req, cols.req_cpu) and np.array_equal(nzm, cols.nz_mem)


def _na_anchors(nr, pr, lo, hi):
    """NodeAffinity normalise anchors of the shard [lo, hi) (minisched_gpu.h
    ms_sweep_device, MS_PLUGINS_NU_NN_NA): per pod, over the shard's feasible nodes
    with a non-zero raw NodeAffinity score, max of ((0xFFFFF - ordinal) << 1 | NN
    match) + 1 — the first such node in LIST order; 0 = none."""
    out = np.zeros(len(pr), dtype=np.uint32)
    ords = np.arange(lo, hi)
    for j in range(len(pr)):
        p = pr[j]
        feas = (nr["unschedulable"][lo:hi] == 0) | (p["tolerates_unschedulable"] != 0)
        hit = feas & (p["pref_zone"] != 0) & (nr["zone"][lo:hi] == p["pref_zone"])
        if hit.any():
            i = int(np.argmax(hit))
            nn = int(nr["name_digit"][lo + i] == p["name_digit"])
            out[j] = (((0xFFFFF - int(ords[i])) << 1) | nn) + 1
    return out


def _na_worker(rank, world, port, n_nodes, n_pods, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nr = synth.nodes(n_nodes, seed=21, zones=True)
    pr = synth.pods(n_pods, seed=21, zones=True)
    lo, hi = sharded.shard_bounds(n_nodes, rank, world)
    pp = sharded.padded_pods(n_pods, world)
    flags = torch.zeros(pp, dtype=torch.int32)
    flags[:n_pods] = torch.from_numpy(_na_anchors(nr, pr, lo, hi).astype(np.int32))
    keys = torch.zeros(pp, dtype=torch.int64)
    kout = torch.zeros(pp // world, dtype=torch.int64)
    fout = torch.zeros(pp // world, dtype=torch.int32)
    sharded.combine_scatter_(keys, kout, flags, fout, flags_op=sharded.FLAGS_U32)
    a, b = sharded.pod_slice(n_pods, rank, world)
    q.put((rank, a, b, fout.numpy().astype(np.uint32)[: b - a].copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_na_anchor_combine_gloo(world):
    # NodeAffinity anchors combine with an element-wise 32-bit MAX;
    # a byte-wise MAX mixes bytes of different shards' anchors
    n_nodes, n_pods = 600, 200
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_na_worker, args=(r, world, port, n_nodes, n_pods, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nr = synth.nodes(n_nodes, seed=21, zones=True)
    pr = synth.pods(n_pods, seed=21, zones=True)
    full = _na_anchors(nr, pr, 0, n_nodes)
    for rank, a, b, fl in got:
        assert np.array_equal(fl, full[a:b]), f"rank {rank}"
    # the byte-wise form really differs on these inputs
    per_shard = [_na_anchors(nr, pr, *sharded.shard_bounds(n_nodes, r, world)) for r in range(world)]
    bytewise = np.max(np.stack([s.view(np.uint8).reshape(-1, 4) for s in per_shard]), 0).copy().view(np.uint32)[:, 0]
    assert (bytewise != full).any()


def test_flags_op_per_plugin_set():
    from minisched_amd import _lib

    assert sharded.flags_op_for(_lib.PLUGINS_NU_NN) is None
    assert sharded.flags_op_for(_lib.PLUGINS_NU_NRF_NN_LA) == sharded.FLAGS_BYTES
    assert sharded.flags_op_for(_lib.PLUGINS_NU_NN_NA) == sharded.FLAGS_U32
