"""N > 1 bench path on one GPU: two ranks (gloo, both on cuda:0) run
sharded.ShardedCycle exactly as bench.py does — the HIP sweep of each node
shard, the cross-shard MAX combine, the decode — in both the pipelined
(cross-step at depth 1 and 2, with and without its own decode stream) and the in-step chunked
forms, and every rank's decoded results must equal the oracle's over the
whole cluster.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from minisched_amd import synth

pytestmark = pytest.mark.gpu

N_NODES, N_PODS, SEED = 30_000, 5_000, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, pipeline, chunks, dstream, depth, q):
    import torch
    import torch.distributed as dist

    from minisched_amd import _lib, sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lo, hi = sharded.shard_bounds(N_NODES, rank, world)
        eng = _lib.Engine(max_nodes=hi - lo, plugin_set=_lib.PLUGINS_NU_NN, node_base=lo, seed=SEED)
        eng.upsert(np.arange(lo, hi, dtype=np.uint32), synth.nodes(hi - lo, seed=SEED, start=lo))
        eng.flush()
        pods = torch.from_numpy(synth.pods(N_PODS, seed=SEED).view(np.uint8).copy()).to(dev)
        stream = torch.cuda.Stream(device=dev)
        torch.cuda.set_stream(stream)
        cyc = sharded.ShardedCycle(eng, N_NODES, N_PODS, pods, stream, chunks=chunks, pipeline=pipeline,
                                   decode_stream=dstream, depth=depth)
        for _ in range(5):  # both key buffers reused after their decodes
            cyc.step(world)
        cyc.finish()
        torch.cuda.synchronize()
        res = cyc.results.cpu().numpy().view(_lib.RESULT).copy()
        eng.close()
        dist.destroy_process_group()
        q.put((rank, res, None))
    except Exception as e:  # reported to the parent, which fails the test
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("pipeline,chunks,dstream,depth",
                         [(True, 1, False, 1), (True, 1, False, 2), (True, 1, True, 1), (True, 1, True, 2),
                          (False, 3, False, 1)])
def test_two_rank_sharded_cycle_on_gpu(oracle, pipeline, chunks, dstream, depth):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, pipeline, chunks, dstream, depth, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=110) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [e for _, _, e in got if e]
    assert not errs, errs
    o = oracle.schedule(synth.nodes(N_NODES, seed=SEED), synth.pods(N_PODS, seed=SEED), seed=SEED)
    for rank, res, _ in got:
        for k_res, k_or in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
            assert np.array_equal(res[k_res], o[k_or]), f"rank {rank} {k_res}"


def _rccl_worker(port, depth, group, dstream, q):
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
        cyc = sharded.ShardedCycle(eng, N_NODES, N_PODS, pods, stream, pipeline=True, decode_stream=dstream,
                                   depth=depth, drain_group=group)
        ordered = cyc._pipe.ordered
        outs = []
        for k in range(7):  # world > 1 form: RCCL all-reduce per step, grouped drains
            cyc.step(2)
        cyc.finish()
        torch.cuda.synchronize()
        outs.append(cyc.results.cpu().numpy().view(_lib.RESULT).copy())
        eng.close()
        dist.destroy_process_group()
        q.put((ordered, outs, None))
    except Exception as e:
        q.put((None, None, repr(e)))


@pytest.mark.parametrize("depth,group,dstream", [(2, 2, False), (3, 3, False), (2, 2, True)])
def test_rccl_grouped_drain(oracle, depth, group, dstream):
    # the RCCL backend takes the ordered path (one wait per drained group)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), depth, group, dstream, q))
    p.start()
    ordered, outs, err = q.get(timeout=110)
    p.join(timeout=60)
    assert err is None, err
    assert ordered
    o = oracle.schedule(synth.nodes(N_NODES, seed=SEED), synth.pods(N_PODS, seed=SEED), seed=SEED)
    for res in outs:
        for k_res, k_or in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
            assert np.array_equal(res[k_res], o[k_or]), k_res


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
            for k_res, k_or in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
                assert np.array_equal(got[k_res], o[k_or]), f"batch {k} {k_res}"
        with pytest.raises(RuntimeError):
            eng.decode_device_jobs(jobs * 3, n_nodes, stream.cuda_stream)  # > MS_DECODE_MAX_JOBS
    finally:
        eng.close()
