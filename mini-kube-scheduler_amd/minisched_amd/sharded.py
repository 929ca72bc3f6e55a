"""Multi-GPU scheduling cycle, one process per GPU (torch.distributed).

Two partitions of the pods x nodes evaluation:

* split="nodes" (config C, the north star's node sharding). Rank r owns the
  contiguous global ordinals [r*N/G, (r+1)*N/G) in its own context
  (ms_config.node_base) and sweeps the whole pod batch against them; the
  shards then combine with ONE reduce-scatter per batch:

    keys  (int64, element-wise MAX): packed keys embed the global ordinal and
          are never negative (score < 2^11), so the signed max of the int64
          view equals the unsigned max — the winner selectHost
          (minisched.go:304-325) would pick over the union of the shards.
    flags (uint32 per pod, one 0/1 byte per filter plugin) combined as a byte-
          wise uint8 MAX, i.e. the OR of "some node on this shard was rejected
          by plugin X" — FitError's Diagnosis.UnschedulablePlugins
          (minisched.go:130-137) over the whole cluster. Needed only for the
          resource-aware plugin set; NU+NN derives its mask from the key and the
          cluster's present-node count.

  The reduce-scatter leaves rank r the combined keys of its own pod slice
  [r*Pg, (r+1)*Pg) (Pg = ceil(P/G)), so every rank decodes only P/G pods:
  the per-pod fixed costs shrink with G like the sweep does.

* split="pods" (config D, pod-split replicas). Every rank holds the whole node
  table (it is 100 KB at config C) and runs the fused single-shard cycle on
  its own pod slice: no collective at all. Pods are independent in the
  stateless batched mode (minisched.go:32-85 schedules each pod alone and the
  NU/NN state they read is not changed by binds).

On GPUs the collectives run INSIDE the library (ms_comm.cpp): every rank's
context joins one RCCL communicator (init_comm: rank 0 creates the id, one
torch.distributed broadcast ships its bytes) and ms_sharded_submit /
ms_sharded_drain do the sweep, the grouped reduce-scatter and the decode —
the path a Go scheduleOne binds through cgo. The Python combine below
(combine_scatter_ over torch.distributed) remains for gloo rehearsals of the
protocol (several ranks on one GPU, which RCCL refuses) and the CPU tests.
"""
from __future__ import annotations

from typing import Optional, Tuple


def shard_bounds(n_nodes: int, rank: int, world: int) -> Tuple[int, int]:
    """[lo, hi) of global node ordinals owned by `rank` (sizes differ by <= 1)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    return rank * n_nodes // world, (rank + 1) * n_nodes // world


def pod_slice(n_pods: int, rank: int, world: int) -> Tuple[int, int]:
    """[a, b) of the pods rank decodes after the reduce-scatter (equal slices of
    ceil(P/G), the last one short; the key buffers are padded to G * ceil(P/G))."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    per = (n_pods + world - 1) // world
    return min(n_pods, rank * per), min(n_pods, (rank + 1) * per)


def padded_pods(n_pods: int, world: int) -> int:
    return ((n_pods + world - 1) // world) * world


def _backend(group=None) -> Optional[str]:
    import torch.distributed as dist

    try:
        return dist.get_backend(group) if dist.is_initialized() else None
    except Exception:
        return None


FLAGS_BYTES = "bytes"  # resource-aware set: one 0/1 byte per filter plugin -> byte-wise uint8 MAX (OR)
FLAGS_U32 = "u32"      # NodeAffinity set: per-pod normalise anchor (< 2^21) -> element-wise 32-bit MAX


def flags_op_for(plugin_set: int) -> Optional[str]:
    """How shards combine ms_sweep_device's flags for a plugin set (minisched_gpu.h)."""
    from . import _lib

    return {_lib.PLUGINS_NU_NN: None, _lib.PLUGINS_NU_NRF_NN_LA: FLAGS_BYTES,
            _lib.PLUGINS_NU_NN_NA: FLAGS_U32, _lib.PLUGINS_NU_TT_NN: None}[plugin_set]


def combine_scatter_(keys, keys_out, flags=None, flags_out=None, group=None, async_op=False, flags_op=FLAGS_BYTES):
    """Cross-shard combine of one batch: keys (int64[G*Pg], this shard's maxima)
    -> keys_out (int64[Pg], the cluster's maxima of this rank's pod slice);
    flags as a byte-wise MAX (flags_op "bytes", the resource-aware filter
    bytes) or an element-wise MAX of 32-bit values ("u32", the NodeAffinity
    anchors: a byte-wise MAX would mix bytes of different shards' anchors).
    With async_op=True returns the pending works: the collectives run on the
    backend's stream after the work already queued on the current stream.

    gloo cannot reduce-scatter device tensors; there (CPU-only tests of the GPU
    path) it all-reduces and copies the slice — the same values."""
    import torch
    import torch.distributed as dist

    if keys.dtype != torch.int64:
        raise TypeError("keys must be an int64 view of the uint64 packed keys")
    if flags_op not in (FLAGS_BYTES, FLAGS_U32):
        raise ValueError("flags_op must be 'bytes' or 'u32'")
    if flags is not None and flags.dtype not in (torch.int32, torch.uint32):
        raise TypeError("flags must be 32-bit")
    world = dist.get_world_size(group)
    if keys.numel() != keys_out.numel() * world:
        raise ValueError("keys must hold world * len(keys_out) entries (padded pod count)")

    def fview(t):  # anchors < 2^21: the signed int32 MAX equals the unsigned one
        return t.view(torch.uint8) if flags_op == FLAGS_BYTES else t.view(torch.int32)

    if _backend(group) == "gloo" and keys.is_cuda:
        rank = dist.get_rank(group)
        n = keys_out.numel()
        dist.all_reduce(keys, op=dist.ReduceOp.MAX, group=group)
        keys_out.copy_(keys[rank * n:(rank + 1) * n])
        if flags is not None:
            dist.all_reduce(fview(flags), op=dist.ReduceOp.MAX, group=group)
            flags_out.copy_(flags[rank * n:(rank + 1) * n])
        return [] if async_op else (keys_out, flags_out)
    work = [dist.reduce_scatter_tensor(keys_out, keys, op=dist.ReduceOp.MAX, group=group, async_op=True)]
    if flags is not None:
        work.append(dist.reduce_scatter_tensor(fview(flags_out), fview(flags), op=dist.ReduceOp.MAX, group=group,
                                               async_op=True))
    if async_op:
        return work
    for w in work:
        w.wait()
    return keys_out, flags_out


class CrossStepPipeline:
    """Overlaps batch k's cross-shard combine with the following batches' sweeps.

    depth + 1 key buffers rotate between batches. step(batch) sweeps the batch
    into its buffer, starts the async combine of that buffer, then, once
    `depth` combines are in flight, drains the oldest `group` of them (wait,
    then decode). finish() drains the rest. Buffer b is swept again only
    depth + 1 batches later, after its decode (stream order).

    With ordered=True (RCCL: one stream per communicator runs the collectives
    in issue order) only the newest drained batch's combine is waited for, so
    the sweep stream pays one cross-queue wait per `group` steps (each costs
    ~10 us of idle device time however early its event completed).

    sweep(buf, batch), decode(buf, batch): enqueue work; combine(buf) -> list
    of async works (torch.distributed) whose wait() orders the caller's stream.
    """

    def __init__(self, sweep, combine, decode, depth: int = 1, nbuf: int = 0, group: int = 1,
                 ordered: bool = False, decode_many=None):
        if depth < 1 or (nbuf and nbuf < depth + 1) or not 1 <= group <= depth:
            raise ValueError("need depth >= 1, nbuf >= depth + 1, 1 <= group <= depth")
        self._sweep, self._combine, self._decode = sweep, combine, decode
        self.depth = depth
        self.nbuf = nbuf or depth + 1
        self.group = group
        self.ordered = ordered
        # decode_many([(buf, batch), ...]): the drained batches' decodes in one launch
        self._decode_many = decode_many
        self._n = 0
        self._pending = []  # [(works, buf, batch)], oldest first

    def step(self, batch=None):
        buf = self._n % self.nbuf
        self._n += 1
        self._sweep(buf, batch)
        self._pending.append((self._combine(buf), buf, batch))
        if len(self._pending) > self.depth:
            self._drain_n(min(self.group, len(self._pending)))

    def _drain_n(self, n):
        batch_list, self._pending = self._pending[:n], self._pending[n:]
        for i, (works, _buf, _batch) in enumerate(batch_list):
            if not self.ordered or i == n - 1:
                for w in works:
                    w.wait()
        if self._decode_many is not None and len(batch_list) > 1:
            self._decode_many([(buf, batch) for _works, buf, batch in batch_list])
            return
        for _works, buf, batch in batch_list:
            self._decode(buf, batch)

    def finish(self):
        if self._pending:
            self._drain_n(len(self._pending))


def init_comm(engine, group=None) -> None:
    """Joins `engine` (this rank's node shard) to the job's in-library RCCL
    communicator: rank 0 creates the id (ms_comm_id_create), one broadcast over
    the torch.distributed group ships its 128 bytes, every rank calls
    ms_comm_init (collective). Without an initialised process group: a 1-rank
    communicator."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from . import _lib

    if not dist.is_initialized():
        engine.comm_init(_lib.comm_id_create(), 0, 1)
        return
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if _backend(group) == "nccl" else torch.device("cpu")
    t = torch.zeros(_lib.COMM_ID_BYTES, dtype=torch.uint8, device=dev)
    if rank == 0:
        t.copy_(torch.from_numpy(np.frombuffer(_lib.comm_id_create(), dtype=np.uint8).copy()))
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast(t, src=src, group=group)
    engine.comm_init(t.cpu().numpy().tobytes(), rank, world)


def _has_comm(engine) -> bool:
    return int(engine.info().comm_world) >= 1  # (0: not joined)


class ShardedCycle:
    """One rank's engine + device buffers for a fixed pod batch (bench / service loop).

    split="nodes", engine joined to a communicator (init_comm): step() =
    ms_sharded_submit — this shard's sweep, the in-library grouped RCCL
    reduce-scatter, the decode of this rank's pod slice, pipelined in the
    library (depth 4); finish() = ms_sharded_drain.
    split="nodes", world > 1 without a communicator (gloo rehearsals): the same
    protocol with the combine over torch.distributed (combine_scatter_,
    CrossStepPipeline).
    split="pods", or world == 1: step() = the fused single-shard cycle
    (ms_select_batch_device) of this rank's pod slice; no collective.

    Every call runs under `with torch.cuda.stream(stream)`, so torch-side
    collectives and copies order after the sweeps on that stream.
    results: decoded ms_result bytes of this rank's pod slice [a, b) of the
    most recent batch (valid once its stream work is done).
    """

    POD_BYTES = 40
    RESULT_BYTES = 24

    def __init__(self, engine, n_nodes_global: int, n_pods: int, pods_dev, stream, split: str = "nodes",
                 want_flags: Optional[bool] = None, group=None, depth: int = 4, drain_group: int = 4,
                 rank: int = 0, world: int = 1, present_total: Optional[int] = None,
                 collective: Optional[bool] = None, library: Optional[bool] = None):
        import torch

        if split not in ("nodes", "pods"):
            raise ValueError("split must be 'nodes' or 'pods'")
        self.eng = engine
        self.N = n_nodes_global
        self.P = n_pods
        self.pods = pods_dev
        self.stream = stream
        self.group = group
        self.split = split
        self.rank, self.world = rank, world
        self.present = n_nodes_global if present_total is None else present_total
        dev = pods_dev.device
        self._pipe = None
        self._flags_op = flags_op_for(engine.plugin_set)
        if want_flags is None:
            want_flags = self._flags_op is not None
        if want_flags and self._flags_op is None:
            raise ValueError("NU+NN keys carry the whole outcome: no flags to combine")
        if not want_flags and self._flags_op is not None:
            raise ValueError("this plugin set needs its flags combined (filter bytes / NodeAffinity anchors)")
        # in-library node-sharded cycle when the engine has a communicator
        self._library = (split == "nodes" and _has_comm(engine)) if library is None else library
        from . import _lib

        if (engine.plugin_set == _lib.PLUGINS_NU_TT_NN and split == "nodes" and world > 1
                and not self._library):
            raise ValueError("TaintToleration node shards combine by summaries: join a communicator "
                             "(init_comm) or use ms_tt_summaries_device / ms_tt_decode_device")
        if self._library:
            self.a, n_mine = engine.sharded_slice(n_pods)
            self.b = self.a + n_mine
            self._collective = True
            self._results = [torch.empty(max(1, n_mine) * self.RESULT_BYTES, dtype=torch.uint8, device=dev)]
            self._last = 0
            # the step is one C call with fixed arguments: no torch stream context, no
            # per-step pointer lookups (host enqueue time bounds the pipelined step at
            # small shards)
            self._submit_args = (engine.h, n_pods, pods_dev.data_ptr(), self._results[0].data_ptr(),
                                 stream.cuda_stream)
            return
        self.a, self.b = pod_slice(n_pods, rank, world)
        # collective=True forces the Python node-split pipeline at world 1 (a 1-rank
        # torch group on one GPU rehearses the reduce-scatter path)
        self._collective = (split == "nodes" and world > 1) if collective is None else collective
        nbuf = depth + 1 if self._collective else 1
        n_mine = max(1, self.b - self.a)
        self._results = [torch.empty(n_mine * self.RESULT_BYTES, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
        self._last = 0
        if not self._collective:
            return
        pp = padded_pods(n_pods, world)
        per = pp // world
        # pad entries past P stay 0 (no feasible node) in every shard's buffer
        self._keys = [torch.zeros(pp, dtype=torch.int64, device=dev) for _ in range(nbuf)]
        self._keys_mine = [torch.zeros(per, dtype=torch.int64, device=dev) for _ in range(nbuf)]
        self._flags = ([torch.zeros(pp, dtype=torch.int32, device=dev) for _ in range(nbuf)]
                       if want_flags else [None] * nbuf)
        self._flags_mine = ([torch.zeros(per, dtype=torch.int32, device=dev) for _ in range(nbuf)]
                            if want_flags else [None] * nbuf)
        self._pipe = CrossStepPipeline(
            self._sweep_buf,
            lambda buf: combine_scatter_(self._keys[buf], self._keys_mine[buf], self._flags[buf],
                                         self._flags_mine[buf], self.group, async_op=True,
                                         flags_op=self._flags_op or FLAGS_BYTES),
            lambda buf, _b: self._decode_buf(buf), depth=depth, nbuf=nbuf, group=drain_group,
            ordered=_backend(group) == "nccl", decode_many=self._decode_many)

    @property
    def library(self) -> bool:
        """True when step() runs the in-library RCCL path."""
        return self._library

    # ---- node-sharded pieces (Python combine) ---------------------------------
    def _sweep_buf(self, buf, _batch=None):
        flags = self._flags[buf].data_ptr() if self._flags[buf] is not None else 0
        self.eng.sweep_device(self.P, self.pods.data_ptr(), self._keys[buf].data_ptr(), flags, self.stream.cuda_stream)

    def sweep(self, buf=0):
        """This shard's keys for all P pods into key buffer `buf` (no combine)."""
        import torch

        if self._library:
            raise RuntimeError("the in-library path sweeps inside ms_sharded_submit")
        with torch.cuda.stream(self.stream):
            self._sweep_buf(buf)

    def _job(self, buf):
        n = self.b - self.a
        pods = self.pods.data_ptr() + self.a * self.POD_BYTES
        flags = self._flags_mine[buf].data_ptr() if self._flags_mine[buf] is not None else 0
        return (n, pods, self._keys_mine[buf].data_ptr(), flags, self._results[buf].data_ptr())

    def _decode_buf(self, buf):
        self._last = buf
        n, pods, keys, flags, res = self._job(buf)
        if n:
            self.eng.decode_device(n, pods, keys, flags, self.present, res, self.stream.cuda_stream)

    def _decode_many(self, bufs):
        from . import _lib

        jobs = [self._job(buf) for buf, _batch in bufs]
        jobs = [j for j in jobs if j[0]]
        if self.eng.plugin_set == _lib.PLUGINS_NU_NN_NA:  # (ms_decode_device_jobs: one launch per job)
            for j in jobs:
                self.eng.decode_device(j[0], j[1], j[2], j[3], self.present, j[4], self.stream.cuda_stream)
        else:
            for i in range(0, len(jobs), _lib.DECODE_MAX_JOBS):
                self.eng.decode_device_jobs(jobs[i:i + _lib.DECODE_MAX_JOBS], self.present, self.stream.cuda_stream)
        self._last = bufs[-1][0]

    # ---- the cycle ------------------------------------------------------------
    @property
    def results(self):
        return self._results[self._last]

    @property
    def keys(self):
        """This rank's padded key buffer of the most recent sweep (Python node split)."""
        return self._keys[self._last] if (self._collective and not self._library) else None

    def step(self):
        import torch

        if self._library:
            rc = self.eng.lib.ms_sharded_submit(*self._submit_args)
            if rc:
                self.eng._check("ms_sharded_submit", rc)
            return
        with torch.cuda.stream(self.stream):
            if self._pipe is not None:
                self._pipe.step()
                return
            n = self.b - self.a
            if n:
                self.eng.select_batch_device(n, self.pods.data_ptr() + self.a * self.POD_BYTES,
                                             self._results[0].data_ptr(), self.stream.cuda_stream)

    def finish(self):
        """Drains a pipelined step's pending combines + decodes (no-op otherwise)."""
        import torch

        with torch.cuda.stream(self.stream):
            if self._library:
                self.eng.sharded_drain(self.stream.cuda_stream)
            elif self._pipe is not None:
                self._pipe.finish()


class ShardedSequential:
    """Node-sharded exact sequential cycle (config E over G GPUs).

    Engine joined to a communicator (init_comm): run() is ONE library call,
    ms_schedule_sequential_device — per window of pods, every shard's
    speculative top-4 with records, an in-library RCCL all-gather, the
    replicated in-order validation, with the queue cursor on the device (no
    host round trip per batch).

    Without one (gloo rehearsals, 1-rank torch groups), the same protocol over
    torch.distributed, batch by batch:
      1. ms_seq_candidates_device: this shard's speculative top-4 per pod with
         the nodes' records, and its filter flags;
      2. all-gather of both over the ranks (two collectives);
      3. ms_seq_validate_device, the same on every rank: the merged global
         top-4 walked in queue order (nodes bound earlier in the batch are
         re-evaluated from their records), up to the first pod the lists
         cannot decide; each rank commits the binds on its own nodes only.
    The next batch starts at a + n_done (n_done >= 1; a host read per batch).
    Every rank ends with every pod's result.
    """

    def __init__(self, engine, n_pods: int, pods_dev, stream, group=None, batch: int = 128,
                 library: Optional[bool] = None):
        import torch
        import torch.distributed as dist

        from . import _lib

        self.eng, self.P, self.pods, self.stream, self.group = engine, n_pods, pods_dev, stream, group
        self.library = _has_comm(engine) if library is None else library
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if self.world > _lib.SEQ_MAX_SHARDS:
            raise ValueError("too many shards for the replicated validator")
        self.B = max(1, min(batch, _lib.SEQ_SHARD_BATCH_MAX))
        dev = pods_dev.device
        cb = _lib.SEQ_CAND.itemsize * _lib.SEQ_TOPK
        self.results = torch.zeros(n_pods * 24, dtype=torch.uint8, device=dev)
        self.batches = 0
        if self.library:
            return
        self._cands = torch.zeros(self.B * cb, dtype=torch.uint8, device=dev)
        self._flags = torch.zeros(self.B, dtype=torch.int32, device=dev)
        self._cands_all = torch.zeros(self.world * self.B * cb, dtype=torch.uint8, device=dev)
        self._flags_all = torch.zeros(self.world * self.B, dtype=torch.int32, device=dev)
        self._n_done = torch.zeros(1, dtype=torch.int32, device=dev)

    def _gather(self, nb):
        import torch.distributed as dist

        from . import _lib

        cb = _lib.SEQ_CAND.itemsize * _lib.SEQ_TOPK
        if self.world == 1:
            self._cands_all[: nb * cb].copy_(self._cands[: nb * cb])
            self._flags_all[:nb].copy_(self._flags[:nb])
            return
        # shard-major [s][p]: gather the first nb pods' entries of every rank
        dist.all_gather_into_tensor(self._cands_all[: self.world * nb * cb], self._cands[: nb * cb].contiguous(),
                                    group=self.group)
        dist.all_gather_into_tensor(self._flags_all[: self.world * nb], self._flags[:nb].contiguous(),
                                    group=self.group)

    def run(self):
        import torch

        sp = self.stream.cuda_stream
        with torch.cuda.stream(self.stream):
            if self.library:
                self.eng.schedule_sequential_device(self.P, self.pods.data_ptr(), self.results.data_ptr(), sp)
                return self.results
            a = 0
            while a < self.P:
                nb = min(self.B, self.P - a)
                pods = self.pods.data_ptr() + 40 * a
                self.eng.seq_candidates_device(nb, pods, self._cands.data_ptr(), self._flags.data_ptr(), sp)
                self._gather(nb)
                self.eng.seq_validate_device(nb, pods, self.world, self._cands_all.data_ptr(),
                                             self._flags_all.data_ptr(), self.results.data_ptr() + 24 * a,
                                             self._n_done.data_ptr(), sp)
                done = int(self._n_done.item())  # (syncs the current stream, self.stream)
                if done < 1:
                    raise RuntimeError("replicated validator made no progress")
                a += done
                self.batches += 1
        return self.results


def present_total(engine, group=None) -> int:
    """Present nodes over every shard (decode's FitError mask for NU+NN needs the
    cluster's count, not this shard's): one all-reduce at setup / after deltas."""
    import torch
    import torch.distributed as dist

    n = int(engine.info().present_nodes)
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return n
    dev = "cuda" if _backend(group) == "nccl" else "cpu"
    t = torch.tensor([n], dtype=torch.int64, device=dev)
    dist.all_reduce(t, group=group)
    return int(t.item())
