"""Node-sharded multi-GPU scheduling cycle (one process per GPU).

Rank r owns the contiguous global ordinals [r*N/G, (r+1)*N/G) in its own
context (ms_config.node_base), sweeps the whole pod batch against them, and
the ranks combine with ONE all-reduce per batch:

  keys  (int64, element-wise MAX): packed keys embed the global ordinal and
        are never negative (score < 2^11), so the signed max of the int64
        view equals the unsigned max — the same winner selectHost
        (minisched.go:304-325) would pick over the union of the shards.
  flags (uint32 per pod, one 0/1 byte per filter plugin) combined as a byte-
        wise uint8 MAX, i.e. the OR of "some node on this shard was rejected
        by plugin X" — FitError's Diagnosis.UnschedulablePlugins
        (minisched.go:130-137) over the whole cluster. Needed only for the
        resource-aware plugin set; NU+NN derives its mask from the key.

On GPUs the collective is RCCL (torch.distributed "nccl") over xGMI; the same
code runs on CPU tensors with gloo for the tests.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple


def shard_bounds(n_nodes: int, rank: int, world: int) -> Tuple[int, int]:
    """[lo, hi) of global node ordinals owned by `rank` (sizes differ by <= 1)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    return rank * n_nodes // world, (rank + 1) * n_nodes // world


def combine_(keys, flags=None, group=None, async_op=False):
    """In-place cross-shard combine of one batch (keys int64[P], flags uint32[P]).

    With async_op=True returns the pending works: the collectives run on the
    backend's stream after the work already queued on the current stream, so
    the caller can keep sweeping the next chunk and wait() before decoding.
    """
    import torch
    import torch.distributed as dist

    if keys.dtype != torch.int64:
        raise TypeError("keys must be an int64 view of the uint64 packed keys")
    work = [dist.all_reduce(keys, op=dist.ReduceOp.MAX, group=group, async_op=True)]
    if flags is not None:
        if flags.dtype not in (torch.int32, torch.uint32):
            raise TypeError("flags must be 32-bit")
        work.append(dist.all_reduce(flags.view(torch.uint8), op=dist.ReduceOp.MAX, group=group, async_op=True))
    if async_op:
        return work
    for w in work:
        w.wait()
    return keys, flags


def chunk_bounds(n: int, chunks: int):
    """Splits [0, n) into `chunks` contiguous ranges, multiples of 64 pods (the sweep's flush unit)."""
    chunks = max(1, min(chunks, (n + 63) // 64))
    step = ((n + chunks - 1) // chunks + 63) // 64 * 64
    return [(a, min(n, a + step)) for a in range(0, n, step)]


def _ordered_backend(group=None) -> bool:
    """True when the group's collectives complete in issue order on one device
    stream (torch's "nccl" = RCCL backend); gloo's worker threads give no such order."""
    import torch.distributed as dist

    try:
        return dist.is_initialized() and dist.get_backend(group) == "nccl"
    except Exception:
        return False


class CrossStepPipeline:
    """Overlaps batch k's cross-shard combine with the following batches' sweeps.

    depth + 1 key buffers rotate between batches (two by default). step(batch)
    sweeps the batch into its buffer, starts the async combine of that buffer,
    then, once `depth` combines are in flight, waits for the OLDEST one and
    decodes it; finish() drains the rest. With depth 1 the device stream runs
    sweep k+1 -> wait(combine k) -> decode k, so the collective of batch k runs
    while batch k+1 sweeps; depth 2 gives each collective two sweeps of slack
    (a collective slower than one sweep, or a cross-queue wait that lands late,
    then no longer idles the sweep stream). Buffer b is swept again only
    depth + 1 batches later, after its decode (stream order).

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
        # group > 1: drain `group` batches at a time. With ordered=True (RCCL: one
        # stream per communicator runs the collectives in issue order) only the
        # newest batch's combine is waited for, so the sweep stream pays one
        # cross-queue wait per `group` steps instead of one per step.
        self.group = group
        self.ordered = ordered
        # decode_many([(buf, batch), ...]): the drained batches' decodes in one launch
        self._decode_many = decode_many
        self._n = 0
        self._pending = []  # [(works, buf, batch)], oldest first

    def step(self, batch=None, drain_stream=None):
        """drain_stream (optional torch stream): the oldest batch's wait() and
        decode are issued with it current, off the sweep stream."""
        buf = self._n % self.nbuf
        self._n += 1
        self._sweep(buf, batch)
        self._pending.append((self._combine(buf), buf, batch))
        if len(self._pending) > self.depth:
            n = min(self.group, len(self._pending))
            if drain_stream is None:
                self._drain_n(n)
            else:
                import torch

                prev = torch.cuda.current_stream()
                torch.cuda.set_stream(drain_stream)
                try:
                    self._drain_n(n)
                finally:
                    torch.cuda.set_stream(prev)

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

    def _drain(self):
        if self._pending:
            self._drain_n(len(self._pending))

    def finish(self):
        self._drain()


class ShardedCycle:
    """One rank's engine + device buffers for a fixed pod batch (bench / service loop).

    step() = per pod chunk: sweep this rank's node shard, then an async RCCL
    MAX all-reduce of the chunk's keys that overlaps the next chunk's sweep;
    finally decode every chunk once its reduction has landed.

    With pipeline=True (N > 1) a step is instead one whole-batch sweep whose
    all-reduce overlaps the next `depth` steps' sweeps (CrossStepPipeline,
    depth + 1 key buffers); the step's decode lands `depth` steps later and
    finish() drains the rest. Pod chunks within a step cost more sweep time than the overlap
    saves at small shards (tools/shard_probe.py), so the pipelined form uses
    one chunk.
    """

    POD_BYTES = 40
    RESULT_BYTES = 24

    def __init__(self, engine, n_nodes_global: int, n_pods: int, pods_dev, stream, want_flags: bool = False,
                 group=None, chunks: int = 1, pipeline: bool = False, decode_stream: bool = False,
                 depth: int = 1, drain_group: int = 1, collective: bool = True):
        import torch

        self.eng = engine
        self.N = n_nodes_global
        self.P = n_pods
        self.pods = pods_dev
        self.stream = stream
        self.group = group
        dev = pods_dev.device
        # with the decode stream, two spare key buffers let the host wait for a
        # buffer's last decode (host-side flow control) long after it finished
        # (MINISCHED_PIPE_SPARE overrides the two, for A/B runs)
        spare = int(os.environ.get("MINISCHED_PIPE_SPARE", "2")) if decode_stream else 0
        nbuf = depth + 1 + spare if pipeline else 1
        self._keys = [torch.empty(n_pods, dtype=torch.int64, device=dev) for _ in range(nbuf)]
        self._flags = ([torch.empty(n_pods, dtype=torch.int32, device=dev) for _ in range(nbuf)]
                       if want_flags else [None] * nbuf)
        self.keys, self.flags = self._keys[0], self._flags[0]
        # one results array per key buffer: a grouped drain decodes several batches at once
        self._results = [torch.empty(n_pods * self.RESULT_BYTES, dtype=torch.uint8, device=dev)
                         for _ in range(nbuf)]
        self._last = 0  # buffer of the most recently decoded batch
        self.chunks = chunk_bounds(n_pods, 1 if pipeline else chunks)
        self._pipe = None
        # collective=False: one shard (N = 1) run through the same pipeline, decodes grouped
        self._collective = collective
        # decode_stream=True (opt-in, MINISCHED_DECODE_STREAM=1 in bench.py): the
        # decode of step k waits for step k's combine on a stream of its own, so
        # the sweep stream never waits on another queue (a cross-queue wait idles
        # the waiting stream ~10 us even when its event completed long before,
        # profiles/r01o_*). A key buffer is reused only after its last decode: the
        # HOST waits for that decode's event, so the sweep stream carries no
        # waits at all. The extra host calls make the small-shard step host-bound,
        # though, and grouped drains on the sweep stream (depth 3, group 3) measure
        # better at every shard size (profiles/r01t_pipeline_group_ab.jsonl).
        self._dstream = None
        self._dec_ev = [None] * nbuf
        self._dec_live = [False] * nbuf
        if pipeline and decode_stream and dev.type == "cuda":
            self._dstream = torch.cuda.Stream(device=dev)
            self._dec_ev = [torch.cuda.Event() for _ in range(nbuf)]
        if pipeline:
            self._pipe = CrossStepPipeline(self._pipe_sweep,
                                           lambda buf: (combine_(self._keys[buf], self._flags[buf], self.group,
                                                                 async_op=True) if collective else []),
                                           lambda buf, _b: self.decode(0, self.P, buf), depth=depth, nbuf=nbuf,
                                           group=drain_group, ordered=_ordered_backend(group),
                                           decode_many=self._decode_many if self._dstream is None else None)

    def _ptrs(self, a, buf=0):
        pods = self.pods.data_ptr() + a * self.POD_BYTES
        keys = self._keys[buf].data_ptr() + a * 8
        flags = self._flags[buf].data_ptr() + a * 4 if self._flags[buf] is not None else 0
        return pods, keys, flags

    def sweep(self, a, b, buf=0):
        pods, keys, flags = self._ptrs(a, buf)
        self.eng.sweep_device(b - a, pods, keys, flags, self.stream.cuda_stream)

    def _pipe_sweep(self, buf, _batch):
        if self._dec_live[buf]:  # host waits for the decode that last read keys[buf]
            self._dec_ev[buf].synchronize()
        self.sweep(0, self.P, buf)

    @property
    def results(self):
        """Decoded ms_result bytes of the most recent batch (valid once its stream work is done)."""
        return self._results[self._last]

    def _decode_many(self, bufs):
        from . import _lib

        jobs = []
        for buf, _batch in bufs:
            pods, keys, flags = self._ptrs(0, buf)
            jobs.append((self.P, pods, keys, flags, self._results[buf].data_ptr()))
        for i in range(0, len(jobs), _lib.DECODE_MAX_JOBS):
            self.eng.decode_device_jobs(jobs[i:i + _lib.DECODE_MAX_JOBS], self.N, self.stream.cuda_stream)
        self._last = bufs[-1][0]

    def decode(self, a, b, buf=0):
        pods, keys, flags = self._ptrs(a, buf)
        res = self._results[buf].data_ptr() + a * self.RESULT_BYTES
        self._last = buf
        if self._dstream is None:
            self.eng.decode_device(b - a, pods, keys, flags, self.N, res, self.stream.cuda_stream)
            return
        # called inside CrossStepPipeline's drain with the decode stream current:
        # the combine's wait() has already ordered this stream after the collective
        self.eng.decode_device(b - a, pods, keys, flags, self.N, res, self._dstream.cuda_stream)
        self._dec_ev[buf].record(self._dstream)
        self._dec_live[buf] = True

    def step(self, world: int, on_sweep=None):
        if self._pipe is not None and (world > 1 or not self._collective):
            self._pipe.step(drain_stream=self._dstream)
            return
        pending = []
        for a, b in self.chunks:
            self.sweep(a, b)
            if on_sweep is not None:
                on_sweep(a, b)
            if world > 1:
                fl = self.flags[a:b] if self.flags is not None else None
                pending.append(combine_(self.keys[a:b], fl, self.group, async_op=True))
        for i, (a, b) in enumerate(self.chunks):
            if world > 1:
                for w in pending[i]:
                    w.wait()
            self.decode(a, b)

    def finish(self):
        """Drains a pipelined step's pending combine + decode (no-op otherwise).

        With the decode stream, the caller's stream is ordered after the last
        decode, so a synchronize of it (or of the device) covers the results.
        """
        if self._pipe is not None:
            if self._dstream is not None:
                import torch

                prev = torch.cuda.current_stream()
                torch.cuda.set_stream(self._dstream)
                try:
                    self._pipe.finish()
                finally:
                    torch.cuda.set_stream(prev)
                self.stream.wait_stream(self._dstream)
            else:
                self._pipe.finish()
