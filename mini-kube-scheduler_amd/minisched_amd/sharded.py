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


class ShardedCycle:
    """One rank's engine + device buffers for a fixed pod batch (bench / service loop).

    step() = per pod chunk: sweep this rank's node shard, then an async RCCL
    MAX all-reduce of the chunk's keys that overlaps the next chunk's sweep;
    finally decode every chunk once its reduction has landed.
    """

    POD_BYTES = 40
    RESULT_BYTES = 24

    def __init__(self, engine, n_nodes_global: int, n_pods: int, pods_dev, stream, want_flags: bool = False,
                 group=None, chunks: int = 1):
        import torch

        self.eng = engine
        self.N = n_nodes_global
        self.P = n_pods
        self.pods = pods_dev
        self.stream = stream
        self.group = group
        dev = pods_dev.device
        self.keys = torch.empty(n_pods, dtype=torch.int64, device=dev)
        self.flags = torch.empty(n_pods, dtype=torch.int32, device=dev) if want_flags else None
        self.results = torch.empty(n_pods * self.RESULT_BYTES, dtype=torch.uint8, device=dev)
        self.chunks = chunk_bounds(n_pods, chunks)

    def _ptrs(self, a):
        pods = self.pods.data_ptr() + a * self.POD_BYTES
        keys = self.keys.data_ptr() + a * 8
        flags = self.flags.data_ptr() + a * 4 if self.flags is not None else 0
        return pods, keys, flags

    def sweep(self, a, b):
        pods, keys, flags = self._ptrs(a)
        self.eng.sweep_device(b - a, pods, keys, flags, self.stream.cuda_stream)

    def decode(self, a, b):
        pods, keys, flags = self._ptrs(a)
        res = self.results.data_ptr() + a * self.RESULT_BYTES
        self.eng.decode_device(b - a, pods, keys, flags, self.N, res, self.stream.cuda_stream)

    def step(self, world: int, on_sweep=None):
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
