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


def combine_(keys, flags=None, group=None):
    """In-place cross-shard combine of one batch (keys int64[P], flags uint32[P])."""
    import torch
    import torch.distributed as dist

    if keys.dtype != torch.int64:
        raise TypeError("keys must be an int64 view of the uint64 packed keys")
    work = [dist.all_reduce(keys, op=dist.ReduceOp.MAX, group=group, async_op=True)]
    if flags is not None:
        if flags.dtype not in (torch.int32, torch.uint32):
            raise TypeError("flags must be 32-bit")
        work.append(dist.all_reduce(flags.view(torch.uint8), op=dist.ReduceOp.MAX, group=group, async_op=True))
    for w in work:
        w.wait()
    return keys, flags


class ShardedCycle:
    """One rank's engine + device buffers for a fixed pod batch (bench / service loop)."""

    def __init__(self, engine, n_nodes_global: int, n_pods: int, pods_dev, stream, want_flags: bool, group=None):
        import torch

        self.eng = engine
        self.N = n_nodes_global
        self.P = n_pods
        self.pods = pods_dev
        self.stream = stream
        self.group = group
        dev = pods_dev.device
        self.keys = torch.empty(n_pods, dtype=torch.int64, device=dev)
        self.flags: Optional[torch.Tensor] = (
            torch.empty(n_pods, dtype=torch.int32, device=dev) if want_flags else None
        )
        self.results = torch.empty(n_pods * 24, dtype=torch.uint8, device=dev)

    def step(self, world: int):
        sp = self.stream.cuda_stream
        fl = self.flags.data_ptr() if self.flags is not None else 0
        self.eng.sweep_device(self.P, self.pods.data_ptr(), self.keys.data_ptr(), fl, sp)
        if world > 1:
            combine_(self.keys, self.flags, self.group)
        self.eng.decode_device(self.P, self.pods.data_ptr(), self.keys.data_ptr(), fl, self.N,
                               self.results.data_ptr(), sp)
