#!/usr/bin/env python3
"""K launches of the K1 sweep of ONE strong-scaling shard (rank G-1 of config
C's 100k rows over G ranks, all 100k pods, keys out) on one stream, for
rocprofv3 kernel-trace / --pmc passes of that shape alone (tools/profile_g8.sh).
PAIR=1: the coalesced two-batch form (two 100k-pod batches per launch,
ms_sharded_submit's pairing) instead of one batch per launch."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def main():
    import torch

    from minisched_amd import _lib, sharded, synth

    G, K = int(os.environ.get("G", 8)), int(os.environ.get("K", 50))
    N = P = 100_000
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    pods = torch.from_numpy(synth.pods(P, seed=1).view(np.uint8).copy()).to(dev)
    lo, hi = sharded.shard_bounds(N, G - 1, G)
    eng = _lib.Engine(max_nodes=hi - lo, node_base=lo, seed=1)
    eng.upsert(np.arange(lo, hi), synth.nodes(hi - lo, seed=1, start=lo))
    eng.flush()
    kb = torch.empty(P, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    for _ in range(3):
        eng.sweep_device(P, pods.data_ptr(), kb.data_ptr(), 0, s.cuda_stream)
    s.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        eng.sweep_device(P, pods.data_ptr(), kb.data_ptr(), 0, s.cuda_stream)
    s.synchronize()
    dt = (time.perf_counter() - t0) / K
    print(json.dumps({"G": G, "shard_rows": hi - lo, "pods": P, "launches": K, "us_per_launch_wall": dt * 1e6}))
    eng.close()


if __name__ == "__main__":
    main()
