#!/usr/bin/env python3
"""Per-rank device work of bench.py's N > 1 node-split step, on one GPU.

For a shard of N/G rows (G = 2, 4, 8 at config C): the sweep of all P pods
against the shard (ms_sweep_device, K1 pp) and the decode of this rank's P/G
pods (ms_decode_device), back to back on one stream, HIP events around K
repetitions. The collective (reduce-scatter of P x 8 B) runs on RCCL's own
stream in the real step and overlaps the next steps' sweeps; it is not here.
Also the pod-split alternative: the fused cycle of P/G pods against all N rows.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def main():
    import torch

    from minisched_amd import _lib, sharded, synth

    N, P, K = 100_000, 100_000, int(os.environ.get("PROBE_REPS", 20))
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    pr = synth.pods(P, seed=1)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    out = {}
    for G in (1, 2, 4, 8):
        lo, hi = sharded.shard_bounds(N, G - 1, G)  # the last rank's shard
        eng = _lib.Engine(max_nodes=hi - lo, node_base=lo, seed=1)
        eng.upsert(np.arange(lo, hi), synth.nodes(hi - lo, seed=1, start=lo))
        eng.flush()
        keys = torch.empty(sharded.padded_pods(P, G), dtype=torch.int64, device=dev)
        res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
        a, b = sharded.pod_slice(P, G - 1, G)

        def step():
            eng.sweep_device(P, pods.data_ptr(), keys.data_ptr(), 0, s.cuda_stream)
            eng.decode_device(b - a, pods.data_ptr() + 40 * a, keys.data_ptr() + 8 * a, 0, N, res.data_ptr(),
                              s.cuda_stream)

        def timed(fn):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(K):
                fn()
            e1.record(s)
            e1.synchronize()
            return e0.elapsed_time(e1) / K

        node_ms = timed(step)
        sweep_ms = timed(lambda: eng.sweep_device(P, pods.data_ptr(), keys.data_ptr(), 0, s.cuda_stream))
        eng.close()
        full = _lib.Engine(max_nodes=N, seed=1)
        full.upsert(np.arange(N), synth.nodes(N, seed=1))
        full.flush()
        pod_ms = timed(lambda: full.select_batch_device(b - a, pods.data_ptr() + 40 * a, res.data_ptr(), s.cuda_stream))
        full.close()
        out[f"G{G}"] = {"shard_rows": hi - lo, "node_split_sweep_decode_ms": node_ms, "node_split_sweep_ms": sweep_ms,
                        "pod_split_cycle_ms": pod_ms, "pods_per_rank": b - a}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
