#!/usr/bin/env python3
"""Per-rank device work of bench.py's default (weak-scaling) N > 1 step, on one GPU.

At G GPUs every rank sweeps the job's G x 100k pods against its 100k/G-row
shard (ms_sweep_device, K1 pp) and decodes its own 100k pods
(ms_decode_device): the per-rank evaluations stay 1e10 as G grows. HIP events
around K repetitions on one stream. The reduce-scatter of G x 100k x 8 B runs
on RCCL's stream in the real step, overlapped with the next steps' sweeps; it
is not here. Prints one JSON line: per-G ms and ms(G=1) / ms(G), the
efficiency the device work alone allows.
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

    N, P1, K = 100_000, 100_000, int(os.environ.get("PROBE_REPS", 20))
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    out = {}
    for G in (1, 2, 4, 8):
        P = P1 * G
        pods = torch.from_numpy(synth.pods(P, seed=1).view(np.uint8).copy()).to(dev)
        lo, hi = sharded.shard_bounds(N, G - 1, G)  # the last rank's shard
        eng = _lib.Engine(max_nodes=hi - lo, node_base=lo, seed=1)
        eng.upsert(np.arange(lo, hi), synth.nodes(hi - lo, seed=1, start=lo))
        eng.flush()
        keys = torch.empty(sharded.padded_pods(P, G), dtype=torch.int64, device=dev)
        res = torch.empty(P1 * 24, dtype=torch.uint8, device=dev)
        a, b = sharded.pod_slice(P, G - 1, G)

        def step():
            eng.sweep_device(P, pods.data_ptr(), keys.data_ptr(), 0, s.cuda_stream)
            eng.decode_device(b - a, pods.data_ptr() + 40 * a, keys.data_ptr() + 8 * a, 0, N, res.data_ptr(),
                              s.cuda_stream)

        step()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(K):
            step()
        e1.record(s)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / K
        eng.close()
        out[f"G{G}"] = {"shard_rows": hi - lo, "job_pods": P, "rank_ms": ms}
    base = out["G1"]["rank_ms"]
    for v in out.values():
        v["device_efficiency"] = base / v["rank_ms"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
