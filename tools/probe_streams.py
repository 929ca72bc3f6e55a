#!/usr/bin/env python3
"""Do consecutive K1 pp sweeps gain from running on two streams? (G = 8 shard)

One 12.5k-row shard x 100k pods, K sweeps:
  one    : all on one stream (each launch waits for the previous to finish)
  two    : alternating two streams, two contexts holding the same shard (no
           cross-stream dependency: the launch ramp / tail of one sweep
           overlaps the next)
  two_ev : like two, plus one wait per launch on an already-signalled event
           recorded on a third stream (the cost of a dependency edge)
Prints us per sweep (HIP events around all K launches).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def main():
    import torch

    from minisched_amd import _lib, synth

    N, P, K = int(os.environ.get("PS_NODES", 12_500)), int(os.environ.get("PS_PODS", 100_000)), 40
    base = 100_000 - N
    dev = torch.device("cuda:0")
    nr = synth.nodes(N, seed=1, start=base)
    engs = []
    for _ in range(2):
        e = _lib.Engine(max_nodes=N, node_base=base, seed=1)
        e.upsert(np.arange(base, base + N), nr)
        e.flush()
        engs.append(e)
    pods = torch.from_numpy(synth.pods(P, seed=1).view(np.uint8).copy()).to(dev)
    keys = [torch.empty(P, dtype=torch.int64, device=dev) for _ in range(2)]
    st = [torch.cuda.Stream(device=dev) for _ in range(3)]
    ev_third = torch.cuda.Event()
    ev_third.record(st[2])
    out = {}
    for mode in ("one", "two", "two_ev", "one", "two", "two_ev"):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0.record(st[0])
        st[1].wait_event(t0)
        for k in range(K):
            i = 0 if mode == "one" else k & 1
            if mode == "two_ev":
                st[i].wait_event(ev_third)
            engs[i].sweep_device(P, pods.data_ptr(), keys[i].data_ptr(), 0, st[i].cuda_stream)
        e1 = torch.cuda.Event()
        e1.record(st[1])
        st[0].wait_event(e1)
        t1.record(st[0])
        t1.synchronize()
        out[mode] = round(t0.elapsed_time(t1) * 1e3 / K, 2)
    assert torch.equal(keys[0], keys[1])
    print(json.dumps({"nodes": N, "pods": P, "us_per_sweep": out}))


if __name__ == "__main__":
    main()
