#!/usr/bin/env python3
"""Per-rank K1 sweep time for 2-D splits of config C over G GPUs: node shards Gn x pod
groups Gp = G, a rank sweeps P/Gp pods against N/Gn rows (ms_sweep_device, back to back
on one stream, HIP events). G=8: (8,1) is the 1-D node split, (1,8) the pod split."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def main():
    import torch

    from minisched_amd import _lib, sharded, synth

    N, P, K = 100_000, 100_000, int(os.environ.get("PROBE_STEPS", 100))
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    pods_all = synth.pods(P, seed=1)
    out = {}
    for G in [int(g) for g in os.environ.get("PROBE_G", "8,4").split(",")]:
        gn = G
        while gn >= 1:
            gp = G // gn
            lo, hi = sharded.shard_bounds(N, gn - 1, gn)
            np_ = -(-P // gp)
            pods = torch.from_numpy(pods_all[:np_].view(np.uint8).copy()).to(dev)
            eng = _lib.Engine(max_nodes=hi - lo, node_base=lo, seed=1)
            eng.upsert(np.arange(lo, hi), synth.nodes(hi - lo, seed=1, start=lo))
            eng.flush()
            kb = torch.empty(np_, dtype=torch.int64, device=dev)
            for _ in range(5):
                eng.sweep_device(np_, pods.data_ptr(), kb.data_ptr(), 0, s.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(K):
                eng.sweep_device(np_, pods.data_ptr(), kb.data_ptr(), 0, s.cuda_stream)
            e1.record(s)
            e1.synchronize()
            out[f"G{G}_n{gn}xp{gp}_us"] = round(e0.elapsed_time(e1) * 1e3 / K, 2)
            eng.close()
            print(json.dumps(out), flush=True)
            gn //= 2


if __name__ == "__main__":
    main()
