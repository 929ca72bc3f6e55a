#!/usr/bin/env python3
"""K1 pp sweep time against pods at fixed rows and against rows at fixed pods
(ms_sweep_device back to back on one stream): the intercepts are the per-launch
fixed costs that set the strong-scaling per-rank step."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def main():
    import torch

    from minisched_amd import _lib, synth

    K = int(os.environ.get("PROBE_STEPS", 50))
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    pods_all = torch.from_numpy(synth.pods(400_000, seed=1).view(np.uint8).copy()).to(dev)
    kb = torch.empty(400_000, dtype=torch.int64, device=dev)
    out = {}
    shapes = [(12_500, p) for p in (12_500, 25_000, 50_000, 100_000, 200_000, 400_000)] + \
             [(r, 100_000) for r in (3_125, 6_250, 25_000, 50_000, 100_000)]
    # PROBE_CTX=1: the engine's own context stream (no cross-stream events per call)
    ctx = os.environ.get("PROBE_CTX") == "1"
    for rows, P in shapes:
        eng = _lib.Engine(max_nodes=rows, node_base=0, seed=1)
        eng.upsert(np.arange(rows), synth.nodes(rows, seed=1))
        eng.flush()
        st = 0 if ctx else s.cuda_stream
        for _ in range(5):
            eng.sweep_device(P, pods_all.data_ptr(), kb.data_ptr(), 0, st)
        if ctx:  # time on the context stream: host wall after a sync, K calls, sync
            import time
            eng.info()
            t0 = time.perf_counter()
            for _ in range(K):
                eng.sweep_device(P, pods_all.data_ptr(), kb.data_ptr(), 0, st)
            eng.info()
            out[f"r{rows}_p{P}_us"] = round((time.perf_counter() - t0) * 1e6 / K, 2)
            eng.close()
            print(json.dumps(out), flush=True)
            continue
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(K):
            eng.sweep_device(P, pods_all.data_ptr(), kb.data_ptr(), 0, st)
        e1.record(s)
        e1.synchronize()
        out[f"r{rows}_p{P}_us"] = round(e0.elapsed_time(e1) * 1e3 / K, 2)
        eng.close()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
