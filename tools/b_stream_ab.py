#!/usr/bin/env python3
"""Config B (5k nodes x 10k pods, exact sequential, NU+NN): wall time of
ms_schedule_sequential_device on the context stream (NULL) vs a caller
stream (one cross-queue event each way), median of 21 after a warm-up."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def main():
    import torch

    from minisched_amd import _lib, synth

    N, P = 5000, 10000
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    nr = synth.nodes(N, seed=1)
    pr = synth.pods(P, seed=1)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
    eng = _lib.Engine(max_nodes=N, seed=1)
    out = {}
    for name, sp in (("ctx_stream", 0), ("caller_stream", s.cuda_stream), ("ctx_stream2", 0)):
        ts = []
        for i in range(22):
            eng.upsert(np.arange(N), nr)
            eng.flush()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.schedule_sequential_device(P, pods.data_ptr(), res.data_ptr(), sp)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name] = {"median_us": float(np.median(ts[1:])) * 1e6, "min_us": float(np.min(ts[1:])) * 1e6}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
