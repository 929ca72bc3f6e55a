#!/usr/bin/env python3
"""Config E one batch per call: per-batch wall time and validator counters
(re-swept tiles, recomputed entries) for the first batches of the queue, to
locate the early slow-path burst. Not a bench: each call pays
its own sweep + merge + validation with no overlap."""
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

    N, P, B = 50_000, int(os.environ.get("PROBE_PODS", 12800)), 128
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    nr = synth.nodes(N, seed=1, resources=True)
    pr = synth.pods(P, seed=1, resources=True)
    pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
    res = torch.empty(P * 24, dtype=torch.uint8, device=dev)
    eng = _lib.Engine(max_nodes=N, plugin_set=_lib.PLUGINS_NU_NRF_NN_LA, seed=1)
    eng.upsert(np.arange(N), nr)
    eng.flush()
    rows = []
    prev = eng.info()
    for a in range(0, P, B):
        t0 = time.perf_counter()
        eng.schedule_sequential_device(B, pods.data_ptr() + 40 * a, res.data_ptr() + 24 * a, s.cuda_stream)
        s.synchronize()
        dt = (time.perf_counter() - t0) * 1e6
        inf = eng.info()
        rows.append([a // B, round(dt, 1), inf.seq_resweep_tiles - prev.seq_resweep_tiles,
                     inf.seq_recomputes - prev.seq_recomputes])
        prev = inf
    r = res.cpu().numpy().view(_lib.RESULT)
    print(json.dumps({"batches": rows, "codes": {k: int((r["code"] == v).sum()) for k, v in
                                                 (("success", 0), ("error", 1), ("fit_error", 2))}}))


if __name__ == "__main__":
    main()
