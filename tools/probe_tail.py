#!/usr/bin/env python3
"""K1 pp sweep time (100k pods, back to back on one stream) against rows near a
multiple of 64 x 30 = 1920 rows: the last lane word of a partial 64-group
word costs a full word's instructions on the SIMD that holds it."""
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
    P = 100_000
    pods = torch.from_numpy(synth.pods(P, seed=1).view(np.uint8).copy()).to(dev)
    kb = torch.empty(P, dtype=torch.int64, device=dev)
    rows_list = [int(r) for r in os.environ.get("PROBE_ROWS", "99840,99870,100000,101760,101790,97920,97950").split(",")]
    out = {}
    for rep in range(2):
        for rows in rows_list:
            eng = _lib.Engine(max_nodes=rows, node_base=0, seed=1)
            eng.upsert(np.arange(rows), synth.nodes(rows, seed=1))
            eng.flush()
            for _ in range(5):
                eng.sweep_device(P, pods.data_ptr(), kb.data_ptr(), 0, s.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(K):
                eng.sweep_device(P, pods.data_ptr(), kb.data_ptr(), 0, s.cuda_stream)
            e1.record(s)
            e1.synchronize()
            out.setdefault(f"r{rows}_us", []).append(round(e0.elapsed_time(e1) * 1e3 / K, 2))
            eng.close()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
