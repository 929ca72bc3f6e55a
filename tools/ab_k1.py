#!/usr/bin/env python3
"""Interleaved A/B of the NU+NN sweep variants in ONE process (rule: perf deltas
from interleaved rounds on one device). Prints per-variant kernel ms (HIP events
on the launch stream), median and min over rounds."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def main():
    import torch

    from minisched_amd import _lib, synth

    N = int(os.environ.get("AB_NODES", 100_000))
    P = int(os.environ.get("AB_PODS", 100_000))
    rounds = int(os.environ.get("AB_ROUNDS", 8))
    variants = os.environ.get("AB_VARIANTS", "v7,v0").split(",")
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    eng = _lib.Engine(max_nodes=N, seed=1)
    eng.upsert(np.arange(N), synth.nodes(N, seed=1))
    eng.flush()
    pods = torch.from_numpy(synth.pods(P, seed=1).view(np.uint8).copy()).to(dev)
    keys = {v: torch.empty(P, dtype=torch.int64, device=dev) for v in variants}
    times = {v: [] for v in variants}
    for r in range(rounds + 1):
        for v in variants:
            if "=" in v:  # an env setting read per launch, e.g. MINISCHED_K1_GROUP=0
                k, val = v.split("=", 1)
                os.environ[k] = val
            else:
                os.environ["MINISCHED_K1"] = v
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            eng.sweep_device(P, pods.data_ptr(), keys[v].data_ptr(), 0, s.cuda_stream)
            b.record(s)
            b.synchronize()
            if r:
                times[v].append(a.elapsed_time(b))
    same = all(torch.equal(keys[variants[0]], keys[v]) for v in variants[1:])
    out = {v: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
               "evals_per_s": N * P / (np.median(t) * 1e-3)} for v, t in times.items()}
    out["keys_identical"] = bool(same)
    out["nodes"], out["pods"] = N, P
    print(json.dumps(out))


if __name__ == "__main__":
    main()
