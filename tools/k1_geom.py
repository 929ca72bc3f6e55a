#!/usr/bin/env python3
"""K1 geometry sweep in ONE process: rows per lane x pods per wave, per shard size.

Each launch reads MINISCHED_K1_RPL / MINISCHED_K1_CHUNK from the environment
(ms_kernels.hip launch_v7), so the variants interleave round by round on one
device. Prints one JSON line per (shard rows, rpl, chunk): median / min kernel
ms by HIP events on the launch stream. Keys are checked identical per shard.
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

    pod_counts = [int(x) for x in os.environ.get("GEOM_PODS", "100000").split(",")]
    rounds = int(os.environ.get("GEOM_ROUNDS", 6))
    shards = [int(x) for x in os.environ.get("GEOM_SHARDS", "100000,50000,25000,12500").split(",")]
    rpls = os.environ.get("GEOM_RPL", "20,30,32").split(",")
    chunks = os.environ.get("GEOM_CHUNK", "0,48,96,192,384").split(",")
    k1s = os.environ.get("GEOM_K1", "v7").split(",")
    waves = os.environ.get("GEOM_WAVES", "1").split(",")
    tols = os.environ.get("GEOM_TOL", "1").split(",")  # MINISCHED_K1_TOL
    reps = int(os.environ.get("GEOM_REPS", 1))  # back-to-back launches per timing (hides launch gaps)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    pods_all = torch.from_numpy(synth.pods(max(pod_counts), seed=1).view(np.uint8).copy()).to(dev)
    for N, P in [(n, p) for n in shards for p in pod_counts]:
        pods = pods_all[: P * 40]
        eng = _lib.Engine(max_nodes=N, seed=1)
        eng.upsert(np.arange(N), synth.nodes(N, seed=1))
        eng.flush()
        variants = [(r, c, k, wv, tl) for r in rpls for c in chunks for k in k1s for wv in waves for tl in tols]
        keys = {v: torch.empty(P, dtype=torch.int64, device=dev) for v in variants}
        times = {v: [] for v in variants}
        for rd in range(rounds + 1):
            for v in variants:
                os.environ["MINISCHED_K1_RPL"] = v[0]
                os.environ["MINISCHED_K1"] = v[2]
                os.environ["MINISCHED_K1_WAVES"] = v[3]
                os.environ["MINISCHED_K1_TOL"] = v[4]
                if v[1] == "0":
                    os.environ.pop("MINISCHED_K1_CHUNK", None)
                else:
                    os.environ["MINISCHED_K1_CHUNK"] = v[1]
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                for _ in range(reps):
                    eng.sweep_device(P, pods.data_ptr(), keys[v].data_ptr(), 0, s.cuda_stream)
                b.record(s)
                b.synchronize()
                if rd:
                    times[v].append(a.elapsed_time(b) / reps)
        ref = keys[variants[0]]
        same = all(torch.equal(ref, keys[v]) for v in variants[1:])
        for v in variants:
            t = times[v]
            print(json.dumps({"shard_rows": N, "pods": P, "rpl": int(v[0]), "chunk": int(v[1]) or "auto", "k1": v[2], "waves": v[3], "tol_lists": v[4],
                              "reps": reps, "median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
                              "keys_identical": bool(same)}), flush=True)
        eng.close()
    os.environ.pop("MINISCHED_K1_RPL", None)
    os.environ.pop("MINISCHED_K1_CHUNK", None)
    os.environ.pop("MINISCHED_K1_WAVES", None)


if __name__ == "__main__":
    main()
