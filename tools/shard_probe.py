#!/usr/bin/env python3
"""One rank's share of an N-GPU config C step, timed on one GPU (no collective).

For G in --worlds, builds rank 0's node shard of 100k nodes (sharded.shard_bounds)
and times ShardedCycle.step(world=1) over all 100k pods with 1 and 4 pod chunks,
plus the bare sweep. It bounds what the driver's 2/4/8-GPU runs can reach before
RCCL: the all-reduce cost comes on top. Prints one JSON line per (G, chunks).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--chunks", default="1,4")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch

    from minisched_amd import _lib, sharded, synth

    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    N, P = synth.CONFIGS["C"]["nodes"], synth.CONFIGS["C"]["pods"]
    pods = torch.from_numpy(synth.pods(P, seed=1).view(np.uint8).copy()).to(dev)
    for G in (int(x) for x in args.worlds.split(",")):
        lo, hi = sharded.shard_bounds(N, 0, G)
        eng = _lib.Engine(max_nodes=hi - lo, plugin_set=_lib.PLUGINS_NU_NN, node_base=lo, seed=1)
        eng.upsert(np.arange(lo, hi, dtype=np.uint32), synth.nodes(hi - lo, seed=1, start=lo))
        eng.flush()
        for ch in (int(x) for x in args.chunks.split(",")):
            cyc = sharded.ShardedCycle(eng, N, P, pods, stream, chunks=ch)

            def timed(fn):
                for _ in range(3):
                    fn()
                ev = []
                for _ in range(args.reps):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(stream)
                    fn()
                    b.record(stream)
                    ev.append((a, b))
                torch.cuda.synchronize()
                return float(np.median([a.elapsed_time(b) for a, b in ev]))

            step_ms = timed(lambda: cyc.step(1))
            sweep_ms = timed(lambda: [cyc.sweep(a, b) for a, b in cyc.chunks])
            print(json.dumps({"world": G, "shard_rows": hi - lo, "chunks": len(cyc.chunks),
                              "step_ms": step_ms, "sweep_ms": sweep_ms}), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
