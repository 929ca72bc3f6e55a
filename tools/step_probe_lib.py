#!/usr/bin/env python3
"""Per-rank step of bench.py's N > 1 path through the in-library communicator,
on one GPU: a 1-rank communicator whose context holds the shard rank G-1 of
config C would own (100k/G rows), stepping all 100k pods through
ms_sharded_submit (sweep on the alternating sweep streams, reduce-scatter,
slice decode on the decode stream) exactly as ShardedCycle does, K steps
between HIP events, then ms_sharded_drain. With one rank the reduce-scatter is
a copy and the slice is all 100k pods (a G-rank slice is 100k/G), so this
slightly over-counts the decode. MINISCHED_SHARD_STREAMS=1 (set per variant)
puts every sweep on one stream; MINISCHED_SHARD_COALESCE=0 gives each submit
its own sweep launch (default: two consecutive submits share one K1 launch).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def main():
    import torch

    from minisched_amd import _lib, sharded, synth

    N, P, K = 100_000, 100_000, int(os.environ.get("PROBE_STEPS", 100))
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    pods = torch.from_numpy(synth.pods(P, seed=1).view(np.uint8).copy()).to(dev)
    out = {}
    # PROBE_VARIANTS "prio:streams,...": MINISCHED_SWEEP_PRIO x MINISCHED_SHARD_STREAMS
    variants = os.environ.get("PROBE_VARIANTS", "")
    variants = [v.split(":") for v in variants.split(",")] if variants else \
        [("1", st) for st in os.environ.get("PROBE_STREAMS", "2,1").split(",")]
    # PROBE_COALESCE "1,0": MINISCHED_SHARD_COALESCE per variant (two submits' sweeps in one launch)
    coal = os.environ.get("PROBE_COALESCE", "1").split(",")
    variants = [(p_, st, co) for p_, st in variants for co in coal]
    for prio, streams, co in variants * int(os.environ.get("PROBE_REPEAT", "1")):
        os.environ["MINISCHED_SHARD_STREAMS"] = streams
        os.environ["MINISCHED_SHARD_COALESCE"] = co
        os.environ["MINISCHED_SWEEP_PRIO"] = prio
        streams = f"{streams}p{prio}" + ("" if co == "1" else "c0")
        for G in [int(g) for g in os.environ.get("PROBE_G", "1,2,4,8,16").split(",")]:
            lo, hi = sharded.shard_bounds(N, G - 1, G)
            eng = _lib.Engine(max_nodes=hi - lo, node_base=lo, seed=1)
            eng.upsert(np.arange(lo, hi), synth.nodes(hi - lo, seed=1, start=lo))
            eng.flush()
            sharded.init_comm(eng)
            cyc = sharded.ShardedCycle(eng, N, P, pods, s)
            for _ in range(10):
                cyc.step()
            cyc.finish()
            s.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            t0 = time.perf_counter()
            for _ in range(K):
                cyc.step()
            host = time.perf_counter() - t0
            cyc.finish()
            e1.record(s)
            e1.synchronize()
            out.setdefault(f"G{G}_streams{streams}_us", []).append(round(e0.elapsed_time(e1) * 1e3 / K, 2))
            out.setdefault(f"G{G}_streams{streams}_host_enqueue_us", []).append(round(host * 1e6 / K, 2))
            # the sweep alone, back to back on one stream (the per-rank compute floor)
            kb = torch.empty(P, dtype=torch.int64, device=dev)
            e0.record(s)
            for _ in range(K):
                eng.sweep_device(P, pods.data_ptr(), kb.data_ptr(), 0, s.cuda_stream)
            e1.record(s)
            e1.synchronize()
            out[f"G{G}_sweep_only_us"] = round(e0.elapsed_time(e1) * 1e3 / K, 2)
            eng.close()
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
