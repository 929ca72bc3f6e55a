#!/usr/bin/env python3
"""Host cost of one rank's bench step at N = 1/2/4/8, on one GPU.

A 1-rank RCCL process group stands in for the N-rank one (same Python, torch
and RCCL call path; the collective itself is a local copy), so a rank's step
(sweep of its shard + async all-reduce + decode, sharded.CrossStepPipeline)
is timed end to end by the host clock and by HIP events. When the host clock
exceeds the device time, the step is launch-bound. With --graph the step
pair is also captured into one HIP graph (torch.cuda.CUDAGraph) and replayed.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,8")
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist

    from minisched_amd import _lib, sharded, synth

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    N, P = synth.CONFIGS["C"]["nodes"], synth.CONFIGS["C"]["pods"]
    pods = torch.from_numpy(synth.pods(P, seed=1).view(np.uint8).copy()).to(dev)
    for G in (int(x) for x in args.worlds.split(",")):
        lo, hi = sharded.shard_bounds(N, 0, G)
        eng = _lib.Engine(max_nodes=hi - lo, plugin_set=_lib.PLUGINS_NU_NN, node_base=lo, seed=1)
        eng.upsert(np.arange(lo, hi, dtype=np.uint32), synth.nodes(hi - lo, seed=1, start=lo))
        eng.flush()
        cyc = sharded.ShardedCycle(eng, N, P, pods, stream, pipeline=True,
                                   decode_stream=os.environ.get("MINISCHED_DECODE_STREAM", "0") == "1",
                               depth=int(os.environ.get("MINISCHED_PIPE_DEPTH", "4")),
                               drain_group=int(os.environ.get("MINISCHED_PIPE_GROUP", "4")))
        for _ in range(5):
            cyc.step(2)
        cyc.finish()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record(stream)
        for _ in range(args.steps):
            cyc.step(2)  # world > 1: the pipelined form with its all-reduce
        cyc.finish()
        b.record(stream)
        t_issue = time.perf_counter() - t0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        dev_ms = a.elapsed_time(b) / args.steps
        # the bare device work of one step: sweep + decode, launched back to back
        torch.cuda.synchronize()
        a.record(stream)
        for _ in range(args.steps):
            cyc.sweep(0, P)
            cyc.decode(0, P)
        b.record(stream)
        torch.cuda.synchronize()
        bare_ms = a.elapsed_time(b) / args.steps
        print(json.dumps({"world": G, "shard_rows": hi - lo, "step_wall_ms": wall * 1e3 / args.steps,
                          "host_issue_ms_per_step": t_issue * 1e3 / args.steps, "step_device_ms": dev_ms,
                          "sweep_decode_back_to_back_ms": bare_ms}), flush=True)
        eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
