#!/usr/bin/env python3
"""One rank's pipelined node-split step on one GPU, through a 1-rank RCCL group.

For shard sizes of config C at N = 2 / 4 / 8 (50k / 25k / 12.5k rows, the
last rank's ordinals) this runs bench.py's N > 1 step exactly (ShardedCycle
with its CrossStepPipeline: sweep, async reduce_scatter_tensor through torch's
"nccl" backend, grouped waits, grouped decodes), with collective=True on a
1-rank group. The collective is trivial here and the decode covers all P pods
(a real rank decodes P/N), so the device step is an upper bound of a real
rank's device work minus the collective's own cost. Reports the wall step
time, the device time (events around the K steps) and the host issue time
(perf_counter around the step calls, no sync): a host issue time near the
device time means the step is host-bound.
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
    import torch.distributed as dist

    from minisched_amd import _lib, sharded, synth

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    N, P, K = 100_000, 100_000, int(os.environ.get("PROBE_STEPS", 40))
    pods = torch.from_numpy(synth.pods(P, seed=1).view(np.uint8).copy()).to(dev)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    out = {}
    for G in (1, 2, 4, 8):
        lo, hi = sharded.shard_bounds(N, G - 1, G)
        eng = _lib.Engine(max_nodes=hi - lo, node_base=lo, seed=1)
        eng.upsert(np.arange(lo, hi), synth.nodes(hi - lo, seed=1, start=lo))
        eng.flush()
        cyc = sharded.ShardedCycle(eng, N, P, pods, stream, depth=4, drain_group=4, collective=G > 1,
                                   present_total=N)
        for _ in range(8):
            cyc.step()
        cyc.finish()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(K):
            cyc.step()
        t_issue = time.perf_counter() - t0
        cyc.finish()
        e1.record(stream)
        torch.cuda.synchronize()
        t_wall = time.perf_counter() - t0
        out[f"G{G}"] = {"shard_rows": hi - lo, "wall_ms_per_step": t_wall * 1e3 / K,
                        "device_ms_per_step": e0.elapsed_time(e1) / K, "host_issue_ms_per_step": t_issue * 1e3 / K}
        eng.close()
    dist.destroy_process_group()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
