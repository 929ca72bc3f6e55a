#!/usr/bin/env python3
"""Per-rank step of bench.py's N > 1 path at config C, one rank at a time on one
GPU, as a real rank of a G-GPU run does it.

The test-only loopback build (libminisched_gpu_loopback.so: ms_comm.cpp with the
RCCL calls replaced by an in-process communicator) in its solo mode
(MS_LB_SOLO=1): ONE context joins a G-rank communicator as rank G-1 with that
rank's 100k/G-row shard, and every step is the library's own ms_sharded_submit
-- the shard sweep of all 100k pods (coalesced pairs, K1), the grouped
reduce-scatter (here a G-way MAX over G copies of its own keys: the combine a
rank computes, without the xGMI transfers), the decode of ITS ceil(P/G)-pod
slice -- pipelined exactly as in the driver's run, ms_sharded_drain at the end.
(tools/step_probe_lib.py's 1-rank communicator decoded all 100k pods and its
"reduce-scatter" was an 800 KB copy.) Prints one JSON object per G: the step by
HIP events over K steps, host enqueue per step, the shard sweep alone, and the
linear-scaling target 0.245 ms / G (the single-GPU step, profiles/r06c_bench.json).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))
os.environ["MS_LB_SOLO"] = "1"


def main():
    import torch

    from minisched_amd import _lib, sharded, synth

    lb = _lib.load(_lib.LOOPBACK_LIB_PATH)
    N, P, K = 100_000, 100_000, int(os.environ.get("PROBE_STEPS", 200))
    single_ms = float(os.environ.get("PROBE_SINGLE_MS", "0.245"))
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    pods = torch.from_numpy(synth.pods(P, seed=1).view(np.uint8).copy()).to(dev)
    for G in [int(g) for g in os.environ.get("PROBE_G", "2,4,8").split(",")]:
        r = G - 1
        lo, hi = sharded.shard_bounds(N, r, G)
        eng = _lib.Engine(max_nodes=hi - lo, node_base=lo, seed=1, lib=lb)
        eng.upsert(np.arange(lo, hi), synth.nodes(hi - lo, seed=1, start=lo))
        eng.flush()
        eng.comm_init(_lib.comm_id_create(lb), r, G)
        cyc = sharded.ShardedCycle(eng, N, P, pods, s)
        assert cyc.library
        for _ in range(max(20, K // 5)):  # (warm: clocks up, pipeline full)
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
        step_us = e0.elapsed_time(e1) * 1e3 / K
        kb = torch.empty(P, dtype=torch.int64, device=dev)
        e0.record(s)
        for _ in range(K):
            eng.sweep_device(P, pods.data_ptr(), kb.data_ptr(), 0, s.cuda_stream)
        e1.record(s)
        e1.synchronize()
        sweep_us = e0.elapsed_time(e1) * 1e3 / K
        eng.close()
        print(json.dumps({"G": G, "rank": r, "shard_rows": hi - lo, "slice_pods": cyc.b - cyc.a,
                          "step_us": round(step_us, 2), "host_enqueue_us": round(host * 1e6 / K, 2),
                          "sweep_only_us": round(sweep_us, 2), "linear_us": round(single_ms * 1e3 / G, 2),
                          "frac_of_linear": round(single_ms * 1e3 / G / step_us, 3)}), flush=True)


if __name__ == "__main__":
    main()
