#!/usr/bin/env python3
"""Where does the timed region's one-off go?

The driver runs `bench.py --steps 20 --warmup 5`; in BENCH_r05 the event-timed
region (device_ms_per_step 0.2636) exceeded 20 x the kernel alone (0.2548 ms)
by ~175 us. This probe rebuilds bench.py's N = 1 cycle exactly (ShardedCycle,
the same stream, warm-up, synchronize) and then times the 20 steps with an
event between every step and a host clock after every launch call, after an
idle gap of 0 / 2 / 20 / 200 ms, so that a slow first step (clock ramp after
idle, first-call host work) separates from a uniform per-step cost.
Prints one JSON object per trial.
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

    steps = int(os.environ.get("PROBE_STEPS", "20"))
    warm = int(os.environ.get("PROBE_WARMUP", "5"))
    N = P = 100_000
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = _lib.Engine(max_nodes=N, plugin_set=_lib.PLUGINS_NU_NN, seed=1, device=0)
    eng.upsert(np.arange(N, dtype=np.uint32), synth.nodes(N, seed=1))
    eng.flush()
    pods_np = synth.pods(P, seed=1)
    pods = torch.from_numpy(pods_np.view(np.uint8).copy()).to(dev)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    cyc = sharded.ShardedCycle(eng, N, P, pods, stream, split="nodes", rank=0, world=1)
    for gap_ms in (0, 2, 20, 200, 0):
        for _ in range(warm):
            cyc.step()
        cyc.finish()
        torch.cuda.synchronize()
        torch.cuda.synchronize()
        if gap_ms:
            time.sleep(gap_ms * 1e-3)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        host = []
        t0 = time.perf_counter()
        evs[0].record(stream)
        for i in range(steps):
            cyc.step()
            host.append(time.perf_counter() - t0)
            evs[i + 1].record(stream)
        cyc.finish()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        per = [evs[i].elapsed_time(evs[i + 1]) for i in range(steps)]
        print(json.dumps({"gap_ms": gap_ms, "steps": steps, "wall_ms_per_step": wall * 1e3 / steps,
                          "event_ms_per_step": evs[0].elapsed_time(evs[-1]) / steps,
                          "step_ms": [round(x, 4) for x in per],
                          "first_minus_median_us": (per[0] - float(np.median(per))) * 1e3,
                          "host_launch_us": [round(h * 1e6, 1) for h in host[:5]]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
