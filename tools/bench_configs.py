#!/usr/bin/env python3
"""Secondary measurements for BASELINE.json's other configs (not the driver line).

  B  5k x 10k   NU+NN  exact sequential      device-resident (ms_schedule_sequential_device)
  C  100k x 100k NU+NN batched, host API     PCIe-inclusive (ms_schedule_batch, host arrays)
  D  50k x 1M   NU+NN  batched                device-resident fused cycle (ms_select_batch_device)
  E  50k x 200k NU+NRF+NN+LA exact sequential device-resident (speculative sweep + in-order validator)

Each line: evals/s (P*N/time), pods/s, median of --reps after one warm-up.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))


def timed(fn, reps, sync):
    fn()
    sync()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        sync()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), float(np.min(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="B,C,D,E")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--e-pods", type=int, default=200_000)
    args = ap.parse_args()
    import torch

    from minisched_amd import _lib, synth

    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(s)
    # the device-resident configs run on the engine's own (context) stream, the
    # API default (stream NULL): a caller stream adds a cross-queue event each
    # way per call (~19 us at config B, tools/b_stream_ab.py)
    sp = 0
    out = []
    for c in args.configs.split(","):
        cfg = synth.CONFIGS[c]
        N, P = cfg["nodes"], cfg["pods"]
        res = c == "E"
        if c == "E":
            P = args.e_pods
        ps = _lib.PLUGINS_NU_NRF_NN_LA if res else _lib.PLUGINS_NU_NN
        nr = synth.nodes(N, seed=1, resources=res)
        pr = synth.pods(P, seed=1, resources=res)
        eng = _lib.Engine(max_nodes=N, plugin_set=ps, seed=1, max_batch=1 << 17)
        pods = torch.from_numpy(pr.view(np.uint8).copy()).to(dev)
        results = torch.empty(P * 24, dtype=torch.uint8, device=dev)
        keys = torch.empty(P, dtype=torch.int64, device=dev)
        extra = {}
        if c in ("B", "E"):
            def reset():
                eng.upsert(np.arange(N), nr)  # fresh node state (requested = 0) each rep
                eng.flush()

            def run():
                eng.schedule_sequential_device(P, pods.data_ptr(), results.data_ptr(), sp)
                torch.cuda.synchronize()

            reset()
            run()
            s.synchronize()
            ts = []
            for _ in range(args.reps):
                reset()
                t0 = time.perf_counter()
                run()
                s.synchronize()
                ts.append(time.perf_counter() - t0)
            med, mn = float(np.median(ts)), float(np.min(ts))
            r = results.cpu().numpy().view(_lib.RESULT)
            extra["codes"] = {k: int((r["code"] == v).sum()) for k, v in (("success", 0), ("error", 1), ("fit_error", 2))}
            inf = eng.info()
            extra["seq_counters_all_reps"] = dict(pods=inf.seq_pods, resweep_tiles=inf.seq_resweep_tiles,
                                                  recomputes=inf.seq_recomputes, overflow=inf._pad)
            mode = "exact sequential (device-resident, context stream)"
        elif c == "C":
            eng.upsert(np.arange(N), nr)
            eng.flush()
            med, mn = timed(lambda: eng.schedule(pr, _lib.MODE_BATCHED), args.reps, lambda: None)
            mode = "batched via ms_schedule_batch (host arrays, PCIe-inclusive; commits binds)"
        else:
            eng.upsert(np.arange(N), nr)
            eng.flush()

            def run():
                eng.select_batch_device(P, pods.data_ptr(), results.data_ptr(), sp)
                torch.cuda.synchronize()

            med, mn = timed(run, args.reps, s.synchronize)
            mode = "batched (device-resident fused cycle, one launch, context stream)"
        line = dict(config=c, nodes=N, pods=P, plugins=cfg["plugins"], mode=mode, median_s=med, min_s=mn,
                    evals_per_s=N * P / med, pods_per_s=P / med, **extra)
        print(json.dumps(line), flush=True)
        out.append(line)
        eng.close()


if __name__ == "__main__":
    main()
