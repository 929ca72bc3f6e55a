#!/usr/bin/env python3
"""Config E per-batch cost from a rocprofv3 kernel-trace CSV of
tools/bench_configs.py --configs E (fused single-stream mode): every
k_seq_step / k_topk_merge dispatch in order, split into runs of 1563 batches,
and where the time goes: the median step, the excess over it per batch
window, and the slowest steps.
usage: python tools/e_batches.py <kernel_trace.csv> [batches_per_run]"""
import csv
import json
import sys

import numpy as np


def main(path, per_run=1563):
    rows = list(csv.DictReader(open(path)))

    def sel(tag):
        r = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in rows if tag in x["Kernel_Name"])
        return np.array(r, dtype=np.int64).reshape(-1, 2)

    st, mg = sel("k_seq_step"), sel("k_topk_merge")
    out = {"steps": int(len(st)), "merges": int(len(mg))}
    runs = len(st) // per_run
    for k in range(runs):
        s = st[k * per_run:(k + 1) * per_run]
        d = (s[:, 1] - s[:, 0]) / 1e3
        wall = (s[-1, 1] - s[0, 0]) / 1e6
        med = float(np.median(d))
        ex = np.clip(d - med, 0, None)
        win = [float(ex[i:i + 50].sum()) / 1e3 for i in range(0, per_run, 50)]
        top = np.argsort(d)[::-1][:12]
        out[f"run{k}"] = {
            "wall_ms": round(wall, 3), "step_sum_ms": round(float(d.sum()) / 1e3, 3), "step_median_us": round(med, 2),
            "excess_ms": round(float(ex.sum()) / 1e3, 3),
            "excess_ms_per_50_batches": [round(x, 3) for x in win],
            "slowest": [(int(i), round(float(d[i]), 1)) for i in top],
            "p90_us": round(float(np.percentile(d, 90)), 2), "p99_us": round(float(np.percentile(d, 99)), 2),
        }
        if len(mg) >= (k + 1) * per_run:
            m = mg[k * per_run:(k + 1) * per_run]
            dm = (m[:, 1] - m[:, 0]) / 1e3
            out[f"run{k}"]["merge_median_us"] = round(float(np.median(dm)), 2)
            out[f"run{k}"]["merge_sum_ms"] = round(float(dm.sum()) / 1e3, 3)
            # gaps between a merge's end and the next step's start (launch hand-off)
            gaps = (st[k * per_run + 1:(k + 1) * per_run, 0] - m[:per_run - 1, 1]) / 1e3
            out[f"run{k}"]["merge_to_step_gap_median_us"] = round(float(np.median(gaps)), 2)
            g2 = (m[:, 0] - s[:, 1]) / 1e3
            out[f"run{k}"]["step_to_merge_gap_median_us"] = round(float(np.median(g2)), 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
