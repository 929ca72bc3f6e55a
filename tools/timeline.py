#!/usr/bin/env python3
"""Per-kernel busy time and inter-kernel idle gaps from a rocprofv3 kernel trace.

usage: timeline.py run_kernel_trace.csv [last_n_kernels]
Sorts the trace by start time and, over the last n kernels, prints each
kernel name's count / mean duration and the idle time between one kernel's
end and the next kernel's start (the GPU-side cost of launches and cross-stream
hand-offs).
"""
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)[-last:]
agg, gaps = {}, {}
for i, (s, e, n) in enumerate(ev):
    key = n.replace("void ", "").replace("msgpu::(anonymous namespace)::", "").split("(")[0][:60]
    a = agg.setdefault(key, [0, 0.0])
    a[0] += 1
    a[1] += (e - s) / 1e3
    if i:
        prev = ev[i - 1]
        g = (s - prev[1]) / 1e3
        pk = prev[2].replace("void ", "").replace("msgpu::(anonymous namespace)::", "").split("(")[0][:40]
        gk = gaps.setdefault(f"{pk} -> {key[:40]}", [0, 0.0])
        gk[0] += 1
        gk[1] += g
span = (ev[-1][1] - ev[0][0]) / 1e3
print(json.dumps({"kernels": len(ev), "span_us": span,
                  "busy_us": {k: {"n": v[0], "mean_us": v[1] / v[0]} for k, v in agg.items()},
                  "gap_us": {k: {"n": v[0], "mean_us": v[1] / v[0]} for k, v in gaps.items()}}, indent=1))
