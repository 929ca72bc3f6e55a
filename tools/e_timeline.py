#!/usr/bin/env python3
"""Config E timeline from a rocprofv3 kernel-trace CSV: per-batch validator
duration, the sweep + merge durations, and the gaps on the validator's
critical path (validate k start - validate k-1 end), medians over the run.
usage: python tools/e_timeline.py <kernel_trace.csv>"""
import csv
import json
import sys

import numpy as np


def main(path):
    rows = list(csv.DictReader(open(path)))
    def sel(tag):
        r = [(int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in rows if tag in x["Kernel_Name"]]
        return np.array(sorted(r), dtype=np.int64)
    v, sw, mg = sel("k_validate_seq"), sel("k_sweep_full_topk"), sel("k_topk_merge")
    out = {"batches": int(len(v))}
    if len(v) > 1:
        dur = v[:, 1] - v[:, 0]
        gap = v[1:, 0] - v[:-1, 1]
        out.update(validate_us=float(np.median(dur)) / 1e3, validate_mean_us=float(dur.mean()) / 1e3,
                   gap_us=float(np.median(gap)) / 1e3, gap_mean_us=float(gap.mean()) / 1e3,
                   period_us=float(np.median(v[1:, 0] - v[:-1, 0])) / 1e3)
        # merge k end -> validate k start (validate waits on it when positive lag is small)
        n = min(len(mg), len(v))
        out["merge_end_to_validate_start_us"] = float(np.median(v[:n, 0] - mg[:n, 1])) / 1e3
    for name, a in (("sweep", sw), ("merge", mg)):
        if len(a):
            out[name + "_us"] = float(np.median(a[:, 1] - a[:, 0])) / 1e3
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
