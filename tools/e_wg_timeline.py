#!/usr/bin/env python3
"""Per-workgroup timeline of config-E steps from the MS_VSTAMPS build
(MS_TIMELINE=<file>: u64 [16 steps][256 workgroups][8], s_memrealtime ticks of
10 ns; fields: 0 start, 1 swept + counted, 2 worker wait done, 3 worker merges
done, 4 validator done (workgroup 0)). Prints, per step, microseconds from the
first workgroup's start: the start spread, swept min / median / max, the
workers' wait done (median / max), merges done (max) and the validator's end.
usage: python tools/e_wg_timeline.py <file> [json_out]"""
import json
import sys

import numpy as np


def main(path, out=None):
    tl = np.fromfile(path, dtype=np.uint64).reshape(16, 256, 8).astype(np.int64)
    rows = []
    for s in range(16):
        b = tl[s, :, 0]
        live = b > 0
        if not live.any():
            continue
        t0 = b[live].min()
        us = lambda v: (v - t0) / 100.0  # noqa: E731
        r = {"step": 200 + s, "workgroups": int(live.sum()), "start_spread_us": float(us(b[live].max()))}
        sw = tl[s, live, 1]
        sw = sw[sw > 0]
        if len(sw):
            r.update(swept_min=float(us(sw.min())), swept_median=float(us(np.median(sw))), swept_max=float(us(sw.max())))
        w = tl[s, live, 2]
        w = w[w > 0]
        if len(w):
            r.update(waited_median=float(us(np.median(w))), waited_max=float(us(w.max())))
        m = tl[s, live, 3]
        m = m[m > 0]
        if len(m):
            r.update(merged_median=float(us(np.median(m))), merged_max=float(us(m.max())))
        if tl[s, 0, 4] > 0:
            r["validator_done"] = float(us(tl[s, 0, 4]))
        # workgroup 0 (the validator's): 6 prologue done, 5 decisions done, 7 write-back issued
        for f, name in ((6, "val_prologue"), (5, "val_decided"), (7, "val_written")):
            if tl[s, 0, f] > 0:
                r[name] = float(us(tl[s, 0, f]))
        for f, name in ((5, "staged"), (6, "wave0_tasks"), (7, "all_tasks")):
            x = tl[s, 1:, f][live[1:]]
            x = x[x > 0]
            if len(x):
                r[name + "_median"] = float(us(np.median(x)))
                r[name + "_max"] = float(us(x.max()))
        rows.append(r)
    keys = ["start_spread_us", "staged_median", "staged_max", "wave0_tasks_median", "all_tasks_median",
            "all_tasks_max", "swept_min", "swept_median", "swept_max", "waited_median", "waited_max",
            "merged_median", "merged_max", "val_prologue", "val_decided", "val_written", "validator_done"]
    med = {k: float(np.median([r[k] for r in rows if k in r])) for k in keys if any(k in r for r in rows)}
    for r in rows:
        print(" ".join(f"{k}={r[k]:.2f}" if isinstance(r[k], float) else f"{k}={r[k]}" for k in r))
    print("median over steps:", json.dumps(med))
    if out:
        json.dump({"steps": rows, "median": med}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
