#!/usr/bin/env python3
"""Per-workgroup timeline of config-E steps from the diagnostic timeline build
(MS_TIMELINE=<file>: u64 [steps][256 workgroups][8], s_memrealtime ticks of
10 ns, steps 0 .. 2047 of the last run; fields: 0 start, 2 sweep done / merge
worker starts, 3 worker merges stored, 4 validator done (workgroup 0); merge
workers (since r06aa) also 4 the first pod's lists all arrived, 1 its ranks merged).
Workgroup 0 (the validator's) also stamps 1 bulk LDS copies landed, 2 wave-0
loads landed (single-wave prologue), 3 stale nodes mapped, 6 prologue done,
5 decisions done, 7 write-back issued; sweep workgroups 5 tile staged, 6 wave
0's tasks done, 7 all tasks done.

Prints the per-phase medians over steps 200 .. 215 (the window earlier rounds
recorded) and, over the whole run, each step's validator end V and merge-path
end M (the last merge worker's), both from the step's first workgroup start,
with the step's length to the next step's start: how often the validator is
the critical path and what either path would save.
usage: python tools/e_wg_timeline.py <file> [json_out]"""
import json
import os
import sys

import numpy as np


def step_row(tl, s):
    b = tl[s, :, 0]
    live = b > 0
    if not live.any():
        return None
    t0 = b[live].min()
    us = lambda v: (v - t0) / 100.0  # noqa: E731
    r = {"step": s, "workgroups": int(live.sum()), "start_spread_us": float(us(b[live].max())), "t0": int(t0)}
    # merge workgroups (tagged lists, the default since round 5): 2 = its sweep done, 4 = the first
    # pod's lists all arrived, 1 = that pod's ranks merged (round 6 r06aa on), 3 = its merges stored
    for f, name in ((1, "ranked"), (2, "waited"), (3, "merged"), (4, "polled")):
        x = tl[s, 1:, f][live[1:]]
        x = x[x > 0]
        if len(x):
            r[name + "_median"] = float(us(np.median(x)))
            r[name + "_max"] = float(us(x.max()))
    if tl[s, 0, 4] > 0:
        r["validator_done"] = float(us(tl[s, 0, 4]))
    for f, name in ((1, "val_dma"), (2, "val_loads"), (3, "val_mapped"), (6, "val_prologue"),
                    (5, "val_decided"), (7, "val_written")):
        if tl[s, 0, f] > 0:
            r[name] = float(us(tl[s, 0, f]))
    for f, name in ((5, "staged"), (6, "wave0_tasks"), (7, "all_tasks")):
        x = tl[s, 1:, f][live[1:]]
        x = x[x > 0]
        if len(x):
            r[name + "_median"] = float(us(np.median(x)))
            r[name + "_max"] = float(us(x.max()))
    return r


def main(path, out=None):
    n_steps = os.path.getsize(path) // (256 * 8 * 8)
    tl = np.fromfile(path, dtype=np.uint64).reshape(n_steps, 256, 8).astype(np.int64)
    rows = [r for r in (step_row(tl, s) for s in range(n_steps)) if r]
    window = [r for r in rows if 200 <= r["step"] < 216]
    keys = ["start_spread_us", "staged_median", "staged_max", "wave0_tasks_median", "all_tasks_median",
            "all_tasks_max", "waited_median", "waited_max", "polled_median", "polled_max", "ranked_median",
            "ranked_max",
            "merged_median", "merged_max", "val_dma", "val_loads", "val_mapped", "val_prologue", "val_decided",
            "val_written", "validator_done"]
    med = {k: float(np.median([r[k] for r in window if k in r])) for k in keys if any(k in r for r in window)}
    for r in window:
        print(" ".join(f"{k}={r[k]:.2f}" if isinstance(r[k], float) else f"{k}={r[k]}" for k in r if k != "t0"))
    print("median over steps 200-215:", json.dumps(med))
    # whole run: V (validator end), M (merge-path end: the last merge worker, or the
    # last sweep workgroup where no merge ran), step length D to the next start
    run = {}
    full = [r for r in rows if "validator_done" in r]
    if len(full) > 1:
        V = np.array([r["validator_done"] for r in full])
        M = np.array([r.get("merged_max", 0.0) for r in full])
        t0 = np.array([r["t0"] for r in full], dtype=np.int64)
        D = np.diff(t0) / 100.0
        V1, M1 = V[:-1], M[:-1]
        run = {"steps": len(full), "run_us_first_to_last_start": float((t0[-1] - t0[0]) / 100.0),
               "step_us_mean": float(D.mean()), "V_mean": float(V.mean()), "M_mean": float(M.mean()),
               "V_median": float(np.median(V)), "M_median": float(np.median(M)),
               "V_p90": float(np.percentile(V, 90)), "frac_validator_critical": float((V > M).mean()),
               "sum_max_VM_us": float(np.maximum(V1, M1).sum()), "sum_D_us": float(D.sum()),
               "gap_us_mean": float((D - np.maximum(V1, M1)).mean()),
               "validator_excess_us": float(np.maximum(V1 - M1, 0).sum()),
               "merge_excess_us": float(np.maximum(M1 - V1, 0).sum())}
        print("whole run:", json.dumps(run))
    if out:
        with open(out, "w") as f:
            json.dump({"steps": window, "median": med, "run": run,
                       "per_step": [{"step": r["step"], "V": r.get("validator_done"),
                                     "M": r.get("merged_max"),
                                     "prologue": r.get("val_prologue")} for r in full]}, f, indent=0)


if __name__ == "__main__":
    main(*sys.argv[1:])
