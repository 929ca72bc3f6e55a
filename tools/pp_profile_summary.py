#!/usr/bin/env python3
"""Summarise a tools/profile_pp.sh run into profiles/<tag>_pmc_C.json and
profiles/<tag>_kernel_stats.csv (counters per launch of k_sweep_nunn_pp).

traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KB;
FETCH_SIZE reads half the bytes of wide coalesced streams on gfx950, so the
corrected read figure is 2 x FETCH_SIZE (raw values kept beside it).
SQ_ACTIVE_INST_VALU counts quad-cycles summed over waves (§ constants table).
"""
import csv
import json
import os
import shutil
import sys

KERNEL = "k_sweep_nunn_pp"
src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles")


def per_kernel(path):
    agg = {}
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


stats = os.path.join(src, "stats", "run_kernel_stats.csv")
shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
avg_ns = calls = None
for r in csv.DictReader(open(stats)):
    if KERNEL in r["Name"]:
        avg_ns, calls = float(r["AverageNs"]), int(r["Calls"])
bench = json.loads(open(os.path.join(src, "bench_stats.json")).read().strip().splitlines()[-1])
sq = per_kernel(os.path.join(src, "sq", "run_counter_collection.csv"))
fetch = per_kernel(os.path.join(src, "fetch", "run_counter_collection.csv")).get("FETCH_SIZE")
write = per_kernel(os.path.join(src, "write", "run_counter_collection.csv")).get("WRITE_SIZE")
out = {
    "kernel": KERNEL,
    "nodes": bench["config"]["nodes"],
    "pods": bench["config"]["pods"],
    "kernel_avg_ns_rocprof": avg_ns,
    "calls": calls,
    "SQ_INSTS_VALU": sq.get("SQ_INSTS_VALU"),
    "SQ_INSTS_SALU": sq.get("SQ_INSTS_SALU"),
    "SQ_WAVES": sq.get("SQ_WAVES"),
    "sq_counters_per_launch": sq,
    "FETCH_SIZE_KB_per_launch": fetch,
    "WRITE_SIZE_KB_per_launch": write,
    "hbm_bytes_per_launch_raw": (fetch + write) * 1024 if fetch is not None and write is not None else None,
    "hbm_bytes_per_launch": (2 * fetch + write) * 1024 if fetch is not None and write is not None else None,
    "note": "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 wide-read correction); "
            "writes are the decoded ms_result (24 B/pod)",
}
if sq and avg_ns:
    clk = sq.get("GRBM_GUI_ACTIVE", 0) / 8 / (avg_ns * 1e-9)
    out["effective_clock_ghz"] = clk / 1e9
    out["valu_busy_frac"] = sq.get("SQ_ACTIVE_INST_VALU", 0) * 4 / 1024 / (avg_ns * 1e-9 * clk) if clk else None
    out["valu_wave_instr_per_s"] = sq["SQ_INSTS_VALU"] / (avg_ns * 1e-9)
json.dump(out, open(os.path.join(dst, f"{tag}_pmc_C.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
