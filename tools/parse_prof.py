#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>_*.{csv,json}.

traffic (bytes per launch of the headline kernel) follows MI355X_MICROARCH.md
§HBM: FETCH_SIZE and WRITE_SIZE are KB; on gfx950 FETCH_SIZE reads half the
bytes of wide (16 B/lane) coalesced streams, so the corrected read figure is
2 x FETCH_SIZE; both raw and corrected values are kept.
"""
import csv
import json
import os
import shutil
import sys

src, tag, kernel_key = sys.argv[1], sys.argv[2], (sys.argv[3] if len(sys.argv) > 3 else "k_sweep_nunn_v")
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles")


def per_kernel(path):
    agg = {}
    for r in csv.DictReader(open(path)):
        if kernel_key not in r["Kernel_Name"]:
            continue
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


stats = os.path.join(src, "stats", "run_kernel_stats.csv")
shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
avg_ns, kernel_name = None, None
for r in csv.DictReader(open(stats)):
    if kernel_key in r["Name"]:
        avg_ns = float(r["AverageNs"])
        kernel_name = r["Name"].replace("void msgpu::(anonymous namespace)::", "").split("(")[0]
fetch = per_kernel(os.path.join(src, "fetch", "run_counter_collection.csv")).get("FETCH_SIZE")
write = per_kernel(os.path.join(src, "write", "run_counter_collection.csv")).get("WRITE_SIZE")
sq = {}
p = os.path.join(src, "sq", "run_counter_collection.csv")
if os.path.exists(p):
    sq = per_kernel(p)
out = {
    "kernel": kernel_key,
    "kernel_name": kernel_name,
    "kernel_avg_ns_rocprof": avg_ns,
    "FETCH_SIZE_KB_per_launch": fetch,
    "WRITE_SIZE_KB_per_launch": write,
    "hbm_bytes_per_launch_raw": (fetch + write) * 1024 if fetch is not None and write is not None else None,
    "hbm_bytes_per_launch": (2 * fetch + write) * 1024 if fetch is not None and write is not None else None,
    "note": "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 wide-read correction); "
    "WRITE_SIZE is dominated by memory-side 64-bit atomicMax traffic (8 B per wave-pod result)",
    "sq_counters_per_launch": sq,
}
if sq and avg_ns:
    clk = sq.get("GRBM_GUI_ACTIVE", 0) / 8 / (avg_ns * 1e-9)
    out["effective_clock_ghz"] = clk / 1e9
    # SQ_ACTIVE_INST_VALU counts quad-cycles summed over waves; per-SIMD busy share:
    out["valu_busy_frac"] = sq.get("SQ_ACTIVE_INST_VALU", 0) * 4 / 1024 / (avg_ns * 1e-9 * clk) if clk else None
    out["valu_insts_per_launch"] = sq.get("SQ_INSTS_VALU")
json.dump(out, open(os.path.join(dst, f"{tag}_traffic.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
