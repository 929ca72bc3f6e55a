#!/usr/bin/env python3
"""tools/profile_shards.sh output -> profiles/<tag>_pmc_shard<rows>.json, in the
pp_profile_summary format bench.py's load_profile reads (K1 counters per launch of one
strong-scaling shard's sweep: N/G rows x 100k pods)."""
import csv
import glob
import json
import os
import sys

KERNEL = "k_sweep_nunn_pp"
src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for gdir in sorted(glob.glob(os.path.join(src, "G*"))):
    run = json.loads(open(os.path.join(gdir, "run.json")).read().strip().splitlines()[-1])
    avg = calls = None
    for f in glob.glob(os.path.join(gdir, "stats", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Name"]:
                avg, calls = float(r["AverageNs"]), int(r["Calls"])
    agg = {}
    for f in glob.glob(os.path.join(gdir, "sq", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    sq = {k: sum(v) / len(v) for k, v in agg.items()}
    out = {"kernel": KERNEL, "nodes": run["shard_rows"], "pods": run["pods"], "G": run["G"],
           "kernel_avg_ns_rocprof": avg, "calls": calls, "SQ_INSTS_VALU": sq.get("SQ_INSTS_VALU"),
           "SQ_INSTS_SALU": sq.get("SQ_INSTS_SALU"), "SQ_WAVES": sq.get("SQ_WAVES"), "sq_counters_per_launch": sq,
           "hbm_bytes_per_launch": None,
           "note": "one strong-scaling shard's K1 sweep (tools/g8_shard_sweep.py, keys out, 100k pods); no "
                   "FETCH/WRITE passes (the shard's bit planes are 5-45 KB, DRAM traffic is the pods and keys)"}
    path = os.path.join(root, "profiles", f"{tag}_pmc_shard{run['shard_rows']}.json")
    json.dump(out, open(path, "w"), indent=1)
    print(path, out["kernel_avg_ns_rocprof"], out["SQ_INSTS_VALU"])
