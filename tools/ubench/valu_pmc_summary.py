#!/usr/bin/env python3
"""Summarise tools/ubench/valu_pmc.sh into profiles/<tag>_valu_issue.json.

Per (instruction, W waves per SIMD), from the --pmc pass (the second, timed
launch of each pair; values are per dispatch):
  clock_GHz        = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md
                     DVFS note; reads high on dispatches shorter than ~0.3 ms)
  cyc_per_inst_simd= (GRBM_GUI_ACTIVE / 8) / (SQ_INSTS_VALU / 1024 SIMDs): chip cycles
                     per wave-instruction on one SIMD (the issue rate the roofline uses)
  active_cyc_per_inst = 4 * SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU (quad-cycles -> cycles,
                     per wave: how long one wave is busy per VALU instruction)
and from the event pass the ns per wave-instruction per SIMD.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NAMES = {"k_add": "v_add_u32", "k_xor": "v_xor_b32", "k_mullo": "v_mul_lo_u32", "k_mul24": "v_mul_u32_u24",
         "k_mulhi": "v_mul_hi_u32", "k_ffbl": "v_ffbl_b32", "k_max": "v_max_u32", "k_bitop3": "v_bitop3_b32",
         "k_mad24": "v_mad_u32_u24", "k_max3": "v_max3_u32", "k_fmaf3": "v_fma_f32", "k_xsdwa": "v_xor_b32_sdwa",
         "k_fma64": "v_fma_f64", "k_add64": "v_add_f64", "k_max64": "v_max_f64", "k_min64": "v_min_f64",
         "k_umax64": "u64max(cmp+2cndmask)", "k_pkfma": "v_pk_fma_f32", "k_pkaddu16": "v_pk_add_u16",
         "k_cvt64": "v_cvt_u32_f64+v_cvt_f64_u32", "k_mad64": "v_mad_u64_u32"}

ev = {}
for line in open(os.path.join(src, "event_rates.txt")):
    m = re.match(r"(\S+)\s+W=(\d+)\s+([\d.]+) ms\s+([\d.]+) ns", line)
    if m:
        ev[(m.group(1), int(m.group(2)))] = {"ms": float(m.group(3)), "ns_per_inst_simd": float(m.group(4))}

cnt = defaultdict(dict)
grid = {}
names = {}
for r in csv.DictReader(open(os.path.join(src, "pmc", "run_counter_collection.csv"))):
    d = int(r["Dispatch_Id"])
    cnt[d][r["Counter_Name"]] = float(r["Counter_Value"])
    grid[d] = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
    names[d] = r["Kernel_Name"]
dur = {}
kt = os.path.join(src, "pmc", "run_kernel_trace.csv")
if os.path.exists(kt):
    for r in csv.DictReader(open(kt)):
        dur[int(r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])

rows = []
seen = defaultdict(int)
for d in sorted(cnt):
    k = re.sub(r"\(.*", "", names[d]).split()[-1]
    op = NAMES.get(k, k)
    threads = grid[d]
    W = max(1, threads // 64 // 1024)  # 256 CUs x 4 SIMDs, one-wave workgroups
    seen[(op, W)] += 1
    c = cnt[d]
    # the program launches each (op, W) 4 times (2 reps x warm + timed): keep the last
    insts = c.get("SQ_INSTS_VALU", 0)
    gui = c.get("GRBM_GUI_ACTIVE", 0)
    ns = dur.get(d)
    row = {"op": op, "W": W, "dispatch": d, "SQ_INSTS_VALU": insts, "SQ_ACTIVE_INST_VALU": c.get("SQ_ACTIVE_INST_VALU"),
           "SQ_BUSY_CYCLES": c.get("SQ_BUSY_CYCLES"), "SQ_WAVES": c.get("SQ_WAVES"),
           "SQ_WAVE_CYCLES": c.get("SQ_WAVE_CYCLES"), "GRBM_GUI_ACTIVE": gui, "duration_ns": ns}
    if insts:
        row["cyc_per_inst_simd"] = (gui / 8) / (insts / 1024) if gui else None
        row["active_cyc_per_inst"] = 4 * c.get("SQ_ACTIVE_INST_VALU", 0) / insts
    if gui and ns:
        row["clock_GHz"] = gui / 8 / ns
    row.update({"event_" + k2: v for k2, v in ev.get((op, W), {}).items()})
    rows.append(row)
last = {}
for r in rows:
    last[(r["op"], r["W"])] = r
out = {"what": "VALU issue cost vs waves per SIMD, tools/ubench/valu_rates.hip + valu_pmc.sh",
       "rows": sorted(last.values(), key=lambda r: (r["op"], r["W"]))}
dst = os.path.join(root, "profiles", f"{tag}_valu_issue.json")
json.dump(out, open(dst, "w"), indent=1)
for r in out["rows"]:
    print(f"{r['op']:28s} W={r['W']:2d} cyc/inst/SIMD={r.get('cyc_per_inst_simd') or 0:6.2f} "
          f"active/inst={r.get('active_cyc_per_inst') or 0:6.2f} clock={r.get('clock_GHz') or 0:5.2f} "
          f"event_ns={r.get('event_ns_per_inst_simd', 0):.3f}")
