#!/bin/bash
# SQ counter passes for one K1 variant (tools/ab_k1.py), one --pmc run per pass.
set -o pipefail
V=${1:-v7}
OUT=gpurun_out/pmc_${V}
mkdir -p $OUT
export TMPDIR=/tmp
B="python tools/ab_k1.py"
export AB_VARIANTS=$V AB_ROUNDS=3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- $B > $OUT/p1.out 2> $OUT/p1.err || { echo p1 failed; tail $OUT/p1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU -d $OUT/p2 -o run --output-format csv -- $B > $OUT/p2.out 2> $OUT/p2.err || { echo p2 failed; tail $OUT/p2.err; exit 1; }
python - "$OUT" <<'PY'
import csv, sys, glob
out = sys.argv[1]
agg = {}
for f in glob.glob(out + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_sweep_nunn" not in r["Kernel_Name"]:
            continue
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:24s} {sum(v)/len(v):16.0f}")
PY
