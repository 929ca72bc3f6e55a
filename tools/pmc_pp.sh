#!/bin/bash
# rocprofv3 passes over the fused NU+NN cycle (tools/ab_pp.py, one variant):
# kernel stats, then SQ counter passes, then FETCH_SIZE / WRITE_SIZE, one --pmc run each.
set -o pipefail
TAG=${1:-pp}
OUT=gpurun_out/pmc_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
export AB_ROUNDS=${AB_ROUNDS:-5}
B="python tools/ab_pp.py"
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $B > $OUT/stats.out 2> $OUT/stats.err || { echo stats failed; tail $OUT/stats.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- $B > /dev/null 2> $OUT/sq.err || { echo sq failed; tail $OUT/sq.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_CYCLES_SALU -d $OUT/sq2 -o run --output-format csv -- $B > /dev/null 2> $OUT/sq2.err || { echo sq2 failed; tail $OUT/sq2.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > /dev/null 2> $OUT/fetch.err || { echo fetch failed; tail $OUT/fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > /dev/null 2> $OUT/write.err || { echo write failed; tail $OUT/write.err; exit 1; }
python - "$OUT" <<'PY'
import csv, sys, glob, json
out = sys.argv[1]
agg = {}
for f in glob.glob(out + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_sweep_nunn_pp" not in r["Kernel_Name"]:
            continue
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
res = {k: sum(v) / len(v) for k, v in sorted(agg.items())}
for r in csv.DictReader(open(out + "/stats/run_kernel_stats.csv")):
    if "k_sweep_nunn_pp" in r["Name"]:
        res["avg_ns"] = float(r["AverageNs"])
        res["calls"] = int(r["Calls"])
print(json.dumps(res))
PY
