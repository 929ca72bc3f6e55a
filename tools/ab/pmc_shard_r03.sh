#!/bin/bash
# SQ counters of K1 pp at a strong-scaling shard (12.5k rows x 100k pods) vs one
# GPU's 100k rows, one --pmc pass each (no tracing domains).
set -o pipefail
mkdir -p gpurun_out/pmc_shard_r03
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
run() {  # tag nodes base waves
  AB_NODES=$2 AB_NODE_BASE=$3 AB_PODS=100000 AB_MODE=sweep AB_ROUNDS=3 AB_VARIANTS="def:MINISCHED_PP_WAVES=$4" \
    timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_shard_r03/$1 -o run --output-format csv -- python tools/ab_pp.py > /dev/null 2> gpurun_out/pmc_shard_r03/$1.err || { echo pmc $1 failed; tail -3 gpurun_out/pmc_shard_r03/$1.err; exit 1; }
}
run s8w4 12500 87500 4 && run s8w2 12500 87500 2 && run s1w16 100000 0 16 && run s4w4 25000 75000 4 || exit 1
python3 - <<'PY'
import csv, glob, collections
for tag in ("s1w16", "s4w4", "s8w4", "s8w2"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/pmc_shard_r03/{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_sweep_nunn_pp" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(tag, {k: round(sum(v) / len(v)) for k, v in sorted(agg.items())})
PY
