#!/bin/bash
# SQ counter passes for the sequential validator (config E, a 20k-pod prefix).
set -o pipefail
OUT=gpurun_out/pmc_val
mkdir -p $OUT
export TMPDIR=/tmp
B="python tools/bench_configs.py --configs E --reps 1 --e-pods 20000"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH -d $OUT/p1 -o run --output-format csv -- $B > $OUT/p1.out 2> $OUT/p1.err || { echo p1 failed; tail $OUT/p1.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD -d $OUT/p2 -o run --output-format csv -- $B > $OUT/p2.out 2> $OUT/p2.err || { echo p2 failed; tail $OUT/p2.err; exit 1; }
python - "$OUT" <<'PY'
import csv, sys, glob
out = sys.argv[1]
for kname in ("k_validate_seq", "k_sweep_full_topk"):
    agg = {}
    for f in glob.glob(out + "/p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if kname not in r["Kernel_Name"]:
                continue
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(kname)
    for k, v in sorted(agg.items()):
        print(f"  {k:24s} {sum(v)/len(v):16.0f} per launch ({len(v)} launches)")
PY
