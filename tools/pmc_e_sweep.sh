#!/bin/bash
# PMC of config E's speculative sweep, standalone (two-stream mode) and inside the fused step (default mode)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_e; rm -rf $OUT; mkdir -p $OUT
B="python tools/bench_configs.py --configs E --reps 1 --e-pods 20000"
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
MINISCHED_SEQ_PIPE=1 timeout -s KILL 240 rocprofv3 --pmc $C -d $OUT/sq -o run --output-format csv -- $B > /dev/null 2> $OUT/sq.err || { echo sq pass failed; tail $OUT/sq.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc $C -d $OUT/sqf -o run --output-format csv -- $B > /dev/null 2> $OUT/sqf.err || { echo sqf pass failed; tail $OUT/sqf.err; exit 1; }
MINISCHED_SEQ_PIPE=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/st -o run --output-format csv -- $B > /dev/null 2> $OUT/st.err || { echo stats failed; tail $OUT/st.err; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/stf -o run --output-format csv -- $B > /dev/null 2> $OUT/stf.err || { echo stats failed; tail $OUT/stf.err; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for tag in ('sq', 'sqf'):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f'gpurun_out/pmc_e/{tag}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            import re; m = re.search(r'(k_\w+)', r['Kernel_Name']); k = m.group(1) if m else r['Kernel_Name'][:30]
            agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, d in agg.items():
        if any(x in k for x in ('topk', 'validate', 'merge', 'seq_step')):
            print(tag, k, {c: round(sum(v)/len(v)) for c, v in d.items()})
for tag in ('st', 'stf'):
    for f in glob.glob(f'gpurun_out/pmc_e/{tag}/**/*kernel_stats.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            print(tag, 'stats', r['Name'][:50], r['Calls'], r['AverageNs'])
PY
