#!/bin/bash
# PMC of config E's speculative sweep (k_sweep_full_topk, two-stream mode so it runs standalone)
set -o pipefail
export TMPDIR=/tmp MINISCHED_SEQ_PIPE=1
OUT=gpurun_out/pmc_e; rm -rf $OUT; mkdir -p $OUT
B="python tools/bench_configs.py --configs E --reps 1 --e-pods 20000"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- $B > /dev/null 2> $OUT/sq.err || { echo sq pass failed; tail $OUT/sq.err; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/st -o run --output-format csv -- $B > /dev/null 2> $OUT/st.err || { echo stats failed; tail $OUT/st.err; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/pmc_e/sq/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].split('::')[-1]
        agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
for f in glob.glob('gpurun_out/pmc_e/st/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print('stats', r['Name'][:50], r['Calls'], r['AverageNs'])
for k, d in agg.items():
    if 'sweep_full_topk' in k or 'validate' in k or 'merge' in k:
        print(k, {c: sum(v)/len(v) for c, v in d.items()})
PY
