#!/bin/bash
# PMC + trace of the pp sweep at a 12.5k-row shard (N = 8 rank) vs the full 100k rows
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_shard; rm -rf $OUT; mkdir -p $OUT
for cfg in "12500 87500" "100000 0"; do
  set -- $cfg
  tag=r$1
  B="python tools/ab_pp.py"
  export AB_MODE=sweep AB_NODES=$1 AB_NODE_BASE=$2 AB_ROUNDS=4 AB_VARIANTS="pp:X=1"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/$tag/sq -o run --output-format csv -- $B > /dev/null 2> $OUT/$tag.sq.err || { echo sq failed; tail -3 $OUT/$tag.sq.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/$tag/st -o run --output-format csv -- $B > $OUT/$tag.ab.json 2> $OUT/$tag.st.err || { echo st failed; exit 1; }
  python3 - $OUT/$tag <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(d + '/sq/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_sweep_nunn_pp' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
print(d, {k: round(sum(v) / len(v)) for k, v in agg.items()})
for f in glob.glob(d + '/st/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'pp' in r['Name']: print(d, 'stats', r['Name'][:40], r['Calls'], r['AverageNs'])
PY
done
