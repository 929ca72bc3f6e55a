# kernel stats of config E, in-step merge vs merge launch (rocprofv3 --kernel-trace --stats)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04zk}
for m in instep launch; do
  MINISCHED_SEQ_MERGE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_$m -o run --output-format csv -- python tools/bench_configs.py --configs E --reps 1 > gpurun_out/prof_${T}_$m.log 2>&1 || { tail gpurun_out/prof_${T}_$m.log; exit 1; }
done
for m in instep launch; do echo "== $m"; f=$(find gpurun_out/prof_${T}_$m -name "*kernel_stats.csv" | head -1); python -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'seq_step' in r['Name'] or 'topk_merge' in r['Name'] or 'sweep_tp' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), round(float(r['TotalDurationNs'])/1e6,2), 'min', round(float(r['MinNs'])/1e3,2), 'max', round(float(r['MaxNs'])/1e3,2))
"; done
