# config E: the split transposed sweep (MINISCHED_SEQ_SPLIT) x the in-step merge (MINISCHED_SEQ_MERGE)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r04zp}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -k "resource or config_e or sequential or commit or chunked" > gpurun_out/${T}_e_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_e_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${T}_e_tests.log | head -20; exit $rc; }
MINISCHED_SEQ_MERGE=instep timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "resource or config_e or sequential" > gpurun_out/${T}_e_tests_instep.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_e_tests_instep.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${T}_e_tests_instep.log | head -20; exit $rc; }
O=gpurun_out/${T}_e_split.txt
for i in 1 2; do
  for v in "1 instep" "1 launch" "0 instep" "0 launch"; do
    set -- $v
    ms=$(MINISCHED_SEQ_SPLIT=$1 MINISCHED_SEQ_MERGE=$2 timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3), d['seq_counters_all_reps'])") || exit 1
    echo "split=$1 merge=$2 E_ms=$ms" >> $O
  done
done
cat $O
for m in instep launch; do
  MINISCHED_SEQ_MERGE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_$m -o run --output-format csv -- python tools/bench_configs.py --configs E --reps 1 > gpurun_out/prof_${T}_$m.log 2>&1 || { tail gpurun_out/prof_${T}_$m.log; exit 1; }
  f=$(find gpurun_out/prof_${T}_$m -name "*kernel_stats.csv" | head -1); python -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'seq_step' in r['Name'] or 'topk_merge' in r['Name']:
        print('$m', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,2))
"
done
