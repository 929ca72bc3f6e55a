set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread -k "sequential or resource or config_e or seq" > gpurun_out/e_tests.log 2>&1; rc=$?; tail -3 gpurun_out/e_tests.log; [ $rc -eq 0 ] || exit $rc
for v in "X=0" "MINISCHED_SEQ_PIPE=1"; do
  echo -n "$v: "
  env $v timeout -k 10 120 python -u tools/bench_configs.py --configs E --reps 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['median_s'], d['codes'], d['seq_counters_all_reps'])" || exit 1
done
MINISCHED_LIB=$PWD/mini-kube-scheduler_amd/minisched_amd/libminisched_gpu_vstamps.so timeout -k 10 200 python -u tools/bench_configs.py --configs E --reps 2 > gpurun_out/e_vst.jsonl 2>gpurun_out/e_vst.err || exit 1
grep MS_VSTAMPS gpurun_out/e_vst.err
OUT=gpurun_out/e_prof; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python tools/bench_configs.py --configs E --reps 1 > $OUT/bench.jsonl 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
f=$(find $OUT -name "*kernel_trace.csv" | head -1); s=$(find $OUT -name "*kernel_stats.csv" | head -1)
cp $s $OUT/kernel_stats.csv; rm -f $f
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'])" | head -4
