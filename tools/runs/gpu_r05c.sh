# round 5: config E, batch k+1's merge inside step k (MINISCHED_SEQ_MERGE=instep) on top of the binary64
# sweep — merge-form parity (incl. full E), same-run A/B instep vs launch, kernel trace of the instep form
set -o pipefail
T=${1:-r05c}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "merge_forms or config_e_full or resource_sequential_batch" > gpurun_out/${T}_e_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_e_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in launch instep; do
    ms=$(MINISCHED_SEQ_MERGE=$v timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3), d.get('seq_counters_all_reps',''))") || exit 1
    echo "$v E_ms=$ms" | tee -a gpurun_out/${T}_e_ab.txt
  done
done
MINISCHED_SEQ_MERGE=instep timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_etrace -o run --output-format csv -- python tools/bench_configs.py --configs E --reps 1 > /dev/null 2> gpurun_out/${T}_etrace.err || { echo trace failed; tail gpurun_out/${T}_etrace.err; exit 1; }
python tools/e_batches.py gpurun_out/${T}_etrace/run_kernel_trace.csv > gpurun_out/${T}_e_batches.json || exit 1
python -c "import json;d=json.load(open('gpurun_out/${T}_e_batches.json'));print({k:(v if not isinstance(v,dict) else {kk:vv for kk,vv in v.items() if not isinstance(vv,list)}) for k,v in d.items()})"
