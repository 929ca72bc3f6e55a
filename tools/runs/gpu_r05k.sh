# round 5: config E warm-up batch sizes (MINISCHED_SEQ_WARM=<pods>:<batch>): parity of the full E
# fixture under two settings, then E per setting, twice
set -o pipefail
T=${1:-r05k}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for w in 8192:32 16384:64; do
  MINISCHED_SEQ_WARM=$w timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "config_e_full" > gpurun_out/${T}_tests_$w.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_tests_$w.log; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for w in 0:0 4096:32 8192:32 16384:32 8192:64 16384:64 32768:64; do
    ms=$(MINISCHED_SEQ_WARM=$w timeout -k 10 200 python tools/bench_configs.py --configs E --reps 3 2>/dev/null | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['median_s']*1e3,3), d.get('seq_counters_all_reps',''))") || exit 1
    echo "warm=$w E_ms=$ms" | tee -a gpurun_out/${T}_e_warm.txt
  done
done
